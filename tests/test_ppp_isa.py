"""ISA guard for the persistent prefill GEMM (csrc/kernels/pgemm.hip, pgemm_ppp_kernel).

Its interior epilogue leaves exactly S stores in flight and the next tile's first two waits keep
them outstanding with vmcnt(8 + S).  That is exact only while the compiler emits exactly S store
instructions there (fewer would make those waits retire less than the next segment reads) and no
scratch traffic (spills are vector-memory operations counted by the same vmcnt).  This test reads
the built gfx950 code object (no GPU needed) and pins, per instantiation, the store instructions
of the interior block plus the 32 of the register-direct edge path, and zero scratch operations.
"""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

from copilot_for_consensus_amd._build import KERNELS_LIB

OBJDUMP = Path("/opt/rocm/lib/llvm/bin/llvm-objdump")

# (EPI, STG) -> store instructions of the whole kernel: interior S + edge path (pg_epilogue)
EXPECTED = {
    ("0", "1"): {"global_store_dwordx4": 16, "global_store_dwordx2": 32, "global_store_dword": 0},   # bf16, staged
    ("0", "0"): {"global_store_dwordx4": 0, "global_store_dwordx2": 64, "global_store_dword": 0},    # bf16, direct
    ("3", "1"): {"global_store_dwordx4": 8, "global_store_dwordx2": 0, "global_store_dword": 32},    # SwiGLU, staged
    ("3", "0"): {"global_store_dwordx4": 0, "global_store_dwordx2": 0, "global_store_dword": 64},    # SwiGLU, direct
}


def _kernel_bodies(tmp_path):
    lib = tmp_path / KERNELS_LIB.name
    shutil.copy(KERNELS_LIB, lib)
    # extracts every offload bundle of the library next to the copy (inside tmp_path)
    subprocess.run([str(OBJDUMP), "--offloading", str(lib)], capture_output=True, check=True, cwd=tmp_path)
    bodies = {}
    for obj in sorted(tmp_path.glob(lib.name + ".*gfx950")):
        dis = subprocess.run([str(OBJDUMP), "-d", str(obj)], capture_output=True, text=True, check=True).stdout
        parts = re.split(r"\n[0-9a-f]+ <([^>]+)>:\n", dis)
        for name, body in zip(parts[1::2], parts[2::2]):
            m = re.search(r"pgemm_ppp_kernelILi(\d)ELb(\d)E", name)
            if m:
                bodies[(m.group(1), m.group(2))] = body
    return bodies


@pytest.mark.skipif(not OBJDUMP.exists() or not KERNELS_LIB.exists(), reason="llvm-objdump or the built library missing")
def test_persistent_gemm_epilogue_store_counts_match_its_vmcnt_waits(tmp_path):
    bodies = _kernel_bodies(tmp_path)
    assert set(bodies) == set(EXPECTED), sorted(bodies)
    for key, want in EXPECTED.items():
        body = bodies[key]
        got = {op: len(re.findall(r"\s" + op + r"\s", body)) for op in want}
        assert got == want, (key, got)
        assert not re.search(r"\sscratch_(load|store)", body), key
        assert not re.search(r"\sbuffer_store", body), key
