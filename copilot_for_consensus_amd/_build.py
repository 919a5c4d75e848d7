"""In-tree native build for copilot_for_consensus_amd.

Two shared libraries are produced next to the package sources (git-ignored, but they travel to
the GPU box with the gpurun snapshot):

* ``_lib/libcfc_kernels.so`` -- every ``csrc/kernels/*.hip`` compiled by ``hipcc`` for gfx950
  (CDNA4 / MI355X only; no other offload arch, no CUDA path).
* ``_lib/libcfc_runtime.so`` -- the host-side C++ runtime (``csrc/runtime/*.cpp``): BPE and
  WordPiece tokenizers, paged-KV block allocator, mbox splitter.
* ``_lib/cfc-broker`` -- the native message broker executable (``csrc/broker/cfc_broker.cpp``),
  the RabbitMQ replacement for multi-process deployments (``bus/cfcbroker.py``).

The build is incremental (object files are rebuilt only when their source or a header changed)
and compiles translation units in parallel.
"""
from __future__ import annotations

import concurrent.futures as _fut
import hashlib
import os
import shutil
import subprocess
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
CSRC = REPO_DIR / "csrc"
LIB_DIR = PKG_DIR / "_lib"
OBJ_DIR = REPO_DIR / "build" / "obj"

OFFLOAD_ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", shutil.which("g++") or "c++")

HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={OFFLOAD_ARCH}", "-ffp-contract=fast",
             "-Wno-unused-result"]
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function"]
# per-source additions.  attention.hip: no NaN ever enters the softmax (masked scores are -inf,
# which stays honoured), and without NaN semantics fmaxf needs no canonicalising v_max_f32 in front
# of every MFMA output it reads -- 33 fewer VALU instructions per prefill KV tile
FILE_FLAGS = {"attention.hip": ["-fno-honor-nans"]}

KERNELS_LIB = LIB_DIR / "libcfc_kernels.so"
RUNTIME_LIB = LIB_DIR / "libcfc_runtime.so"
BROKER_BIN = LIB_DIR / "cfc-broker"


def _digest(paths: list[Path], extra: list[str]) -> str:
    h = hashlib.sha256()
    for p in sorted(paths):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    h.update(" ".join(extra).encode())
    return h.hexdigest()[:16]


def _compile(cmd: list[str], src: Path, obj: Path, stamp: Path, digest: str) -> str:
    if obj.exists() and stamp.exists() and stamp.read_text() == digest:
        return f"up-to-date {src.name}"
    obj.parent.mkdir(parents=True, exist_ok=True)
    res = subprocess.run(cmd + ["-c", str(src), "-o", str(obj)], capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{res.stderr[-8000:]}")
    stamp.write_text(digest)
    return f"built {src.name}"


def _build_lib(sources: list[Path], headers: list[Path], compiler: str, flags: list[str], out: Path,
               link_flags: list[str], jobs: int, verbose: bool) -> Path:
    out.parent.mkdir(parents=True, exist_ok=True)
    objs = []
    tasks = []
    with _fut.ThreadPoolExecutor(max_workers=max(1, jobs)) as pool:
        for src in sources:
            obj = OBJ_DIR / (src.stem + (".hip.o" if src.suffix == ".hip" else ".o"))
            stamp = obj.with_suffix(obj.suffix + ".stamp")
            fflags = [*flags, *FILE_FLAGS.get(src.name, [])]
            digest = _digest([src, *headers], fflags)
            cmd = [compiler, *fflags, f"-I{src.parent}"]
            tasks.append(pool.submit(_compile, cmd, src, obj, stamp, digest))
            objs.append(obj)
        for t in tasks:
            msg = t.result()
            if verbose:
                print(f"[cfc-build] {msg}")
    newest = max(o.stat().st_mtime for o in objs)
    if not out.exists() or out.stat().st_mtime < newest:
        res = subprocess.run([compiler, "-shared", "-o", str(out), *map(str, objs), *link_flags],
                             capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed: {out}\n{res.stderr[-8000:]}")
        if verbose:
            print(f"[cfc-build] linked {out}")
    return out


def build_kernels(jobs: int | None = None, verbose: bool = True) -> Path:
    srcs = sorted((CSRC / "kernels").glob("*.hip"))
    hdrs = sorted((CSRC / "kernels").glob("*.h"))
    return _build_lib(srcs, hdrs, HIPCC, HIP_FLAGS, KERNELS_LIB, [f"--offload-arch={OFFLOAD_ARCH}"],
                      jobs or min(8, os.cpu_count() or 4), verbose)


def build_runtime(jobs: int | None = None, verbose: bool = True) -> Path:
    srcs = sorted((CSRC / "runtime").glob("*.cpp"))
    hdrs = sorted((CSRC / "runtime").glob("*.h"))
    return _build_lib(srcs, hdrs, CXX, CXX_FLAGS, RUNTIME_LIB, ["-lpthread"],
                      jobs or min(8, os.cpu_count() or 4), verbose)


def build_broker(verbose: bool = True, out: Path | None = None, extra_flags: list[str] | None = None) -> Path:
    """Single-TU executable; rebuilt when the source or the flags change."""
    src = CSRC / "broker" / "cfc_broker.cpp"
    out = out or BROKER_BIN
    flags = ["-O2", "-std=c++17", "-Wall", "-Wextra", *(extra_flags or [])]
    stamp = out.with_name(out.name + ".stamp")
    digest = _digest([src], flags)
    if out.exists() and stamp.exists() and stamp.read_text() == digest:
        return out
    out.parent.mkdir(parents=True, exist_ok=True)
    res = subprocess.run([CXX, *flags, str(src), "-o", str(out)], capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"broker build failed\n{res.stderr[-8000:]}")
    stamp.write_text(digest)
    if verbose:
        print(f"[cfc-build] linked {out}")
    return out


def build_all(verbose: bool = True) -> tuple[Path, Path, Path]:
    return build_kernels(verbose=verbose), build_runtime(verbose=verbose), build_broker(verbose=verbose)


if __name__ == "__main__":
    build_all()
