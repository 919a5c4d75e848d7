"""Host sanitizer runs of the C++ runtime: ASan+UBSan over tokenizers, mbox splitter
and block pool; TSan over concurrent block-pool use.  Compiled with the system g++ for the host
(the runtime is host-only code; GPU sanitizers are not available on the GPU pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = [os.path.join(ROOT, "csrc", "runtime", f) for f in ("blockpool.cpp", "tokenizer.cpp")]
TEST = os.path.join(ROOT, "csrc", "runtime", "tests", "selftest.cpp")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")


def _build_run(tmp_path, flags, arg=None, env=None):
    exe = str(tmp_path / "selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, *SRCS, TEST, "-o", exe, "-lpthread"]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if b.returncode != 0 and "sanitize" in b.stderr and "unrecognized" in b.stderr:
        pytest.skip("sanitizer runtime not available")
    assert b.returncode == 0, b.stderr[-3000:]
    r = subprocess.run([exe] + ([arg] if arg else []), capture_output=True, text=True, timeout=300,
                       env={**os.environ, **(env or {})})
    assert r.returncode == 0 and "selftest ok" in r.stdout, (r.stdout + r.stderr)[-4000:]


def test_runtime_asan_ubsan(tmp_path):
    _build_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
               env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0"})


def test_runtime_tsan(tmp_path):
    _build_run(tmp_path, ["-fsanitize=thread"], arg="threads", env={"TSAN_OPTIONS": "halt_on_error=1"})
