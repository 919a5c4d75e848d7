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


def test_broker_asan_ubsan(tmp_path):
    """The message broker under ASan+UBSan: routing, prefetch, nack -> DLQ, a client dying with
    unacked deliveries, purge / delete, journal replay after a restart; clean exit, no leaks."""
    import json
    import signal
    from pathlib import Path

    from copilot_for_consensus_amd._build import build_broker
    from copilot_for_consensus_amd.bus.cfcbroker import Connection, spawn_broker

    exe = build_broker(verbose=False, out=Path(tmp_path) / "cfc-broker-asan",
                       extra_flags=["-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                                    "-fno-sanitize-recover=undefined"])
    os.environ["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:exitcode=23"
    data = tmp_path / "data"
    for rnd in range(2):
        proc, port = spawn_broker(port=0, data_dir=data, binary=exe, max_redeliveries=1)
        try:
            c = Connection("127.0.0.1", port)
            c.declare("q1")
            c.bind("q1", "ex", "a.#")
            c.declare("tmp", durable=False)
            c.bind("tmp", "ex", "*.b")
            for i in range(50):
                c.publish("ex", "a.b", json.dumps({"i": i, "r": rnd}).encode())
            d = Connection("127.0.0.1", port)
            d.consume("q1", prefetch=4)
            for _ in range(4):
                m = d.next_delivery(2)
                d.nack(m.tag, requeue=True)
            d.close()                                 # dies with redeliveries in flight
            e = Connection("127.0.0.1", port)
            e.consume("q1", prefetch=0)
            n = 0
            while (m := e.next_delivery(0.5)) is not None:
                e.ack(m.tag)
                n += 1
            assert c.purge("tmp") == 50
            c.delete("tmp")
            c.stats()
            e.close()
            c.close()
        finally:
            proc.send_signal(signal.SIGTERM)
            rc = proc.wait(20)
        assert rc == 0, f"broker exited {rc} under the sanitizers (round {rnd})"
