"""The driver's bench.py contract, rehearsed on the CPU: one rank and two ranks under
``torch.distributed.run`` (gloo, 127.0.0.1), tiny random-init models.  Checks the single JSON line
rank 0 prints (keys, whole-job aggregate value, n_gpus, weak-scaling batch, parallelism tag) so the
multi-GPU path the driver runs at N = 2..8 is exercised by construction here."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--model", "tiny", "--encoder", "tiny", "--threads-per-gpu", "2", "--max-new", "3", "--steps", "2",
        "--warmup", "1", "--index-prefill", "0", "--prefill-tokens", "4096", "--service-latency-threads", "3"]
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd):
    env = {**os.environ, "CFC_DIST_BACKEND": "gloo", "OMP_NUM_THREADS": "2", "MASTER_ADDR": "127.0.0.1"}
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout           # exactly one JSON line, from rank 0 only
    return json.loads(lines[0])


def _check(d, n, latency=True):
    assert KEYS <= set(d)
    assert d["n_gpus"] == n and d["steps"] == 2 and d["warmup"] == 1
    assert d["scaling"] == "weak" and d["higher_is_better"] is True and d["dtype"] == "bf16"
    assert d["config"]["global_batch"] == 2 * n and d["config"]["parallelism"] == f"dp{n}"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # value is the whole-job aggregate: threads of every rank over the max elapsed time
    assert d["value"] == pytest.approx(2 * n * 2 / (d["ms_per_step"] * 2 / 1000), rel=0.02)
    if not latency:
        return
    # the latency half: Poisson arrivals on the continuous engine after the timed window
    lm = d["latency_mode"]
    assert lm["threads"] == 2 * 2 * n and lm["arrival_rate_per_gpu"] == 8.0
    assert 0 < lm["p50_s"] <= lm["p95_s"]
    # and the light-load point (one step's threads per rank, far apart)
    ll = d["latency_mode_light"]
    assert ll["threads"] == 2 * n and ll["arrival_rate_per_gpu"] == 0.5
    assert 0 < ll["p50_s"] <= ll["p95_s"]
    # and through the services: archive submit -> report stored, one-thread archives at 0.5 / s
    sl = d["latency_service_light"]
    assert sl["threads"] == 3 * n and sl["arrival_rate_per_gpu"] == 0.5 and sl["path"].startswith("services")
    assert 0 < sl["p50_s"] <= sl["p95_s"]
    # the reporting topic search (embed + kNN top-150 + enrichment) against the P95 0.5 s SLO
    se = d["search_latency"]
    assert se["queries"] == 64 * n and se["top_k"] == 150 and se["slo_p95_ms"] == 500
    assert 0 < se["p50_ms"] <= se["p95_ms"] <= se["max_ms"] and se["reports_per_query"] > 0
    assert "centroid-select" in d["config"]["pipeline"] and "knn" not in d["config"]["pipeline"]


def test_bench_single_process_contract():
    _check(_run([sys.executable, "bench.py", "--gpus", "1", *ARGS]), 1)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_dp_ranks_under_torchrun(n):
    """The driver's N = 2, 4, 8 runs, one rank per (here virtual) GPU: the DP data plane (index
    sharded by thread owner, all_to_all inserts / query merges) at every world size it will see."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", str(n), *ARGS]
    d = _run(cmd)
    _check(d, n)
    assert d["config"]["index"].startswith(f"sharded over {n} GPUs")    # the DP data plane ran


def test_bench_tp2_two_ranks_reports_both_halves():
    """--tp 2 over 2 ranks (one DP replica of a TP=2 engine): the throughput half and both latency
    points, the TP follower replaying the continuous engine's steps."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2", "--tp", "2", *ARGS]
    d = _run(cmd)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp1xtp2" and d["config"]["global_batch"] == 2
    assert d["value"] == pytest.approx(2 * 2 / (d["ms_per_step"] * 2 / 1000), rel=0.02)
    lm, ll = d["latency_mode"], d["latency_mode_light"]
    assert lm["threads"] == 2 * 2 and ll["threads"] == 2 and "TP=2" in lm["engine"]
    assert 0 < lm["p50_s"] <= lm["p95_s"] and 0 < ll["p50_s"] <= ll["p95_s"]
    assert lm["prep_charged"] == "the thread's whole batch preparation"


def test_bench_node_pipeline_contract():
    """--pipeline node: the same JSON contract measured through the real services (Node on the
    in-proc bus, continuous summarization engine), every thread of every step reported."""
    d = _run([sys.executable, "bench.py", "--gpus", "1", "--pipeline", "node", *ARGS])
    _check(d, 1, latency=False)
    assert d["config"]["pipeline"].startswith("node:")


def test_bench_node_pipeline_dp_topology_two_ranks():
    """--pipeline node under torchrun: services.main's DP topology (rank-0 services + a DPNodeWorker on
    each rank); every thread of every step reported, both ranks embedded and summarized threads."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2", "--pipeline", "node", *ARGS]
    d = _run(cmd)
    _check(d, 2, latency=False)
    assert d["config"]["topology"].startswith("services.main node")
    pr = d["per_rank"]
    assert [p["rank"] for p in pr] == [0, 1]
    assert all(p["embedded"] > 0 and p["summaries"] > 0 for p in pr), pr
    # (warmup + 2 steps) x 2 threads x 2 ranks, + the 3 one-thread archives of the light-load probe
    assert sum(p["summaries"] for p in pr) == 2 * 2 * 3 + 3
    sl = d["latency_service_light"]
    assert sl["threads"] == 3 and 0 < sl["p50_s"] <= sl["p95_s"] and d["dp_wait"] == "block"
