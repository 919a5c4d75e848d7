"""Fault-tolerant DP work loop (parallel/dp_runner.py): three worker processes share a TCPStore;
one crashes after its first batch (no clean-up, like a lost GPU process).  The survivors must see
its heartbeat go stale, take over its unfinished items exactly once, and finish the job."""
from __future__ import annotations

import os
import socket
import time

import torch.distributed as dist
import torch.multiprocessing as mp

from copilot_for_consensus_amd.parallel.dp_runner import ResilientDPRunner


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, items, crash_rank, q):
    store = dist.TCPStore("127.0.0.1", port, world + 1, False, timeout=__import__("datetime").timedelta(seconds=60))
    processed = []

    def process(batch):
        if rank == crash_rank and processed:
            os._exit(17)                      # hard crash mid-job: no ledger update, heartbeat stops
        time.sleep(0.05)
        processed.extend(batch)
        return {i: rank for i in batch}

    runner = ResilientDPRunner(store, rank, world, process, batch_size=3, heartbeat_interval=0.1, timeout=1.0,
                               poll=0.05)
    res = runner.run(items, max_seconds=60)
    q.put((rank, res, runner.stats["reclaimed"]))


def test_survivors_finish_a_dead_ranks_items():
    world, port = 3, _free_port()
    master = dist.TCPStore("127.0.0.1", port, world + 1, True, wait_for_workers=False)
    items = {f"t{i:02d}": float(1 + i % 4) for i in range(30)}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, items, 2, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world - 1):
            r, res, reclaimed = q.get(timeout=120)
            got[r] = (res, reclaimed)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert procs[2].exitcode == 17
    assert sorted(got) == [0, 1]
    done = {}
    for r, (res, _) in got.items():
        done.update(res)
    # rank 2 completed (and recorded) its first batch, then died inside its second: the survivors
    # processed everything else, including the batch that was in flight when it died
    from copilot_for_consensus_amd.parallel.dp_runner import _Prefixed
    from copilot_for_consensus_amd.parallel.resilience import WorkLedger
    ledger = WorkLedger(_Prefixed(master, "job/"))
    by_dead = set(ledger.done(2))
    assert len(by_dead) == 3
    assert set(done) | by_dead == set(items) and not (set(done) & by_dead)
    # rank 2 was reclaimed by exactly one survivor
    assert sum(2 in rec or "2" in rec for _, rec in got.values()) == 1
    del master


def test_single_rank_runs_everything():
    port = _free_port()
    store = dist.TCPStore("127.0.0.1", port, 1, True, wait_for_workers=False)
    seen = []
    runner = ResilientDPRunner(store, 0, 1, lambda b: (seen.extend(b), {i: len(i) for i in b})[1], batch_size=4)
    res = runner.run({f"x{i}": 1.0 for i in range(10)})
    assert sorted(seen) == sorted(res) == sorted(f"x{i}" for i in range(10))
    assert runner.stats["batches"] == 3
