"""Fault-tolerant data-parallel work loop: one worker per GPU (or TP group) pulls thread batches
from a shared ledger, heartbeats while it works, and the survivors take over a dead worker's
unfinished threads ("GPU worker watchdog, requeue of in-flight thread batches if a GPU
worker dies").

Coordination goes only through the job's key-value store (torchrun's TCPStore), never through a
collective, so a rank that dies -- process gone, node lost, or stuck in a kernel (its progress
counter stops) -- cannot hang the others.  The reference gets the same property from competing
consumers on a durable RabbitMQ queue (unacked messages are redelivered); here the queue is the
:class:`~.resilience.WorkLedger`:

1. the first rank to arrive (``store.add`` ticket) writes the initial LPT-balanced assignment;
2. each rank repeatedly takes up to ``batch_size`` of its pending items, processes them, marks
   them done and ticks its heartbeat (re-reading its assignment every time, so items reclaimed
   from it while it was presumed dead are not processed twice by it);
3. an idle rank checks the :class:`~.resilience.Watchdog`; dead ranks' pending items are moved to
   the live ranks, each dead rank reclaimed exactly once (``store.add`` ticket);
4. everyone stops when the union of the done sets covers every item.

Processing is at-least-once (a rank presumed dead that was only slow may finish a batch that was
also reassigned); the pipeline's deterministic ids make the duplicate writes idempotent.

Reference counterpart: unacked messages redelivered to another consumer
(rabbitmq_subscriber.py:537-560).
"""
from __future__ import annotations

import json
import time
from typing import Any, Callable

from .dp import balanced_shard
from .resilience import Heartbeat, Watchdog, WorkLedger, _get


class ResilientDPRunner:
    def __init__(self, store, rank: int, world: int, process_batch: Callable[[list[str]], dict[str, Any]],
                 batch_size: int = 128, heartbeat_interval: float = 2.0, timeout: float = 30.0,
                 stall_timeout: float | None = None, poll: float = 0.2, job: str = "job",
                 heartbeat: Heartbeat | None = None, liveness_prefix: str | None = None):
        """``heartbeat`` / ``liveness_prefix``: a long-lived worker (the DP summarization service,
        parallel/dp_service.py) beats under one namespace across all its jobs, so a worker that died
        between jobs is already known dead when the next job starts (no per-job rendezvous wait on
        it); by default liveness is per job."""
        self.store, self.rank, self.world = store, rank, world
        self.process_batch = process_batch
        self.batch_size = max(1, int(batch_size))
        self.poll = poll
        self.job = job
        self.ledger = WorkLedger(_Prefixed(store, f"{job}/"))
        live_ns = _Prefixed(store, liveness_prefix if liveness_prefix is not None else f"{job}/")
        self.hb = heartbeat or Heartbeat(live_ns, rank, interval=heartbeat_interval)
        self._own_hb = heartbeat is None
        self.watchdog = Watchdog(live_ns, world, timeout=timeout, stall_timeout=stall_timeout)
        self.stats = {"batches": 0, "items": 0, "reclaimed": {}}

    # ---------------------------------------------------------------- setup
    def _init_assignment(self, items: dict[str, float], wait_s: float) -> list[str]:
        all_ids = sorted(items)
        # rendezvous: a rank that has not started yet has no heartbeat and would look dead to an
        # early finisher; wait (bounded) for every rank's first heartbeat before the loop starts
        self.store.add(f"{self.job}/arrived", 1)
        deadline = time.monotonic() + wait_s
        while time.monotonic() < deadline:
            arrived = int(self.store.add(f"{self.job}/arrived", 0))
            if arrived >= self.world or (not self._own_hb and arrived >= self.world - len(self.watchdog.dead_ranks())):
                break
            time.sleep(self.poll)
        if int(self.store.add(f"{self.job}/init_ticket", 1)) == 1:
            ids = list(items)
            bins = balanced_shard([float(items[i]) for i in ids], self.world)
            for r, idx in enumerate(bins):
                self.ledger.assign(r, [ids[j] for j in idx])
            self.store.set(f"{self.job}/all_items", json.dumps(all_ids))
            self.store.set(f"{self.job}/ready", "1")
        else:
            deadline = time.monotonic() + wait_s
            while _get(self.store, f"{self.job}/ready") is None:
                if time.monotonic() > deadline:
                    raise TimeoutError("initial assignment never published")
                time.sleep(self.poll)
        return json.loads(_get(self.store, f"{self.job}/all_items"))

    def _all_done(self, all_ids: list[str]) -> bool:
        done: set[str] = set()
        for r in range(self.world):
            done.update(self.ledger.done(r))
        return done.issuperset(all_ids)

    def _maybe_reclaim(self) -> None:
        dead = self.watchdog.dead_ranks()
        fresh = [r for r in dead if r != self.rank and int(self.store.add(f"{self.job}/reclaimed/{r}", 1)) == 1]
        if not fresh:
            return
        live = [r for r in range(self.world) if r not in dead]
        orphans = [i for r in fresh for i in self.ledger.release(r)]
        for r, idx in zip(live, balanced_shard([1.0] * len(orphans), len(live))):
            got = [orphans[j] for j in idx]
            if got:
                self.ledger.assign(r, got)
        self.stats["reclaimed"].update({r: True for r in fresh})

    # ---------------------------------------------------------------- loop
    def run(self, items: dict[str, float], wait_s: float = 120.0, max_seconds: float | None = None) -> dict[str, Any]:
        """``items``: id -> cost (e.g. prompt tokens).  Returns this rank's results (id -> value)."""
        if self._own_hb:
            self.hb.start()
        results: dict[str, Any] = {}
        t0 = time.monotonic()
        try:
            all_ids = self._init_assignment(items, wait_s)
            while True:
                if max_seconds is not None and time.monotonic() - t0 > max_seconds:
                    raise TimeoutError(f"rank {self.rank}: job not finished in {max_seconds}s")
                batch = self.ledger.pending(self.rank)[: self.batch_size]
                if batch:
                    out = self.process_batch(batch)
                    results.update(out)
                    self.ledger.complete(self.rank, batch)
                    self.hb.tick(len(batch))
                    self.stats["batches"] += 1
                    self.stats["items"] += len(batch)
                    continue
                if self._all_done(all_ids):
                    return results
                self._maybe_reclaim()
                time.sleep(self.poll)
        finally:
            if self._own_hb:
                self.hb.stop()


class _Prefixed:
    """Key namespace over a store (several jobs can share one TCPStore)."""

    def __init__(self, store, prefix: str):
        self.store, self.prefix = store, prefix

    def set(self, k, v):
        return self.store.set(self.prefix + k, v)

    def get(self, k):
        return self.store.get(self.prefix + k)

    def add(self, k, n):
        return self.store.add(self.prefix + k, n)

    def check(self, keys):
        return self.store.check([self.prefix + k for k in keys])
