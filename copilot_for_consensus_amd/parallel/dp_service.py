"""Multi-GPU summarization inside the services: data parallel over TP groups, one process per GPU.

The reference scales its summarization stage horizontally: several container replicas consume the
same durable RabbitMQ queue (competing consumers, infra/rabbitmq/definitions.json; replica counts
in infra/azure/modules/containerapps.bicep:711-730).  On one MI355X node the equivalent is one
process per GPU launched by torchrun, grouped as

    ranks [0 .. tp-1] | [tp .. 2tp-1] | ...      CFC_TP consecutive ranks = one TP group (one model)
    TP-group leaders = the DP workers            the DP degree = WORLD_SIZE / CFC_TP

* the service (``services.main node`` / ``summarization``) runs on global rank 0; its
  SummarizationService calls :class:`DPSummarizer`, which turns each batch of threads into a job
  in the job's TCPStore: a :class:`~.dp_runner.ResilientDPRunner` ledger with LPT-balanced
  assignment over the DP workers, heartbeats, and takeover of a dead worker's unfinished threads
  (at-least-once processing, exactly-once results: every thread's summary is written under its
  job key once, by whichever worker finished it first);
* every other TP-group leader runs :func:`dp_worker_loop`: waits for jobs, summarizes its share
  on its own GPU(s), writes the summaries back;
* TP followers run :func:`tp_follow`: they receive each generate call's token ids from their
  leader (gloo twin group) and step the same engine in lockstep (their weight shards, the
  one-shot IPC all-reduces).

Summaries travel as JSON through the store (small: a few KB per thread).
"""
from __future__ import annotations

import dataclasses
import json
import threading
import time

from ..summarization import Citation, Summarizer, Summary, Thread
from .dp_runner import ResilientDPRunner, _Prefixed
from .resilience import Heartbeat, _get

LIVE_PREFIX = "dpsvc/"


def _summary_to_json(s: Summary) -> str:
    return json.dumps(dataclasses.asdict(s))


def _summary_from_json(v) -> Summary:
    d = json.loads(v)
    d["citations"] = [Citation(**c) for c in d.get("citations", [])]
    return Summary(**d)


class _JobRunner:
    """Shared by the leader and the workers: run job k's share on the local summarizer."""

    def __init__(self, store, rank: int, world: int, local: Summarizer, prefix: str, heartbeat: Heartbeat,
                 batch_size: int, timeout: float, poll: float):
        self.store, self.rank, self.world, self.local = store, rank, world, local
        self.prefix, self.hb, self.batch_size, self.timeout, self.poll = prefix, heartbeat, batch_size, timeout, poll

    def run(self, k: int, wait_s: float = 10.0) -> None:
        threads = [Thread(**t) for t in json.loads(self.store.get(f"{self.prefix}job/{k}"))]
        items = {str(i): float(len(t.prompt) + sum(len(m) for m in t.messages)) for i, t in enumerate(threads)}

        def process(ids: list[str]) -> dict:
            outs = self.local.summarize_batch([threads[int(i)] for i in ids])
            for i, s in zip(ids, outs):
                key = f"{self.prefix}res/{k}/{i}"
                # first writer wins: a reclaimed thread finished twice keeps one summary
                if int(self.store.add(f"{key}/ticket", 1)) == 1:
                    self.store.set(key, _summary_to_json(s))
            self.hb.tick(len(ids))
            return {i: True for i in ids}

        ResilientDPRunner(self.store, self.rank, self.world, process, batch_size=self.batch_size,
                          timeout=self.timeout, poll=self.poll, job=f"{self.prefix}run{k}", heartbeat=self.hb,
                          liveness_prefix=LIVE_PREFIX + self.prefix).run(items, wait_s=wait_s)


class DPSummarizer(Summarizer):
    """Rank 0's summarizer: each summarize_batch is sharded over the DP workers (see module doc)."""

    def __init__(self, store, world: int, local: Summarizer, prefix: str = "sum/", batch_size: int = 64,
                 heartbeat_interval: float = 1.0, timeout: float = 10.0, poll: float = 0.05):
        self.backend, self.model = local.backend, local.model
        self.store, self.world, self.local, self.prefix = store, int(world), local, prefix
        self.hb = Heartbeat(_Prefixed(store, LIVE_PREFIX + prefix), 0, interval=heartbeat_interval).start()
        self._runner = _JobRunner(store, 0, self.world, local, prefix, self.hb, batch_size, timeout, poll)
        self._lock = threading.Lock()
        self.stats = {"jobs": 0, "threads": 0}

    def summarize(self, thread: Thread) -> Summary:
        return self.summarize_batch([thread])[0]

    def summarize_batch(self, threads: list[Thread]) -> list[Summary]:
        if not threads:
            return []
        with self._lock:          # one job at a time (the service's batcher is one thread anyway)
            k = int(self.store.add(f"{self.prefix}seq", 1))
            self.store.set(f"{self.prefix}job/{k}", json.dumps([dataclasses.asdict(t) for t in threads]))
            self.store.set(f"{self.prefix}latest", str(k))
            self._runner.run(k)
            self.store.set(f"{self.prefix}done/{k}", "1")     # late workers skip it
            out = [_summary_from_json(self.store.get(f"{self.prefix}res/{k}/{i}")) for i in range(len(threads))]
            self.stats["jobs"] += 1
            self.stats["threads"] += len(threads)
            return out

    def wait_workers(self, timeout: float = 120.0) -> int:
        """Block until every DP worker has started beating (bounded); returns how many did."""
        keys = [f"{LIVE_PREFIX}{self.prefix}hb/{r}" for r in range(self.world)]
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            up = sum(_get(self.store, k) is not None for k in keys)
            if up == self.world:
                return up
            time.sleep(0.05)
        return sum(_get(self.store, k) is not None for k in keys)

    def close(self) -> None:
        """Tell the workers to exit."""
        self.store.set(f"{self.prefix}shutdown", "1")
        self.hb.stop()


def dp_worker_loop(store, rank: int, world: int, local: Summarizer, prefix: str = "sum/", batch_size: int = 64,
                   heartbeat_interval: float = 1.0, timeout: float = 10.0, poll: float = 0.05,
                   stop: threading.Event | None = None, max_idle_s: float | None = None) -> int:
    """A DP worker (TP-group leader of group ``rank``): run every job rank 0 posts until shutdown.
    Returns the number of jobs taken part in."""
    hb = Heartbeat(_Prefixed(store, LIVE_PREFIX + prefix), rank, interval=heartbeat_interval).start()
    runner = _JobRunner(store, rank, world, local, prefix, hb, batch_size, timeout, poll)
    seen, jobs, idle_since = 0, 0, time.monotonic()
    try:
        while not (stop is not None and stop.is_set()):
            if _get(store, f"{prefix}shutdown") is not None:
                break
            latest = _get(store, f"{prefix}latest")
            latest = int(latest) if latest is not None else 0
            if latest > seen:
                for k in range(seen + 1, latest + 1):
                    if _get(store, f"{prefix}done/{k}") is None:      # finished before we got here
                        runner.run(k)
                        jobs += 1
                seen = latest
                idle_since = time.monotonic()
                continue
            if max_idle_s is not None and time.monotonic() - idle_since > max_idle_s:
                break
            time.sleep(poll)
    finally:
        hb.stop()
    return jobs


# ------------------------------------------------------------------ tensor parallel followers
class TPBroadcast:
    """Leader side: hands every engine call's control message to the TP followers
    (HipLLMSummarizer.tp_hook: ("gen", ids) for a static batch, the continuous engine's
    ("cstart" | "cstep" | "creset" | "cstop", ...) messages)."""

    def __init__(self, groups):
        self.g = groups

    def __call__(self, msg) -> None:
        import torch.distributed as dist
        dist.broadcast_object_list([msg], src=self.g.tp_src, group=self.g.tp_cpu_group)

    def stop(self) -> None:
        self(None)


def tp_follow(summarizer, groups) -> int:
    """TP follower: replay the leader's engine calls (HipLLMSummarizer.tp_serve) until it sends None.
    Returns the number of messages served."""
    import torch.distributed as dist
    n = 0
    while True:
        box = [None]
        dist.broadcast_object_list(box, src=groups.tp_src, group=groups.tp_cpu_group)
        if box[0] is None:
            return n
        summarizer.tp_serve(box[0])
        n += 1
