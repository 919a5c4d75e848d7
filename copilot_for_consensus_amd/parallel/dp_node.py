"""Data-parallel node: every GPU embeds, indexes and summarizes the threads it owns.

The reference scales each processing stage as competing consumers of a durable queue (one queue per
routing key, infra/rabbitmq/definitions.json; replica rules infra/azure/modules/containerapps.bicep:
711-730; the embedding service's batch loop embedding/app/service.py:284-293).  On one MI355X node
the stages are GPU work, and the data they need is per THREAD: a thread's chunk vectors feed the
orchestrator's relevance search, its prompt feeds the summarizer.  So the node shards by thread
ownership (``owner_of(thread_id)``, stable sha1 hash over the DP ranks) and keeps each thread's
data on its owner GPU:

* global rank 0 runs the services (bus, document store, REST) exactly as on one GPU; its
  EmbeddingService, OrchestratorService and ReportingService see a :class:`DPNodeVectorStore` and its
  SummarizationService a :class:`DPNodeSummarizer` -- facades that route each call to the owner rank;
* every DP rank (rank 0 included) runs a :class:`DPNodeWorker`: its own encoder, its own HBM index
  shard (the thread's vectors never leave the GPU that embedded them) and its own LLM engine
  (continuous batching when the summarizer streams);
* the control plane is the job's TCPStore (:class:`StoreRPC`): small JSON requests (chunk texts,
  chunk ids, a query vector) and replies (counts, scores, summaries); no tensor crosses ranks;
* summaries stream: a thread is submitted to its owner's engine and its summary comes back through
  the owner's result stream; a rank whose heartbeat stops has its in-flight threads resubmitted to
  a live rank (at-least-once processing, exactly-once results: rank 0 keeps the first summary of a
  thread and drops late duplicates).

Nothing here is a collective, so a dead rank cannot hang the others.
"""
from __future__ import annotations

import dataclasses
import json
import threading
import time
from concurrent.futures import ThreadPoolExecutor

from ..summarization import Summarizer, Summary, Thread
from ..vectorstore import SearchResult, VectorStore
from .dp import owner_of
from .resilience import Heartbeat, _get

RPC_PREFIX = "dprpc/"
SUM_PREFIX = "dpsum/"


def _wait_key(store, key: str, timeout: float) -> bool:
    """Poll until ``key`` exists (short check requests with a backoff of 1 -> 20 ms).  Never a
    blocking store.wait(): a TCPStore client serialises its requests, so one thread parked in a
    wait would stall every other thread's heartbeat / reply on the same client."""
    deadline = time.monotonic() + timeout
    nap = 0.001
    while True:
        if store.check([key]):
            return True
        if time.monotonic() >= deadline:
            return False
        time.sleep(nap)
        nap = min(0.02, nap * 1.5)


class StoreRPC:
    """Request / reply over a key-value store.  ``call(rank, op, args)`` appends a request to
    ``rank``'s inbox (``<prefix><rank>/req/<seq>``, seq from an atomic counter, so any thread of
    any process may call) and waits for ``<prefix><rank>/res/<seq>``; :meth:`serve` executes a
    rank's requests in order.  Calls to the caller's own rank run in place."""

    def __init__(self, store, rank: int, prefix: str = RPC_PREFIX):
        self.store, self.rank, self.prefix = store, int(rank), prefix
        self.handlers: dict = {}

    def call(self, rank: int, op: str, args=None, timeout: float = 120.0):
        if rank == self.rank and op in self.handlers:
            return self.handlers[op](args)
        seq = int(self.store.add(f"{self.prefix}{rank}/seq", 1))
        self.store.set(f"{self.prefix}{rank}/req/{seq}", json.dumps([op, args]))
        key = f"{self.prefix}{rank}/res/{seq}"
        if not _wait_key(self.store, key, timeout):
            raise TimeoutError(f"DP rank {rank} did not answer {op!r} within {timeout:.0f}s")
        res = json.loads(self.store.get(key))
        if not res.get("ok"):
            raise RuntimeError(f"DP rank {rank} {op!r} failed: {res.get('err')}")
        return res.get("v")

    def serve(self, stop: threading.Event, poll_s: float = 0.5) -> int:
        """Run this rank's requests until ``stop`` is set; returns how many were served."""
        seq, n = 0, 0
        while not stop.is_set():
            key = f"{self.prefix}{self.rank}/req/{seq + 1}"
            try:
                if not _wait_key(self.store, key, poll_s):
                    continue
            except Exception:  # noqa: BLE001 -- the store (rank 0's TCPStore) is gone: the job ended
                return n
            seq += 1
            op, args = json.loads(self.store.get(key))
            try:
                res = {"ok": True, "v": self.handlers[op](args)}
            except Exception as e:  # noqa: BLE001 -- reported to the caller
                res = {"ok": False, "err": f"{type(e).__name__}: {e}"}
            self.store.set(f"{self.prefix}{self.rank}/res/{seq}", json.dumps(res))
            n += 1
        return n


def _thread_to_json(t: Thread) -> dict:
    return dataclasses.asdict(t)


def _summary_to_json(s: Summary) -> dict:
    return dataclasses.asdict(s)


def _summary_from_json(d: dict) -> Summary:
    from ..summarization import Citation
    d = dict(d)
    d["citations"] = [Citation(**c) for c in d.get("citations", [])]
    return Summary(**d)


class DPNodeWorker:
    """One DP rank's model side: encoder, HBM index shard, summarizer, served over :class:`StoreRPC`.
    Rank 0 runs one too (its handlers are called in place)."""

    def __init__(self, store, dp_rank: int, dp_size: int, embedder=None, index=None, summarizer=None,
                 heartbeat_interval: float = 1.0):
        self.store, self.rank, self.world = store, int(dp_rank), int(dp_size)
        self.embedder, self.index, self.summarizer = embedder, index, summarizer
        self.rpc = StoreRPC(store, self.rank)
        self.rpc.handlers.update({
            "embed_index": self._embed_index, "add": self._add, "centroid": self._centroid, "query": self._query,
            "delete": self._delete, "count": self._count, "get": self._get, "info": self._info,
            "sum_submit": self._sum_submit})
        self.hb = Heartbeat(_PrefixedStore(store, SUM_PREFIX), self.rank, interval=heartbeat_interval)
        self._out_seq = 0
        self._out_lock = threading.Lock()
        self._pool: ThreadPoolExecutor | None = None
        self.stats = {"embedded": 0, "summaries": 0, "queries": 0}
        self._stop = threading.Event()
        self._server: threading.Thread | None = None

    # ---------------------------------------------------------------- lifecycle
    def start(self, serve: bool = True) -> "DPNodeWorker":
        self.hb.start()
        start = getattr(self.summarizer, "start_continuous", None)
        if callable(start):
            start()
        else:
            self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix=f"dp{self.rank}-sum")
        if serve:
            self._server = threading.Thread(target=self.rpc.serve, args=(self._stop,), name=f"dp{self.rank}-rpc",
                                            daemon=True)
            self._server.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._server is not None:
            self._server.join(timeout=5)
        stop = getattr(self.summarizer, "stop_continuous", None)
        if callable(stop):
            stop()
        if self._pool is not None:
            self._pool.shutdown(wait=True)
        self.hb.stop()

    def run_until_shutdown(self, poll_s: float = 0.2) -> dict:
        """Worker ranks: serve until rank 0 sets the shutdown key (or its store goes away)."""
        self.start()
        try:
            while _get(self.store, f"{SUM_PREFIX}shutdown") is None:
                if self._server is not None and not self._server.is_alive():
                    break
                time.sleep(poll_s)
        finally:
            self.stop()
        return dict(self.stats)

    # ---------------------------------------------------------------- index / encoder
    def _embed_index(self, args):
        chunks = args["chunks"]
        vecs = self.embedder.embed_tensor([c["text"] for c in chunks])
        self.index.add_embeddings([c["id"] for c in chunks], vecs, [c["meta"] for c in chunks])
        if getattr(vecs, "is_cuda", False):
            import torch
            torch.cuda.current_stream(vecs.device).synchronize()   # rows in HBM before the reply
        self.stats["embedded"] += len(chunks)
        return len(chunks)

    def _add(self, args):
        self.index.add_embeddings(args["ids"], args["vectors"], args["metas"])
        return len(args["ids"])

    def _centroid(self, args):
        return self.index.centroid_scores(args["ids"])

    def _query(self, args):
        self.stats["queries"] += 1
        res = self.index.query(args["vector"], int(args["k"]))
        return [[r.id, float(r.score), r.metadata] for r in res]

    def _delete(self, args):
        n = 0
        for i in args["ids"]:
            try:
                self.index.delete(i)
                n += 1
            except KeyError:
                pass
        return n

    def _count(self, _):
        return int(self.index.count())

    def _get(self, args):
        try:
            r = self.index.get(args["id"])
        except KeyError:
            return None
        return [r.id, float(r.score), list(map(float, r.vector)), r.metadata]

    def _info(self, _):
        e = self.embedder
        return {"model": getattr(e, "model_name", "unknown"), "backend": getattr(e, "backend", "unknown"),
                "dimension": int(getattr(e, "dimension", 0))}

    # ---------------------------------------------------------------- summarization
    def _publish(self, key: str, summary: Summary | None, err: BaseException | None) -> None:
        rec = {"key": key, "rank": self.rank,
               "summary": _summary_to_json(summary) if summary is not None else None,
               "err": None if err is None else f"{type(err).__name__}: {err}"}
        with self._out_lock:
            self._out_seq += 1
            seq = self._out_seq
            self.store.set(f"{SUM_PREFIX}out/{self.rank}/{seq}", json.dumps(rec))
        self.stats["summaries"] += 1
        self.hb.tick()

    def _sum_submit(self, args):
        t = Thread(**args["thread"])
        key = args["key"]
        if self._pool is None:                   # streaming summarizer: the continuous engine
            self.summarizer.submit(t, lambda s, e, key=key: self._publish(key, s, e))
        else:
            def run(t=t, key=key):
                try:
                    self._publish(key, self.summarizer.summarize_batch([t])[0], None)
                except Exception as e:  # noqa: BLE001 -- reported to rank 0 as a failure
                    self._publish(key, None, e)
            self._pool.submit(run)
        return True


class _PrefixedStore:
    def __init__(self, store, prefix):
        self.store, self.prefix = store, prefix

    def set(self, k, v):
        return self.store.set(self.prefix + k, v)

    def get(self, k):
        return self.store.get(self.prefix + k)

    def add(self, k, n):
        return self.store.add(self.prefix + k, n)

    def check(self, keys):
        return self.store.check([self.prefix + k for k in keys])


class _Router:
    """Rank 0's view of the DP ranks: owner of a thread among the live ones."""

    def __init__(self, store, world: int, timeout: float):
        self.store, self.world, self.timeout = store, int(world), float(timeout)
        self.dead: set[int] = set()

    def alive(self, rank: int) -> bool:
        if rank in self.dead:
            return False
        v = _get(self.store, f"{SUM_PREFIX}hb/{rank}")
        if v is None:
            return True                           # not started yet: give it the benefit of the doubt
        if time.time() - json.loads(v)["t"] > self.timeout:
            self.dead.add(rank)
            return False
        return True

    def owner(self, thread_id: str) -> int:
        r = owner_of(thread_id, self.world)
        for i in range(self.world):
            c = (r + i) % self.world
            if self.alive(c):
                return c
        raise RuntimeError("no live DP rank")

    def live(self) -> list[int]:
        return [r for r in range(self.world) if self.alive(r)]


class DPNodeVectorStore(VectorStore):
    """Rank 0's vector store over the DP ranks' HBM shards.  A thread's chunk vectors live on its
    owner (they are embedded there: :meth:`embed_and_store`); a topic query fans out to every
    shard and merges the local top-k lists (exact global top-k)."""
    thread_sharded = True

    def __init__(self, worker: DPNodeWorker, router: _Router):
        self.w, self.router = worker, router
        self.rpc = worker.rpc
        self.dim = int(getattr(worker.index, "dim", 0) or 0)
        self._pool = ThreadPoolExecutor(max_workers=max(2, router.world), thread_name_prefix="dpvs")

    def _fan(self, ranks, op, args_for, required: bool = True):
        """``op`` on every rank in parallel.  ``required`` False (reads: search, count): a rank that
        does not answer within the heartbeat timeout is marked dead and left out (its shard's rows
        are missing from the answer until it is back), instead of failing the request."""
        timeout = 120.0 if required else self.router.timeout
        futs = {r: self._pool.submit(self.rpc.call, r, op, args_for(r), timeout) for r in ranks}
        out = {}
        for r, f in futs.items():
            try:
                out[r] = f.result()
            except (TimeoutError, RuntimeError):
                if required:
                    raise
                self.router.dead.add(r)
        return out

    def embed_and_store(self, chunks: list[dict]) -> dict:
        """Embed ``chunks`` ({id, thread_id, text, meta}) on their threads' owner ranks and store the
        vectors there.  Returns {count, model, backend, dimension}."""
        by: dict[int, list] = {}
        for c in chunks:
            by.setdefault(self.router.owner(c["thread_id"]), []).append(
                {"id": c["id"], "text": c["text"], "meta": c["meta"]})
        done = self._fan(list(by), "embed_index", lambda r: {"chunks": by[r]})
        info = self.w._info(None)
        return {"count": sum(done.values()), **info}

    def add_embeddings(self, ids, vectors, metadatas=None):
        from ..vectorstore import _as_matrix
        vecs = _as_matrix(vectors, self.dim or None).float().cpu().tolist()
        metas = list(metadatas) if metadatas is not None else [{} for _ in ids]
        by: dict[int, tuple[list, list, list]] = {}
        for i, v, m in zip(ids, vecs, metas):
            r = self.router.owner(m.get("thread_id") or i)
            a = by.setdefault(r, ([], [], []))
            a[0].append(i), a[1].append(v), a[2].append(m)
        self._fan(list(by), "add", lambda r: {"ids": by[r][0], "vectors": by[r][1], "metas": by[r][2]})

    def centroid_scores(self, ids, thread_id: str | None = None) -> dict[str, float]:
        if thread_id is None:
            out = {}
            for part in self._fan(self.router.live(), "centroid", lambda r: {"ids": list(ids)}, False).values():
                out.update(part)
            return out
        return self.rpc.call(self.router.owner(thread_id), "centroid", {"ids": list(ids)})

    def query(self, query_vector, top_k: int = 10) -> list[SearchResult]:
        import numpy as np
        vec = np.asarray(query_vector, dtype=np.float32).reshape(-1).tolist()
        parts = self._fan(self.router.live(), "query", lambda r: {"vector": vec, "k": int(top_k)}, False)
        hits = [h for p in parts.values() for h in p]
        hits.sort(key=lambda h: (-h[1], h[0]))
        return [SearchResult(i, s, [], m) for i, s, m in hits[:top_k]]

    def delete(self, id: str) -> None:
        n = sum(self._fan(self.router.live(), "delete", lambda r: {"ids": [id]}).values())
        if n == 0:
            raise KeyError(id)

    def clear(self) -> None:
        raise NotImplementedError("clear() of a DP-sharded index: delete by id")

    def count(self) -> int:
        return sum(self._fan(self.router.live(), "count", lambda r: None, False).values())

    def get(self, id: str) -> SearchResult:
        for v in self._fan(self.router.live(), "get", lambda r: {"id": id}, False).values():
            if v is not None:
                return SearchResult(v[0], v[1], v[2], v[3])
        raise KeyError(id)


class DPNodeSummarizer(Summarizer):
    """Rank 0's streaming summarizer over the DP ranks: ``submit(thread, done)`` sends the thread to
    its owner's engine; a collector thread per rank reads that rank's result stream and calls
    ``done`` once per thread; a rank found dead (stale heartbeat) has its in-flight threads
    resubmitted to the live ranks."""

    def __init__(self, worker: DPNodeWorker, router: _Router, poll_s: float = 0.2):
        local = worker.summarizer
        self.backend, self.model = getattr(local, "backend", "hip"), getattr(local, "model", "unknown")
        self.w, self.router, self.poll_s = worker, router, poll_s
        self.rpc = worker.rpc
        self._lock = threading.Lock()
        self._inflight: dict[str, tuple[Thread, object, int]] = {}   # key -> (thread, done, rank)
        self._delivered: set[str] = set()
        self._seq = 0
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self.stats = {"submitted": 0, "completed": 0, "resubmitted": 0, "duplicates": 0,
                      "per_rank": [0] * router.world}

    # the SummarizationService's streaming protocol (start_async -> start_continuous, submit, stop)
    def start_continuous(self, **_) -> None:
        if self._threads:
            return
        for r in range(self.router.world):
            t = threading.Thread(target=self._collect, args=(r,), name=f"dpsum-collect-{r}", daemon=True)
            t.start()
            self._threads.append(t)
        t = threading.Thread(target=self._watch, name="dpsum-watch", daemon=True)
        t.start()
        self._threads.append(t)

    def stop_continuous(self) -> None:
        self._stop.set()
        for t in self._threads:
            t.join(timeout=5)
        self._threads = []
        with self._lock:
            left, self._inflight = list(self._inflight.values()), {}
        err = RuntimeError("DP summarizer stopped before the thread finished")
        for _, done, _ in left:
            _deliver(done, None, err)

    def submit(self, thread: Thread, done) -> None:
        with self._lock:
            self._seq += 1
            key = f"{thread.thread_id}#{self._seq}"
            self._inflight[key] = (thread, done, -1)
        self.stats["submitted"] += 1
        self._send(key)

    def _send(self, key: str) -> None:
        with self._lock:
            item = self._inflight.get(key)
            if item is None:
                return
            thread, done, _ = item
            rank = self.router.owner(thread.thread_id)
            self._inflight[key] = (thread, done, rank)
        try:
            self.rpc.call(rank, "sum_submit", {"thread": _thread_to_json(thread), "key": key}, timeout=30.0)
        except Exception:  # noqa: BLE001 -- the rank is gone: the watchdog resubmits
            self.router.dead.add(rank)

    def _collect(self, rank: int) -> None:
        seq = 0
        while not self._stop.is_set():
            key = f"{SUM_PREFIX}out/{rank}/{seq + 1}"
            if not _wait_key(self.w.store, key, self.poll_s):
                continue
            seq += 1
            rec = json.loads(self.w.store.get(key))
            with self._lock:
                item = self._inflight.pop(rec["key"], None)
                tid = rec["key"].rsplit("#", 1)[0]
                dup = item is None or tid in self._delivered
                if not dup:
                    self._delivered.add(tid)
            if dup:
                self.stats["duplicates"] += 1
                continue
            self.stats["completed"] += 1
            self.stats["per_rank"][rank] += 1
            s = _summary_from_json(rec["summary"]) if rec["summary"] is not None else None
            _deliver(item[1], s, None if s is not None else RuntimeError(rec["err"] or "summarization failed"))

    def _watch(self) -> None:
        while not self._stop.wait(self.poll_s):
            with self._lock:
                lost = [k for k, (_, _, r) in self._inflight.items() if r >= 0 and not self.router.alive(r)]
            for k in lost:
                self.stats["resubmitted"] += 1
                self._send(k)

    # batch API (DP-aware callers without streaming): submit all, wait for all
    def summarize_batch(self, threads: list[Thread]) -> list[Summary]:
        box: dict[int, tuple] = {}
        ev = threading.Event()

        def cb(i):
            def done(s, e):
                box[i] = (s, e)
                if len(box) == len(threads):
                    ev.set()
            return done
        started = bool(self._threads)
        if not started:
            self.start_continuous()
        try:
            for i, t in enumerate(threads):
                self.submit(t, cb(i))
            if threads:
                ev.wait()
        finally:
            if not started:
                self.stop_continuous()
        out = []
        for i in range(len(threads)):
            s, e = box[i]
            if e is not None:
                raise e
            out.append(s)
        return out

    def summarize(self, thread: Thread) -> Summary:
        return self.summarize_batch([thread])[0]


def _deliver(done, s, e) -> None:
    try:
        done(s, e)
    except Exception as ex:  # noqa: BLE001 -- a callback failing must not stop the collector
        import sys
        print(f"[dp-summarizer] done callback failed: {type(ex).__name__}: {ex}", file=sys.stderr, flush=True)


def shutdown_workers(store) -> None:
    store.set(f"{SUM_PREFIX}shutdown", "1")


def build_rank0(store, dp_size: int, worker: DPNodeWorker, heartbeat_timeout: float = 10.0):
    """Rank 0's facades over the DP ranks: (vector store, summarizer)."""
    router = _Router(store, dp_size, heartbeat_timeout)
    return DPNodeVectorStore(worker, router), DPNodeSummarizer(worker, router)
