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
* the control plane is the job's TCPStore (:class:`StoreRPC`): small JSON requests (chunk ids, a
  query vector) and replies (counts, scores, summaries); every request, reply and result key is
  deleted once it is consumed, so rank 0's store stays bounded however long the node runs.  Each
  rank serves two inboxes on two threads: ``bulk`` (encoder forwards, bulk inserts) and ``ctl``
  (summary submits, relevance / topic reads), so a read never queues behind an embedding batch;
* the data plane for chunk texts is a socket: rank 0 serves its document store
  (storage/server.py) and an owner rank reads the texts of the chunk ids it was sent;
* summaries stream: a thread is submitted to its owner's engine and its summary comes back through
  the owner's result stream; a rank whose heartbeat stops has its in-flight threads resubmitted to
  a live rank (at-least-once processing, exactly-once results: a result is matched to its request
  key and a late duplicate of a resubmitted request is dropped).  A rank is dead when its heartbeat
  is stale, or when it is busy and its progress counter (engine decode steps, finished work) has
  not moved for the stall timeout -- a GPU hung inside a kernel, whose heartbeat thread still beats
  (the reference's nack + requeue of a failed consumer, rabbitmq_subscriber.py:537-560, and its
  stuck-document retry job, scripts/retry_stuck_documents.py:314-357).  A slow reply or a handler
  error does not mark a rank dead, and liveness is re-checked on every routing decision, so a rank
  whose heartbeat or progress resumes gets its threads back;
* waits are blocking server-side TCPStore waits on a per-thread client (woken when the key is set),
  not polls; every cursor (request served, result published) is a counter in the store, so a
  restarted rank process continues the numbering its predecessor left.

Nothing here is a collective, so a dead rank cannot hang the others.
"""
from __future__ import annotations

import dataclasses
import json
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor

from ..summarization import Summarizer, Summary, Thread
from ..vectorstore import SearchResult, VectorStore
from .dp import owner_of
from .resilience import Heartbeat, _get

RPC_PREFIX = "dprpc/"
SUM_PREFIX = "dpsum/"
DATA_KEY = "dpnode/docstore"          # [host, port] of the chunk-text server rank 0 publishes
# ops that run an encoder forward or move many rows: served from their own inbox
BULK_OPS = frozenset({"embed_index", "add"})


class RemoteError(RuntimeError):
    """A DP rank's handler raised: the rank is alive, the request failed."""


_waiters = threading.local()
WAIT_SLICE_S = 30.0    # an idle blocked waiter re-checks its deadline / stop flag this often
HOLE_POLL_S = 0.5      # ... and this often while a later number exists (a hole may need skipping)
WAKE_OP = "__wake__"   # a request / result that only wakes its waiter (stop)


def _waiter(store):
    """This thread's own TCPStore client of ``store``'s server, for blocking waits.  A TCPStore
    client serialises its requests, so a thread parked in ``wait`` on the shared client would stall
    every other thread's heartbeat / reply; a client per waiting thread does not, and the server
    wakes it the moment the key is set (no polling).  None for other stores (HashStore, FileStore,
    prefix wrappers): those are polled."""
    try:
        from torch.distributed import TCPStore
    except ImportError:  # pragma: no cover
        return None
    if not isinstance(store, TCPStore) or os.environ.get("CFC_DP_WAIT", "block") == "poll":
        return None                   # CFC_DP_WAIT=poll: round 5's check polling (A/B)
    cache = getattr(_waiters, "clients", None)
    if cache is None:
        cache = _waiters.clients = {}
    addr = (store.host, store.port)
    c = cache.get(addr)
    if c is None:
        import datetime
        c = cache[addr] = TCPStore(store.host, store.port, is_master=False, wait_for_workers=False,
                                   timeout=datetime.timedelta(seconds=60))
    return c


def _wait_key(store, key: str, timeout: float, stop: threading.Event | None = None) -> bool:
    """Wait until ``key`` exists, at most ``timeout`` s (or until ``stop`` is set).  TCPStore: a
    blocking server-side wait on this thread's own client (woken when the key is set), in slices of
    WAIT_SLICE_S so the deadline and ``stop`` are honoured; other stores: check polls with a 1 -> 20
    ms backoff."""
    deadline = time.monotonic() + timeout
    w = _waiter(store)
    if w is not None:
        import datetime
        while True:
            if stop is not None and stop.is_set():
                return False
            left = deadline - time.monotonic()
            if left <= 0:
                return bool(w.check([key]))
            try:
                w.wait([key], datetime.timedelta(seconds=min(left, WAIT_SLICE_S)))
                return True
            except Exception:  # noqa: BLE001 -- DistStoreError on timeout; a lost server ends below
                if not _alive(w):
                    raise
    nap = 0.001
    while True:
        if store.check([key]):
            return True
        if time.monotonic() >= deadline or (stop is not None and stop.is_set()):
            return False
        time.sleep(nap)
        nap = min(0.02, nap * 1.5)


def _alive(store) -> bool:
    try:
        store.check(["__ping__"])
        return True
    except Exception:  # noqa: BLE001
        return False


def _delete(store, key: str) -> bool:
    try:
        return bool(store.delete_key(key))
    except Exception:  # noqa: BLE001 -- stores without delete / the store is gone
        return False


class StoreRPC:
    """Request / reply over a key-value store.  ``call(rank, op, args)`` appends a request to one of
    ``rank``'s inboxes (``<prefix><rank>/<lane>/req/<seq>``, seq from an atomic counter, so any
    thread of any process may call) and waits for ``.../res/<seq>``; :meth:`serve` executes one
    inbox's requests in order.  Both keys are deleted once read (the server deletes the request,
    the caller the reply; a reply that arrives after its caller timed out is deleted by that
    caller's next call).  Calls to the caller's own rank run in place."""

    LANES = ("ctl", "bulk")

    def __init__(self, store, rank: int, prefix: str = RPC_PREFIX, skip_grace_s: float = 10.0):
        self.store, self.rank, self.prefix = store, int(rank), prefix
        self.skip_grace_s = float(skip_grace_s)
        self.handlers: dict = {}
        self.skipped = 0
        self._abandoned: list[str] = []
        self._alock = threading.Lock()

    @staticmethod
    def lane(op: str) -> str:
        return "bulk" if op in BULK_OPS else "ctl"

    def _base(self, rank: int, lane: str) -> str:
        return f"{self.prefix}{rank}/{lane}/"

    def call(self, rank: int, op: str, args=None, timeout: float = 120.0):
        if rank == self.rank and op in self.handlers:
            return self.handlers[op](args)
        self._sweep()
        base = self._base(rank, self.lane(op))
        seq = int(self.store.add(base + "seq", 1))
        self.store.set(f"{base}req/{seq}", json.dumps([op, args]))
        key = f"{base}res/{seq}"
        if not _wait_key(self.store, key, timeout):
            with self._alock:
                self._abandoned.append(key)
            raise TimeoutError(f"DP rank {rank} did not answer {op!r} within {timeout:.0f}s")
        res = json.loads(self.store.get(key))
        _delete(self.store, key)
        if not res.get("ok"):
            raise RemoteError(f"DP rank {rank} {op!r} failed: {res.get('err')}")
        return res.get("v")

    def _sweep(self) -> None:
        """Delete the replies of timed-out calls that have arrived since (bounded list)."""
        with self._alock:
            if not self._abandoned:
                return
            self._abandoned = [k for k in self._abandoned if not _delete(self.store, k)][-1024:]

    def wake(self, lane: str) -> None:
        """Unblock this rank's ``lane`` server (after its stop flag was set): a no-op request through
        the normal numbering, so no sequence number is left unwritten."""
        base = self._base(self.rank, lane)
        seq = int(self.store.add(base + "seq", 1))
        self.store.set(f"{base}req/{seq}", json.dumps([WAKE_OP, None]))

    def serve(self, stop: threading.Event, poll_s: float = WAIT_SLICE_S, lane: str = "ctl") -> int:
        """Run this rank's ``lane`` inbox until ``stop`` is set; returns how many were served.  A
        sequence number whose request never appears (its caller died between reserving it and
        writing it) is skipped once a later request exists and ``skip_grace_s`` has passed.  The
        cursor lives in the store (``<lane>/served``, advanced once per consumed or skipped number),
        so a rank process restarted against the same store resumes where its predecessor stopped
        instead of waiting for request numbers that were consumed long ago."""
        base = self._base(self.rank, lane)
        n, missing_since = 0, None
        try:
            seq = int(self.store.add(base + "served", 0))
        except Exception:  # noqa: BLE001 -- the store is gone
            return 0
        while not stop.is_set():
            key = f"{base}req/{seq + 1}"
            try:
                # a later request already exists while this one is missing: its caller may have
                # died after reserving the number -- wait briefly and skip it after the grace
                hole = int(self.store.add(base + "seq", 0)) > seq + 1
                if not _wait_key(self.store, key, min(poll_s, HOLE_POLL_S) if hole else poll_s, stop):
                    if hole:
                        now = time.monotonic()
                        missing_since = missing_since or now
                        if now - missing_since >= self.skip_grace_s:
                            seq, missing_since = seq + 1, None
                            self.store.add(base + "served", 1)
                            self.skipped += 1
                    continue
                raw = self.store.get(key)
            except Exception:  # noqa: BLE001 -- the store (rank 0's TCPStore) is gone: the job ended
                return n
            seq, missing_since = seq + 1, None
            _delete(self.store, key)
            try:
                self.store.add(base + "served", 1)
            except Exception:  # noqa: BLE001
                return n
            op, args = json.loads(raw)
            if op == WAKE_OP:
                continue                      # stop(): the loop re-checks its flag
            try:
                res = {"ok": True, "v": self.handlers[op](args)}
            except Exception as e:  # noqa: BLE001 -- reported to the caller
                res = {"ok": False, "err": f"{type(e).__name__}: {e}"}
            try:
                self.store.set(f"{base}res/{seq}", json.dumps(res))
            except Exception:  # noqa: BLE001
                return n
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


def _store_texts(store):
    """ids -> texts of those chunks, read from a document store (one $in query)."""
    def texts(ids: list[str]) -> list[str]:
        docs = store.query_documents("chunks", {"_id": {"$in": list(ids)}}, limit=max(1, len(ids)))
        by = {d["_id"]: d.get("text", "") for d in docs}
        missing = [i for i in ids if i not in by]
        if missing:
            raise KeyError(f"{len(missing)} chunk(s) not in the document store, e.g. {missing[0]!r}")
        return [by[i] for i in ids]
    return texts


class DPNodeWorker:
    """One DP rank's model side: encoder, HBM index shard, summarizer, served over :class:`StoreRPC`.
    Rank 0 runs one too (its handlers are called in place)."""

    def __init__(self, store, dp_rank: int, dp_size: int, embedder=None, index=None, summarizer=None,
                 heartbeat_interval: float = 1.0, continuous: dict | None = None):
        self.store, self.rank, self.world = store, int(dp_rank), int(dp_size)
        # the local continuous engine's admission (min_admit, max_wait_s): the summarization
        # service's settings, which rank 0's service cannot hand to the other ranks' engines itself
        self.continuous = dict(continuous or {})
        self.embedder, self.index, self.summarizer = embedder, index, summarizer
        self.rpc = StoreRPC(store, self.rank)
        handlers = {
            "embed_index": self._embed_index, "add": self._add, "centroid": self._centroid, "query": self._query,
            "delete": self._delete, "clear": self._clear, "count": self._count, "get": self._get,
            "info": self._info}
        self.rpc.handlers.update({op: self._counted(fn) for op, fn in handlers.items()})
        self.rpc.handlers["sum_submit"] = self._sum_submit
        # liveness beyond "the process is up": the heartbeat carries how much work this rank holds
        # (busy: accepted summaries not yet published + handlers running) and a progress counter
        # that moves with the engine's decode bursts, finished summaries and finished handlers.
        # The heartbeat thread keeps beating while a GPU call hangs, so rank 0's router declares a
        # rank dead when it is busy and its progress has not moved for the stall timeout
        # (_Router.alive), and the summarizer's watchdog resubmits its threads elsewhere.
        self._busy = 0
        self._done_ops = 0
        self._busy_lock = threading.Lock()
        self.hb = Heartbeat(_PrefixedStore(store, SUM_PREFIX), self.rank, interval=heartbeat_interval,
                            progress_fn=self.progress, busy_fn=lambda: self._busy)
        self._out_lock = threading.Lock()
        # index reads (ctl inbox) and writes (bulk inbox) run on different threads
        self._index_lock = threading.RLock()
        # ids -> chunk texts: rank 0's document store (attached) or its socket server (lazy)
        self.text_source = None
        self._text_lock = threading.Lock()
        self._pool: ThreadPoolExecutor | None = None
        self.stats = {"embedded": 0, "summaries": 0, "queries": 0}
        self._stop = threading.Event()
        self._servers: list[threading.Thread] = []

    # ---------------------------------------------------------------- liveness
    def progress(self) -> int:
        """Forward progress of this rank: finished handlers + published summaries + the local
        summarizer's own counter (decode bursts of its engine), never blocking on the GPU."""
        fn = getattr(self.summarizer, "progress", None)
        try:
            eng = int(fn()) if callable(fn) else 0
        except Exception:  # noqa: BLE001 -- a counter read must never stop the heartbeat
            eng = 0
        return self._done_ops + self.stats["summaries"] + eng

    def _busy_add(self, n: int) -> None:
        with self._busy_lock:
            self._busy += n

    def _counted(self, fn):
        def run(args):
            self._busy_add(1)
            try:
                return fn(args)
            finally:
                self._done_ops += 1
                self._busy_add(-1)
        return run

    # ---------------------------------------------------------------- lifecycle
    def start(self, serve: bool = True) -> "DPNodeWorker":
        self.hb.start()
        start = getattr(self.summarizer, "start_continuous", None)
        if callable(start):
            start(**self.continuous)
        else:
            self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix=f"dp{self.rank}-sum")
        if serve:
            for lane in StoreRPC.LANES:
                t = threading.Thread(target=self.rpc.serve, args=(self._stop,), kwargs={"lane": lane},
                                     name=f"dp{self.rank}-rpc-{lane}", daemon=True)
                t.start()
                self._servers.append(t)
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._servers:
            for lane in StoreRPC.LANES:       # unblock the lanes' waits
                try:
                    self.rpc.wake(lane)
                except Exception:  # noqa: BLE001 -- the store is gone: the waits end on their own
                    pass
        for t in self._servers:
            t.join(timeout=5)
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
                if self._servers and not all(t.is_alive() for t in self._servers):
                    break
                time.sleep(poll_s)
        finally:
            self.stop()
        return dict(self.stats)

    # ---------------------------------------------------------------- index / encoder
    def _texts(self, ids: list[str]) -> list[str]:
        with self._text_lock:
            if self.text_source is None:
                addr = _get(self.store, DATA_KEY)
                if addr is None:
                    raise RuntimeError("no chunk-text server published (DPNodeVectorStore.attach_document_store)")
                from ..storage.server import RemoteDocumentStore
                host, port = json.loads(addr)
                rs = RemoteDocumentStore(host, int(port))
                rs.connect()
                self.text_source = _store_texts(rs)
        return self.text_source(ids)

    def _embed_index(self, args):
        ids = [c["id"] for c in args["chunks"]] if "chunks" in args else list(args["ids"])
        texts = [c["text"] for c in args["chunks"]] if "chunks" in args else self._texts(ids)
        metas = [c["meta"] for c in args["chunks"]] if "chunks" in args else list(args["metas"])
        vecs = self.embedder.embed_tensor(texts)           # the encoder forward runs outside the index lock
        with self._index_lock:
            self.index.add_embeddings(ids, vecs, metas)
        if getattr(vecs, "is_cuda", False):
            import torch
            torch.cuda.current_stream(vecs.device).synchronize()   # rows in HBM before the reply
        self.stats["embedded"] += len(ids)
        return len(ids)

    def _add(self, args):
        with self._index_lock:
            self.index.add_embeddings(args["ids"], args["vectors"], args["metas"])
        return len(args["ids"])

    def _centroid(self, args):
        with self._index_lock:
            return self.index.centroid_scores(args["ids"])

    def _query(self, args):
        self.stats["queries"] += 1
        with self._index_lock:
            res = self.index.query(args["vector"], int(args["k"]))
        return [[r.id, float(r.score), r.metadata] for r in res]

    def _delete(self, args):
        n = 0
        with self._index_lock:
            for i in args["ids"]:
                try:
                    self.index.delete(i)
                    n += 1
                except KeyError:
                    pass
        return n

    def _clear(self, _):
        with self._index_lock:
            n = int(self.index.count())
            self.index.clear()
        return n

    def _count(self, _):
        with self._index_lock:
            return int(self.index.count())

    def _get(self, args):
        with self._index_lock:
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
            # result numbers come from a counter in the store, not from this process: a rank
            # restarted against the same store continues the numbering rank 0's collector follows
            seq = int(self.store.add(f"{SUM_PREFIX}outseq/{self.rank}", 1))
            self.store.set(f"{SUM_PREFIX}out/{self.rank}/{seq}", json.dumps(rec))
        self.stats["summaries"] += 1
        self._busy_add(-1)

    def _sum_submit(self, args):
        t = Thread(**args["thread"])
        key = args["key"]
        self._busy_add(1)
        try:
            if self._pool is None:                   # streaming summarizer: the continuous engine
                self.summarizer.submit(t, lambda s, e, key=key: self._publish(key, s, e))
            else:
                def run(t=t, key=key):
                    try:
                        s = self.summarizer.summarize_batch([t])[0]
                    except Exception as e:  # noqa: BLE001 -- reported to rank 0 as a failure
                        self._publish(key, None, e)
                    else:
                        self._publish(key, s, None)
                self._pool.submit(run)
        except BaseException:
            self._busy_add(-1)
            raise
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
    """Rank 0's view of the DP ranks: owner of a thread among the live ones.  A rank is live while
    its heartbeat is fresh AND it is not stalled -- busy (work accepted, not finished) with a
    progress counter that has not moved for ``stall_timeout`` (a hung GPU: the process and its
    heartbeat thread are up, nothing finishes; the semantics of resilience.Watchdog's stall check).
    Re-read on every decision (cached ``cache_s``), never latched, so a rank that only answered
    slowly, whose handler failed, or whose progress resumes keeps or gets back its threads."""

    def __init__(self, store, world: int, timeout: float, cache_s: float = 0.25,
                 startup_grace_s: float | None = None, stall_timeout: float | None = None):
        self.store, self.world, self.timeout, self.cache_s = store, int(world), float(timeout), float(cache_s)
        # a rank with no heartbeat yet is still loading its models: live for this long after the
        # router starts, dead after it (its threads go to the next live rank instead of waiting on
        # a rank that never came up)
        self.startup_grace_s = float(startup_grace_s if startup_grace_s is not None
                                     else os.environ.get("CFC_DP_STARTUP_GRACE_S", "600"))
        # longer than any legitimate gap between two progress ticks of a busy rank (one decode
        # burst is ~0.2 s, a 16k-token prefill chunk ~0.5 s, a first graph capture a few s)
        st = stall_timeout if stall_timeout is not None else float(os.environ.get("CFC_DP_STALL_TIMEOUT", "120"))
        self.stall_timeout = float(st) if st and float(st) > 0 else None
        self._t0 = time.monotonic()
        self._seen: dict[int, tuple[float, bool]] = {}
        self._prog: dict[int, tuple[object, float]] = {}   # rank -> (progress value, first seen at)
        self.stalls: dict[int, int] = {}                    # rank -> times declared stalled

    def alive(self, rank: int) -> bool:
        now = time.monotonic()
        c = self._seen.get(rank)
        if c is not None and now - c[0] < self.cache_s:
            return c[1]
        v = _get(self.store, f"{SUM_PREFIX}hb/{rank}")
        if v is None:                 # not started yet: live during the start-up grace only
            ok = now - self._t0 <= self.startup_grace_s
        else:
            hb = json.loads(v)
            ok = time.time() - hb["t"] <= self.timeout
            if ok and self.stall_timeout is not None:
                prog, prev = hb.get("progress"), self._prog.get(rank)
                if not hb.get("busy") or prev is None or prev[0] != prog:
                    self._prog[rank] = (prog, now)      # idle, or moving: the stall clock restarts
                elif now - prev[1] > self.stall_timeout:
                    ok = False
                    if c is None or c[1]:
                        self.stalls[rank] = self.stalls.get(rank, 0) + 1
        self._seen[rank] = (now, ok)
        return ok

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
        self._pool = ThreadPoolExecutor(max_workers=max(2, 2 * router.world), thread_name_prefix="dpvs")
        self._data_server = None
        self.stats = {"partial_reads": 0}

    def attach_document_store(self, store) -> None:
        """Chunk texts go to the owner ranks over a socket from rank 0's document store: embed
        requests then carry chunk ids only.  An in-process store is served by a
        :class:`~..storage.server.DocumentStoreServer` on an ephemeral port; a networked one
        (``cfcstore``) is published as is."""
        from ..storage.server import DocumentStoreServer, RemoteDocumentStore
        if isinstance(store, RemoteDocumentStore):
            host, port = store.host, store.port
        else:
            host = os.environ.get("CFC_DP_DATA_HOST", "127.0.0.1")
            self._data_server = DocumentStoreServer(store, host=host, port=0, read_only=True).start()
            port = self._data_server.port
        self.w.text_source = _store_texts(store)
        self.w.store.set(DATA_KEY, json.dumps([host, int(port)]))

    def close(self) -> None:
        if self._data_server is not None:
            self._data_server.server.shutdown()
            self._data_server.server.server_close()
            self._data_server = None
        self._pool.shutdown(wait=False)

    def _fan(self, ranks, op, args_for, required: bool = True):
        """``op`` on every rank in parallel.  A handler error is raised to the caller.  A rank that
        does not answer in time fails the call when ``required``; for reads (search, count) it is
        left out of THIS answer only (its rows are missing from it) -- whether it is dead is the
        heartbeat's call, not a timeout's."""
        timeout = 120.0 if required else self.router.timeout
        futs = {r: self._pool.submit(self.rpc.call, r, op, args_for(r), timeout) for r in ranks}
        out = {}
        for r, f in futs.items():
            try:
                out[r] = f.result()
            except TimeoutError:
                if required:
                    raise
                self.stats["partial_reads"] += 1
        return out

    def embed_and_store(self, chunks: list[dict]) -> dict:
        """Embed ``chunks`` ({id, thread_id, text, meta}) on their threads' owner ranks and store the
        vectors there.  With a document store attached only the ids (and metadata) travel through
        the control plane.  Returns {count, model, backend, dimension}."""
        by: dict[int, list] = {}
        for c in chunks:
            by.setdefault(self.router.owner(c["thread_id"]), []).append(c)
        if self.w.text_source is not None:
            def args_for(r):
                return {"ids": [c["id"] for c in by[r]], "metas": [c["meta"] for c in by[r]]}
        else:
            def args_for(r):
                return {"chunks": [{"id": c["id"], "text": c["text"], "meta": c["meta"]} for c in by[r]]}
        done = self._fan(list(by), "embed_index", args_for)
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
        """Empty every live shard (copilot_vectorstore interface.py:99-102)."""
        self._fan(self.router.live(), "clear", lambda r: None)

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
    ``done`` once per request; a request whose rank's heartbeat went stale, or whose send failed,
    is (re)sent to a live rank by the watchdog.  Results are matched by request key only: a
    thread may be submitted any number of times (different context, or twice in one batch) and
    every submit gets its own result; a late duplicate of a RESENT request is dropped."""

    SEND_RETRY_S = 1.0

    def __init__(self, worker: DPNodeWorker, router: _Router, poll_s: float = 0.2,
                 batch_timeout_s: float | None = None):
        local = worker.summarizer
        self.backend, self.model = getattr(local, "backend", "hip"), getattr(local, "model", "unknown")
        self.w, self.router, self.poll_s = worker, router, poll_s
        self.batch_timeout_s = float(batch_timeout_s if batch_timeout_s is not None
                                     else os.environ.get("CFC_DP_SUMMARY_TIMEOUT", "1800"))
        self.rpc = worker.rpc
        self._lock = threading.Lock()
        # key -> (thread, done, rank, retry_at): rank -1 = being sent, -2 = send failed (retry at retry_at)
        self._inflight: dict[str, tuple[Thread, object, int, float]] = {}
        self._seq = 0
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self._sender = ThreadPoolExecutor(max_workers=2, thread_name_prefix="dpsum-send")
        # each rank's result cursor lives on the instance, not in the collector thread: results are
        # deleted once read, so a collector restarted by stop_continuous / start_continuous (the
        # batch API does both per call) must continue where the previous one stopped
        self._col_seq = [0] * router.world
        self.skip_grace_s = 10.0
        self.stats = {"submitted": 0, "completed": 0, "resubmitted": 0, "duplicates": 0, "send_failures": 0,
                      "per_rank": [0] * router.world}

    # the SummarizationService's streaming protocol (start_async -> start_continuous, submit, stop)
    def start_continuous(self, **_) -> None:
        if self._threads:
            return
        self._stop = threading.Event()        # a fresh flag: a collector that outlived its stop stays stopped
        for r in range(self.router.world):
            t = threading.Thread(target=self._collect, args=(r,), name=f"dpsum-collect-{r}", daemon=True)
            t.start()
            self._threads.append(t)
        t = threading.Thread(target=self._watch, name="dpsum-watch", daemon=True)
        t.start()
        self._threads.append(t)

    def stop_continuous(self) -> None:
        self._stop.set()
        if self._threads:
            # unblock each collector's wait with a no-op result through the rank's own numbering
            for r in range(self.router.world):
                try:
                    seq = int(self.w.store.add(f"{SUM_PREFIX}outseq/{r}", 1))
                    self.w.store.set(f"{SUM_PREFIX}out/{r}/{seq}", json.dumps({"key": None, "rank": r}))
                except Exception:  # noqa: BLE001 -- the store is gone
                    break
        for t in self._threads:
            t.join(timeout=5)
        self._threads = []
        with self._lock:
            left, self._inflight = list(self._inflight.values()), {}
        err = RuntimeError("DP summarizer stopped before the thread finished")
        for _, done, _, _ in left:
            _deliver(done, None, err)

    def submit(self, thread: Thread, done) -> str:
        with self._lock:
            self._seq += 1
            key = f"{thread.thread_id}#{self._seq}"
            self._inflight[key] = (thread, done, -1, 0.0)
        self.stats["submitted"] += 1
        self._send(key)
        return key

    def _send(self, key: str) -> None:
        with self._lock:
            item = self._inflight.get(key)
            if item is None:
                return
            thread, done, _, _ = item
            rank = self.router.owner(thread.thread_id)
            self._inflight[key] = (thread, done, rank, 0.0)
        try:
            self.rpc.call(rank, "sum_submit", {"thread": _thread_to_json(thread), "key": key}, timeout=30.0)
        except Exception:  # noqa: BLE001 -- not delivered (or not confirmed): the watchdog resends
            self.stats["send_failures"] += 1
            with self._lock:
                if key in self._inflight:
                    self._inflight[key] = (thread, done, -2, time.monotonic() + self.SEND_RETRY_S)

    def _collect(self, rank: int) -> None:
        store = self.w.store
        stop = self._stop
        missing_since = None
        while not stop.is_set():
            seq = self._col_seq[rank]
            key = f"{SUM_PREFIX}out/{rank}/{seq + 1}"
            try:
                # a later result already exists while this one is missing: the rank may have died
                # between reserving the number and writing it -- skip it once the grace has passed
                hole = int(store.add(f"{SUM_PREFIX}outseq/{rank}", 0)) > seq + 1
                if not _wait_key(store, key, HOLE_POLL_S if hole else WAIT_SLICE_S, stop):
                    if hole and not stop.is_set():
                        now = time.monotonic()
                        missing_since = missing_since or now
                        if now - missing_since >= self.skip_grace_s:
                            self._col_seq[rank], missing_since = seq + 1, None
                    continue
                rec = json.loads(store.get(key))
            except Exception:  # noqa: BLE001 -- the store is gone: the node is shutting down
                return
            if stop.is_set():
                return                        # leave the result to the next collector of this rank
            self._col_seq[rank], missing_since = seq + 1, None
            _delete(store, key)
            if rec.get("key") is None:           # a stop_continuous wake-up
                continue
            with self._lock:
                item = self._inflight.pop(rec["key"], None)
            if item is None:                  # the other copy of a resent request finished first
                self.stats["duplicates"] += 1
                continue
            self.stats["completed"] += 1
            self.stats["per_rank"][rank] += 1
            s = _summary_from_json(rec["summary"]) if rec["summary"] is not None else None
            _deliver(item[1], s, None if s is not None else RuntimeError(rec["err"] or "summarization failed"))

    def _watch(self) -> None:
        stop = self._stop
        while not stop.wait(self.poll_s):
            now = time.monotonic()
            with self._lock:
                lost = [k for k, (_, _, r, at) in self._inflight.items()
                        if (r >= 0 and not self.router.alive(r)) or (r == -2 and now >= at)]
                for k in lost:
                    t, d, _, _ = self._inflight[k]
                    self._inflight[k] = (t, d, -1, 0.0)      # being resent: not picked again meanwhile
            for k in lost:
                self.stats["resubmitted"] += 1
                self._sender.submit(self._send, k)

    # batch API (DP-aware callers without streaming): submit all, wait for all (bounded)
    def summarize_batch(self, threads: list[Thread]) -> list[Summary]:
        box: dict[int, tuple] = {}
        ev = threading.Event()
        blk = threading.Lock()

        def cb(i):
            def done(s, e):
                with blk:
                    box[i] = (s, e)
                    if len(box) == len(threads):
                        ev.set()
            return done
        started = bool(self._threads)
        if not started:
            self.start_continuous()
        keys = []
        try:
            for i, t in enumerate(threads):
                keys.append(self.submit(t, cb(i)))
            if threads and not ev.wait(self.batch_timeout_s):
                with self._lock:
                    for k in keys:
                        self._inflight.pop(k, None)
                raise TimeoutError(f"DP summarizer: {len(threads) - len(box)} of {len(threads)} threads not "
                                   f"summarized within {self.batch_timeout_s:.0f}s")
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


def build_rank0(store, dp_size: int, worker: DPNodeWorker, heartbeat_timeout: float = 10.0,
                stall_timeout: float | None = None):
    """Rank 0's facades over the DP ranks: (vector store, summarizer).  ``stall_timeout``: a busy
    rank whose progress froze this long is treated as dead ($CFC_DP_STALL_TIMEOUT, 120 s)."""
    router = _Router(store, dp_size, heartbeat_timeout, stall_timeout=stall_timeout)
    return DPNodeVectorStore(worker, router), DPNodeSummarizer(worker, router)
