"""The DP node's control plane (parallel/dp_node.py) over a real TCPStore with 3 ranks on the CPU:
every request / reply / result key is deleted once consumed (the store stays bounded over many
batches), chunk texts travel over the document-store socket (only ids through the store), the
same thread summarized twice gets two results, handler errors reach the caller without marking
the rank dead, reads never queue behind a long embed, and clear() empties every shard."""
from __future__ import annotations

import datetime
import socket
import threading
import time

import pytest
import torch.multiprocessing as mp
from torch.distributed import TCPStore

from copilot_for_consensus_amd.summarization import Summarizer, Summary, Thread


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Sum(Summarizer):
    backend, model = "mock", "rank-mock"

    def __init__(self, rank):
        self.rank = rank

    def summarize(self, thread):
        return self.summarize_batch([thread])[0]

    def summarize_batch(self, threads):
        return [Summary(t.thread_id, f"rank{self.rank}:{t.thread_id}:{t.prompt}", [], self.backend, self.model,
                        1, 1, 0) for t in threads]


class _SlowEmbedder:
    """Mock embedder; texts starting with 'SLOW' take 3 s (an encoder forward on a big batch)."""
    model_name, backend, dimension = "mock-16", "mock", 16

    def __init__(self):
        from copilot_for_consensus_amd.embedding import MockEmbeddingProvider
        self.inner = MockEmbeddingProvider(16)

    def embed_tensor(self, texts):
        if any(t.startswith("SLOW") for t in texts):
            time.sleep(3.0)
        if any(t.startswith("FAIL") for t in texts):
            raise ValueError("encoder rejected the batch")
        return self.inner.embed_tensor(texts)


def _make_worker(store, rank, world):
    from copilot_for_consensus_amd.parallel.dp_node import DPNodeWorker
    from copilot_for_consensus_amd.vectorstore import InMemoryVectorStore
    return DPNodeWorker(store, rank, world, _SlowEmbedder(), InMemoryVectorStore(16), _Sum(rank),
                        heartbeat_interval=0.2)


def _rank_main(port, rank, world, q):
    store = TCPStore("127.0.0.1", port, is_master=False, timeout=datetime.timedelta(seconds=60))
    stats = _make_worker(store, rank, world).run_until_shutdown(poll_s=0.05)
    q.put((rank, stats))


@pytest.fixture
def node3():
    from copilot_for_consensus_amd.parallel.dp_node import build_rank0
    from copilot_for_consensus_amd.storage.document_store import InMemoryDocumentStore
    world = 3
    port = _free_port()
    store = TCPStore("127.0.0.1", port, is_master=True, wait_for_workers=False, timeout=datetime.timedelta(seconds=60))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(port, r, world, q), daemon=True) for r in range(1, world)]
    for p in procs:
        p.start()
    w0 = _make_worker(store, 0, world)
    vs, summ = build_rank0(store, world, w0, heartbeat_timeout=30.0)
    docs = InMemoryDocumentStore()
    docs.connect()
    vs.attach_document_store(docs)
    w0.start(serve=False)
    summ.start_continuous()
    deadline = time.time() + 120
    while not all(store.check([f"dpsum/hb/{r}"]) for r in range(world)):
        assert time.time() < deadline, "DP ranks never started"
        time.sleep(0.05)
    try:
        yield store, vs, summ, docs, w0, q, procs
    finally:
        from copilot_for_consensus_amd.parallel.dp_node import shutdown_workers
        summ.stop_continuous()
        shutdown_workers(store)
        w0.stop()
        vs.close()
        for p in procs:
            p.join(timeout=20)
            if p.is_alive():
                p.kill()


def _chunks(docs, batch, n_threads=6, per_thread=3, prefix=""):
    out = []
    for t in range(n_threads):
        tid = f"{batch:03d}{t:02d}" + "0" * 11
        for c in range(per_thread):
            cid = f"c{batch:03d}-{t}-{c}"
            text = f"{prefix}batch {batch} thread {t} chunk {c} about consensus"
            docs.insert_document("chunks", {"_id": cid, "thread_id": tid, "text": text})
            out.append({"id": cid, "thread_id": tid, "text": text, "meta": {"thread_id": tid, "chunk_index": c}})
    return out


def test_dp_node_store_keys_stay_bounded_over_50_batches(node3):
    store, vs, summ, docs, w0, q, procs = node3
    counts = []
    for b in range(50):
        chunks = _chunks(docs, b)
        assert vs.embed_and_store(chunks)["count"] == len(chunks)
        hits = vs.query([0.5] * 16, top_k=5)
        assert len(hits) == 5
        tids = sorted({c["thread_id"] for c in chunks})
        sc = vs.centroid_scores([c["id"] for c in chunks if c["thread_id"] == tids[0]], thread_id=tids[0])
        assert len(sc) == 3
        # the same thread twice in one batch, with different context: two results, none dropped
        threads = [Thread(tids[0], ["m"], prompt="ctx-a"), Thread(tids[0], ["m"], prompt="ctx-b"),
                   Thread(tids[1], ["m"], prompt="p")]
        out = summ.summarize_batch(threads)
        assert [s.summary_markdown.rsplit(":", 1)[1] for s in out] == ["ctx-a", "ctx-b", "p"]
        counts.append(store.num_keys())
    assert vs.count() == 50 * 18
    # nothing accumulates: request / reply / result keys are deleted once consumed
    assert max(counts[10:]) <= max(counts[:10]) + 2, counts
    assert max(counts) < 40, counts
    assert summ.stats["completed"] == 150 and summ.stats["duplicates"] == 0, summ.stats
    # every rank embedded its threads' chunks, reading the texts by id over the socket
    vs.clear()
    assert vs.count() == 0
    from copilot_for_consensus_amd.parallel.dp_node import shutdown_workers
    shutdown_workers(store)
    got = dict(q.get(timeout=60) for _ in procs)
    assert all(got[r]["embedded"] > 0 for r in (1, 2)), got
    assert w0.stats["embedded"] + got[1]["embedded"] + got[2]["embedded"] == 50 * 18


def test_dp_node_handler_error_is_not_rank_death_and_reads_skip_bulk_queue(node3):
    from copilot_for_consensus_amd.parallel.dp_node import RemoteError
    store, vs, summ, docs, w0, q, procs = node3
    # a failing embed on a worker rank: the caller sees the error, the rank stays routable
    bad = [c for c in _chunks(docs, 900, n_threads=12, prefix="FAIL ")]
    with pytest.raises((RemoteError, ValueError)):     # rank 0's share raises in place
        vs.embed_and_store(bad)
    assert vs.router.live() == [0, 1, 2]
    good = _chunks(docs, 901)
    assert vs.embed_and_store(good)["count"] == len(good)
    # a slow embed (3 s encoder forward) on every rank: topic reads answer meanwhile
    slow = _chunks(docs, 902, n_threads=12, prefix="SLOW ")
    th = threading.Thread(target=vs.embed_and_store, args=(slow,))
    th.start()
    time.sleep(0.5)
    t0 = time.perf_counter()
    n = vs.count()
    dt = time.perf_counter() - t0
    th.join()
    assert n >= len(good) and dt < 1.5, (n, dt)
    assert vs.count() == len(good) + len(slow)
    assert vs.stats["partial_reads"] == 0


def test_store_rpc_skips_a_sequence_number_whose_caller_died():
    from copilot_for_consensus_amd.parallel.dp_node import StoreRPC
    store = TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False, timeout=datetime.timedelta(seconds=10))
    srv = StoreRPC(store, 1, skip_grace_s=0.3)
    srv.handlers["echo"] = lambda a: a
    stop = threading.Event()
    t = threading.Thread(target=srv.serve, args=(stop,), kwargs={"poll_s": 0.05})
    t.start()
    try:
        store.add("dprpc/1/ctl/seq", 1)         # a caller reserved seq 1 and died before writing it
        cli = StoreRPC(store, 0)
        assert cli.call(1, "echo", {"x": 1}, timeout=10) == {"x": 1}
        assert srv.skipped == 1
        assert not store.check(["dprpc/1/ctl/req/2"]) and not store.check(["dprpc/1/ctl/res/2"])
    finally:
        stop.set()
        t.join()


def test_router_liveness_is_the_heartbeat_only_and_never_latched():
    """A rank is dead while its heartbeat is stale and routable again once it beats: nothing marks it
    dead permanently (a slow reply or a handler error never does)."""
    import json as _json

    from copilot_for_consensus_amd.parallel.dp_node import SUM_PREFIX, _Router
    store = TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False, timeout=datetime.timedelta(seconds=10))
    r = _Router(store, 3, timeout=1.0, cache_s=0.0)
    now = time.time()
    for k, t in ((0, now), (1, now - 5.0), (2, now)):
        store.set(f"{SUM_PREFIX}hb/{k}", _json.dumps({"t": t}))
    assert r.live() == [0, 2]
    tid = next(f"t{i}" for i in range(100) if __import__("copilot_for_consensus_amd.parallel.dp",
                                                            fromlist=["owner_of"]).owner_of(f"t{i}", 3) == 1)
    assert r.owner(tid) == 2                      # rank 1's thread goes to the next live rank
    store.set(f"{SUM_PREFIX}hb/1", _json.dumps({"t": time.time()}))
    assert r.live() == [0, 1, 2] and r.owner(tid) == 1   # it beats again: its threads come back


def test_router_rank_that_never_starts_is_dead_after_the_startup_grace():
    import json as _json

    from copilot_for_consensus_amd.parallel.dp_node import SUM_PREFIX, _Router
    store = TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False, timeout=datetime.timedelta(seconds=10))
    store.set(f"{SUM_PREFIX}hb/0", _json.dumps({"t": time.time() + 60}))
    r = _Router(store, 2, timeout=30.0, cache_s=0.0, startup_grace_s=0.3)
    assert r.live() == [0, 1]                     # rank 1 still loading its models
    time.sleep(0.4)
    assert r.live() == [0]                        # never came up: its threads go elsewhere
    store.set(f"{SUM_PREFIX}hb/1", _json.dumps({"t": time.time()}))
    assert r.live() == [0, 1]                     # late start: routable from its first beat


def test_chunk_text_server_is_read_only():
    """The DP data plane serves rank 0's store to the other ranks for reads only."""
    from copilot_for_consensus_amd.storage.document_store import DocumentStoreError, InMemoryDocumentStore
    from copilot_for_consensus_amd.storage.server import DocumentStoreServer, RemoteDocumentStore
    docs = InMemoryDocumentStore()
    docs.connect()
    docs.insert_document("chunks", {"_id": "c1", "text": "hello"})
    srv = DocumentStoreServer(docs, host="127.0.0.1", port=0, read_only=True).start()
    try:
        cli = RemoteDocumentStore("127.0.0.1", srv.port)
        cli.connect()
        assert cli.get_document("chunks", "c1")["text"] == "hello"
        with pytest.raises(DocumentStoreError):
            cli.insert_document("chunks", {"_id": "c2", "text": "x"})
        assert docs.get_document("chunks", "c2") is None
        cli.disconnect()
    finally:
        srv.server.shutdown()
        srv.server.server_close()


# ------------------------------------------------------------------ round 6: hung ranks, restarts
class _HangSum(_Sum):
    """Rank 2's engine blocks (a GPU hung in a kernel) on every thread whose prompt says HANG; its
    process and heartbeat thread stay up."""

    def summarize_batch(self, threads):
        if self.rank == 2 and any("HANG" in t.prompt for t in threads):
            time.sleep(40.0)
        return super().summarize_batch(threads)


def _hang_rank_main(port, rank, world, q):
    from copilot_for_consensus_amd.parallel.dp_node import DPNodeWorker
    from copilot_for_consensus_amd.vectorstore import InMemoryVectorStore
    store = TCPStore("127.0.0.1", port, is_master=False, timeout=datetime.timedelta(seconds=60))
    w = DPNodeWorker(store, rank, world, _SlowEmbedder(), InMemoryVectorStore(16), _HangSum(rank),
                     heartbeat_interval=0.2)
    q.put((rank, w.run_until_shutdown(poll_s=0.05)))


def test_dp_node_hung_rank_threads_are_resubmitted_within_the_stall_timeout():
    """3 ranks; rank 2's summarizer blocks forever while its heartbeat keeps beating.  Its threads
    are declared stalled (busy, progress frozen) and summarized by a live rank within stall_timeout
    + 2 s; threads of the other ranks are unaffected and nothing is delivered twice."""
    from copilot_for_consensus_amd.parallel.dp import owner_of
    from copilot_for_consensus_amd.parallel.dp_node import build_rank0, shutdown_workers
    world, stall = 3, 2.0
    port = _free_port()
    store = TCPStore("127.0.0.1", port, is_master=True, wait_for_workers=False, timeout=datetime.timedelta(seconds=60))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_hang_rank_main, args=(port, r, world, q), daemon=True) for r in range(1, world)]
    for p in procs:
        p.start()
    w0 = _make_worker(store, 0, world)
    vs, summ = build_rank0(store, world, w0, heartbeat_timeout=30.0, stall_timeout=stall)
    w0.start(serve=False)
    try:
        deadline = time.time() + 120
        while not all(store.check([f"dpsum/hb/{r}"]) for r in range(world)):
            assert time.time() < deadline, "DP ranks never started"
            time.sleep(0.05)
        tids = [f"{i:016x}" for i in range(400)]
        on2 = [t for t in tids if owner_of(t, world) == 2][:3]
        on1 = [t for t in tids if owner_of(t, world) == 1][:2]
        threads = [Thread(t, ["m"], prompt=f"HANG {t}") for t in on2] + [Thread(t, ["m"], prompt="p") for t in on1]
        t0 = time.perf_counter()
        out = summ.summarize_batch(threads)
        dt = time.perf_counter() - t0
        assert [s.thread_id for s in out] == [t.thread_id for t in threads]
        # rank 2's threads were finished elsewhere (rank 0 or 1), rank 1's by rank 1
        assert all(not s.summary_markdown.startswith("rank2:") for s in out), [s.summary_markdown for s in out]
        assert all(s.summary_markdown.startswith("rank1:") for s in out[3:])
        assert dt < stall + 2.0 + 1.0, dt          # + one heartbeat / watchdog period of slack
        assert summ.stats["resubmitted"] >= 3 and vs.router.stalls.get(2, 0) >= 1, (summ.stats, vs.router.stalls)
        assert not vs.router.alive(2) and vs.router.alive(1)
        # an idle rank is never "stalled": rank 1 did nothing since, and stays routable
        time.sleep(stall + 0.5)
        assert vs.router.alive(1)
    finally:
        summ.stop_continuous()
        shutdown_workers(store)
        w0.stop()
        vs.close()
        for p in procs:
            p.join(timeout=3)
            if p.is_alive():
                p.kill()


def test_dp_summarizer_batch_api_twice_without_a_started_stream(node3):
    """The batch API starts and stops the collectors per call (micro-batcher / synchronous callers):
    the second call must continue from the first call's result cursor (results are deleted once
    read, so a collector restarting at 1 would wait forever)."""
    store, vs, summ, docs, w0, q, procs = node3
    summ.stop_continuous()                        # the fixture streamed; this caller never starts one
    tids = [f"{i:016x}" for i in range(12)]
    for rnd in range(3):
        t0 = time.perf_counter()
        out = summ.summarize_batch([Thread(t, ["m"], prompt=f"r{rnd}") for t in tids])
        assert [s.summary_markdown.rsplit(":", 1)[1] for s in out] == [f"r{rnd}"] * len(tids)
        assert time.perf_counter() - t0 < 10.0
    assert summ.stats["duplicates"] == 0


def test_store_rpc_restarted_server_resumes_at_the_store_cursor():
    """A rank process restarted against the same store serves the next request at once: its cursor
    comes from the store's served counter, not from 0 (which would skip each consumed number after
    a 10 s grace)."""
    from copilot_for_consensus_amd.parallel.dp_node import StoreRPC
    store = TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False, timeout=datetime.timedelta(seconds=10))
    cli = StoreRPC(store, 0)
    for life in range(2):
        srv = StoreRPC(store, 1, skip_grace_s=30.0)
        srv.handlers["echo"] = lambda a, life=life: [life, a]
        stop = threading.Event()
        t = threading.Thread(target=srv.serve, args=(stop,), kwargs={"poll_s": 0.05})
        t.start()
        try:
            for i in range(5):
                t0 = time.perf_counter()
                assert cli.call(1, "echo", i, timeout=5) == [life, i]
                assert time.perf_counter() - t0 < 2.0
            assert srv.skipped == 0
        finally:
            stop.set()
            t.join()


def test_worker_result_numbers_continue_across_a_restart():
    """Result keys are numbered from a store counter: a restarted worker publishes at N+1, where
    rank 0's collector is waiting."""
    from copilot_for_consensus_amd.parallel.dp_node import SUM_PREFIX, DPNodeWorker
    from copilot_for_consensus_amd.vectorstore import InMemoryVectorStore
    store = TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False, timeout=datetime.timedelta(seconds=10))
    for life in range(2):
        w = DPNodeWorker(store, 1, 2, _SlowEmbedder(), InMemoryVectorStore(16), _Sum(1))
        for i in range(3):
            w._publish(f"k{life}{i}", None, RuntimeError("x"))
    assert [store.check([f"{SUM_PREFIX}out/1/{n}"]) for n in range(1, 8)] == [True] * 6 + [False]


def test_router_declares_a_busy_rank_with_frozen_progress_stalled_and_forgives_it():
    import json as _json

    from copilot_for_consensus_amd.parallel.dp_node import SUM_PREFIX, _Router
    store = TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False, timeout=datetime.timedelta(seconds=10))
    r = _Router(store, 2, timeout=30.0, cache_s=0.0, stall_timeout=0.3)

    def beat(rank, progress, busy):
        store.set(f"{SUM_PREFIX}hb/{rank}", _json.dumps({"t": time.time(), "progress": progress, "busy": busy}))
    beat(0, 5, 0)
    beat(1, 7, 2)
    assert r.live() == [0, 1]
    time.sleep(0.4)
    beat(0, 5, 0)                 # idle, no progress: fine
    beat(1, 7, 2)                 # busy, no progress for > 0.3 s: stalled
    assert r.live() == [0] and r.stalls == {1: 1}
    beat(1, 8, 2)                 # progress again: routable again
    assert r.live() == [0, 1]
