"""Data-parallel summarization in the services (parallel/dp_service.py, services/main.py under
torchrun): rank 0's DPSummarizer shards every batch over the DP workers through the job store;
every thread gets exactly one summary, also when a worker is killed mid-batch; the torchrun entry
point assigns the roles (2 gloo ranks on the CPU, mock LLM)."""
from __future__ import annotations

import os
import signal
import socket
import time

import pytest
import torch.multiprocessing as mp
from torch.distributed import TCPStore

from copilot_for_consensus_amd.summarization import Summarizer, Summary, Thread


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class RankSummarizer(Summarizer):
    """Tags each summary with the rank that produced it; rank ``slow`` blocks on its first batch
    (so the test can kill it while it holds unfinished threads)."""
    backend, model = "mock", "rank-mock"

    def __init__(self, rank, store=None, slow=None):
        self.rank, self.store, self.slow, self.calls = rank, store, slow, 0

    def summarize(self, thread):
        return self.summarize_batch([thread])[0]

    def summarize_batch(self, threads):
        self.calls += 1
        if self.rank == self.slow and self.store is not None:
            self.store.set(f"started/{self.rank}", "1")
            time.sleep(3600)
        time.sleep(0.01 * len(threads))
        return [Summary(t.thread_id, f"rank{self.rank}:{t.thread_id}", [], self.backend, self.model, 1, 1, 0)
                for t in threads]


def _worker(port, rank, world, slow, q):
    from copilot_for_consensus_amd.parallel.dp_service import dp_worker_loop
    store = TCPStore("127.0.0.1", port, is_master=False, timeout=__import__("datetime").timedelta(seconds=60))
    jobs = dp_worker_loop(store, rank, world, RankSummarizer(rank, store, slow), batch_size=4, timeout=3.0,
                          heartbeat_interval=0.3, max_idle_s=60)
    q.put((rank, jobs))


def _threads(n, tag="t"):
    return [Thread(f"{tag}{i:03d}", [f"message {i}"], prompt=f"prompt {i} " * (1 + i % 7)) for i in range(n)]


def _start(world, slow=None):
    import datetime

    from copilot_for_consensus_amd.parallel.dp_service import DPSummarizer
    port = _free_port()
    store = TCPStore("127.0.0.1", port, is_master=True, wait_for_workers=False,
                     timeout=datetime.timedelta(seconds=60))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = {r: ctx.Process(target=_worker, args=(port, r, world, slow, q), daemon=True) for r in range(1, world)}
    for p in procs.values():
        p.start()
    dps = DPSummarizer(store, world, RankSummarizer(0), batch_size=4, timeout=3.0, heartbeat_interval=0.3)
    assert dps.wait_workers(120) == world
    return store, dps, procs, q


def test_dp_summarizer_covers_every_thread_once():
    store, dps, procs, q = _start(3)
    try:
        for batch in (_threads(30, "a"), _threads(7, "b"), _threads(1, "c")):
            out = dps.summarize_batch(batch)
            assert [s.thread_id for s in out] == [t.thread_id for t in batch]
            assert all(s.summary_markdown.endswith(":" + s.thread_id) for s in out)
        ranks = {s.summary_markdown.split(":")[0] for s in dps.summarize_batch(_threads(40, "d"))}
        assert len(ranks) >= 2, ranks           # the work really spread over the workers
        dps.close()
        done = dict(q.get(timeout=60) for _ in procs)
        assert set(done) == {1, 2} and all(1 <= v <= 4 for v in done.values()), done
    finally:
        for p in procs.values():
            p.join(timeout=10)
            if p.is_alive():
                p.kill()


def test_killed_worker_threads_are_taken_over():
    store, dps, procs, q = _start(3, slow=2)
    try:
        import threading
        box = {}
        th = threading.Thread(target=lambda: box.setdefault("out", dps.summarize_batch(_threads(24, "k"))))
        th.start()
        deadline = time.time() + 60
        while not store.check(["started/2"]):
            assert time.time() < deadline, "worker 2 never started its batch"
            time.sleep(0.05)
        os.kill(procs[2].pid, signal.SIGKILL)        # dies holding unfinished threads
        th.join(timeout=90)
        assert not th.is_alive(), "the job never completed after the worker died"
        out = box["out"]
        assert [s.thread_id for s in out] == [f"k{i:03d}" for i in range(24)]
        assert {s.summary_markdown.split(":")[0] for s in out} <= {"rank0", "rank1"}
        dps.close()
        assert q.get(timeout=60)[0] == 1
    finally:
        for p in procs.values():
            p.join(timeout=10)
            if p.is_alive():
                p.kill()


_DP_NODE_ENV = {"DOCUMENT_STORE_TYPE": "inmemory", "MESSAGE_BUS_TYPE": "inproc", "METRICS_TYPE": "noop",
                "LOG_TYPE": "silent", "ERROR_REPORTER_TYPE": "silent", "EMBEDDING_BACKEND_TYPE": "mock",
                "VECTOR_STORE_TYPE": "inmemory", "ARCHIVE_STORE_TYPE": "inmemory", "SECRET_PROVIDER_TYPE": "env",
                "LLM_BACKEND_TYPE": "mock", "MOCK_LATENCY_MS": "20", "CFC_DIST_BACKEND": "gloo",
                "CUDA_VISIBLE_DEVICES": "", "SUMMARIZATION_CONTINUOUS_BATCHING": "true"}


def _write_mbox(path, n_threads, seed=1):
    from copilot_for_consensus_amd.utils.synthetic import SyntheticArchive
    path.mkdir(parents=True, exist_ok=True)
    (path / "list.mbox").write_bytes(SyntheticArchive(seed=seed).mbox(n_threads, messages_per_thread=(2, 3)))


def _dp_node_rank(rank, world, port, src_dir, n_threads, q, kill_rank=None):
    os.environ.update(_DP_NODE_ENV, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    if kill_rank is not None and rank == kill_rank:
        os.environ["MOCK_LATENCY_MS"] = "600000"            # never finishes a thread: killed holding work
    if kill_rank is None:
        # nothing is killed here: a rank stalled by a loaded CPU (parallel test workers) must not be
        # taken for dead, which would move its threads and break the both-ranks-worked checks
        os.environ["CFC_DP_HEARTBEAT_TIMEOUT"] = "120"
    try:
        from copilot_for_consensus_amd.services import main as M
        ctx = M._distributed()
        if not ctx["serve"]:
            M._model_rank(ctx)
            q.put((rank, "worker", ctx.get("worker_stats")))
            return
        from copilot_for_consensus_amd.services.node import Node
        node = Node(env=_DP_NODE_ENV, summarizer=ctx["summarizer"], vector_store=ctx["vector_store"],
                    embedding_provider=ctx["embedder"])
        node.start(threaded=True)
        try:
            ing = node.services["ingestion"]
            ing.create_source({"name": "dp", "source_type": "local", "url": src_dir})
            ing.trigger_ingestion("dp")
            if kill_rank is not None:
                deadline = time.time() + 120
                summ = ctx["summarizer"]
                while time.time() < deadline and not any(r == kill_rank for *_, r in list(summ._inflight.values())):
                    time.sleep(0.05)
                time.sleep(0.5)
                q.put((rank, "kill", kill_rank))             # it holds threads: the test kills it now
            deadline = time.time() + 240
            while time.time() < deadline and node.store.count_documents("summaries") < n_threads:
                time.sleep(0.1)
            n_sum = node.store.count_documents("summaries")
            n_thr = node.store.count_documents("threads")
            hits = node.services["reporting"].search_reports_by_topic("the working group discussion", limit=5,
                                                                       min_score=-1.0)
            q.put((rank, "leader", type(ctx["summarizer"]).__name__, n_thr, n_sum, dict(ctx["summarizer"].stats),
                   dict(ctx["worker"].stats), ctx["vector_store"].count(), len(hits)))
        finally:
            node.stop()
            M._close_distributed(ctx)
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def _run_dp_node(tmp_path, world, n_threads, kill_rank=None):
    src = tmp_path / "src"
    _write_mbox(src, n_threads)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_node_rank, args=(r, world, port, str(src), n_threads, q, kill_rank))
             for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        while len(got) < world:
            item = q.get(timeout=300)
            if item[1] == "kill":
                os.kill(procs[item[2]].pid, signal.SIGKILL)
                got[item[2]] = (item[2], "killed")
                continue
            got[item[0]] = item
        for p in procs:
            p.join(timeout=60)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    return got, procs


def test_services_main_torchrun_roles(tmp_path):
    """services.main under a 2-rank (gloo) torchrun env, the whole node on rank 0 with DP routing
    (parallel/dp_node.py): BOTH ranks embed chunks into their own index shards and summarize the
    threads they own; every thread gets exactly one summary; topic search fans out over the shards;
    rank 1 exits when rank 0 closes."""
    n = 12
    got, procs = _run_dp_node(tmp_path, 2, n)
    assert got[0][1] == "leader" and got[0][2] == "DPNodeSummarizer", got
    _, _, _, n_thr, n_sum, sstats, w0, n_vec, n_hits = got[0]
    assert n_thr == n and n_sum == n, got[0]
    assert sstats["completed"] == n and sstats["duplicates"] == 0, sstats
    assert all(c > 0 for c in sstats["per_rank"]), sstats          # both ranks summarized
    assert got[1][1] == "worker", got
    w1 = got[1][2]
    assert w0["embedded"] > 0 and w1["embedded"] > 0, (w0, w1)      # both ranks embedded their threads' chunks
    assert w0["embedded"] + w1["embedded"] == n_vec and w1["summaries"] == sstats["per_rank"][1]
    assert w1["queries"] >= 1 and n_hits >= 1                        # the topic search reached rank 1's shard
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_dp_node_killed_rank_threads_taken_over(tmp_path):
    """3 DP ranks; rank 2 is killed while it holds threads: its heartbeat goes stale, rank 0
    resubmits them to the live ranks and every thread still gets exactly one summary."""
    n = 12
    got, procs = _run_dp_node(tmp_path, 3, n, kill_rank=2)
    assert got[0][1] == "leader", got
    _, _, _, n_thr, n_sum, sstats, *_ = got[0]
    assert n_sum == n_thr == n, got[0]
    assert sstats["resubmitted"] >= 1 and sstats["per_rank"][2] == 0, sstats
    assert sstats["completed"] == n, sstats
    assert got[1][1] == "worker" and got[2][1] == "killed", got


_TP_NODE_ENV = {"DOCUMENT_STORE_TYPE": "inmemory", "MESSAGE_BUS_TYPE": "inproc", "METRICS_TYPE": "noop",
                "LOG_TYPE": "silent", "ERROR_REPORTER_TYPE": "silent", "EMBEDDING_BACKEND_TYPE": "mock",
                "VECTOR_STORE_TYPE": "inmemory", "ARCHIVE_STORE_TYPE": "inmemory", "SECRET_PROVIDER_TYPE": "env",
                "LLM_BACKEND_TYPE": "hip", "LLM_MODEL_PRESET": "tiny", "CFC_TP": "2", "LLM_DEVICE": "cpu",
                "LLM_MAX_NEW_TOKENS": "8", "LLM_KV_CACHE_TOKENS": "8192", "LLM_MAX_BATCH": "8",
                "SUMMARIZATION_CONTINUOUS_BATCHING": "true", "CFC_DIST_BACKEND": "gloo", "CUDA_VISIBLE_DEVICES": ""}


def _tp_node_rank(rank, port, src_dir, q):
    os.environ.update(_TP_NODE_ENV, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK=str(rank))
    import torch
    torch.set_num_threads(2)
    try:
        from copilot_for_consensus_amd.services import main as M
        ctx = M._distributed()
        if not ctx["serve"]:
            q.put((rank, "follower", M._model_rank(ctx)))
            return
        from copilot_for_consensus_amd.services.node import Node
        node = Node(env=_TP_NODE_ENV, summarizer=ctx["summarizer"])
        node.start(threaded=True)
        try:
            ing = node.services["ingestion"]
            ing.create_source({"name": "tp", "source_type": "local", "url": src_dir})
            ing.trigger_ingestion("tp")
            deadline = time.time() + 240
            while time.time() < deadline and node.store.count_documents("summaries") < 2:
                time.sleep(0.1)
            sums = node.store.query_documents("summaries", {}, limit=10)
            engine = ctx["local"]._ce
            q.put((rank, "leader", type(ctx["summarizer"]).__name__, len(sums), dict(engine.stats) if engine else None))
        finally:
            node.stop()
            M._close_distributed(ctx)
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def test_services_main_tp2_continuous_node_summarizes_and_exits(tmp_path):
    """services.main roles with CFC_TP=2 and continuous batching on (tiny decoder, 2 gloo ranks on
    the CPU): rank 0 runs the whole node, its summarizer the TP leader's continuous engine; rank 1
    replays every engine step (prefills, decode bursts: their all-reduces pair up).  The node
    summarizes the fixture's threads through the bus and both ranks exit cleanly -- the round-3
    deadlock (followers waiting on a broadcast the continuous engine never sent) is gone."""
    import shutil
    src = tmp_path / "src"
    src.mkdir()
    shutil.copy(os.path.join(os.path.dirname(__file__), "fixtures", "sample.mbox"), src / "a.mbox")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tp_node_rank, args=(r, port, str(src), q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got = {}
        for _ in procs:
            item = q.get(timeout=300)
            got[item[0]] = item
        assert got[0][1] == "leader", got
        assert got[0][2] == "HipLLMSummarizer" and got[0][3] == 2, got
        assert got[0][4]["admitted"] == 2 and got[0][4]["finished"] == 2, got
        assert got[1][1] == "follower" and got[1][2] == 0, got      # _model_rank exit code
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0, [p.exitcode for p in procs]
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
