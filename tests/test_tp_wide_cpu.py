"""Tensor parallelism beyond two ranks, on the CPU (gloo): TP = 4 and TP = 8 of a decoder with
Llama-3-70B's head layout (64 q / 8 kv heads, so TP = 8 leaves ONE kv head per rank; preset
``tiny-70b-heads``), through the LLMEngine (prefill + decode, vocab-parallel argmax reduce) and
through ``services.main`` (continuous engine, TP followers replaying the leader's steps).

Numerics: greedy tokens are compared with TP = 1 on the same weights; the first token where they
differ (partial sums reduced in another order) must be a near-tie of the TP = 1 logits at that
prefix (teacher forced), and the TP prefill logits of every prefix must match TP = 1's."""
from __future__ import annotations

import os
import shutil
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

CFG = "tiny-70b-heads"
PROMPTS = [[1, 5, 9, 200, 17, 33, 7], [1] + list(range(40, 100)), [1, 2, 3], [1] + [77] * 21]
N_NEW = 6


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _engine(model, kv_heads):
    from copilot_for_consensus_amd.models.decoder import get_config
    from copilot_for_consensus_amd.runtime.engine import LLMEngine
    from copilot_for_consensus_amd.runtime.kv_cache import PagedKVCache
    cfg = get_config(CFG)
    return LLMEngine(model, PagedKVCache(cfg.layers, 96, kv_heads, cfg.head_dim, "cpu"), max_prefill_tokens=8192,
                     use_graph=False)


def _prefix_logits(eng, model, prefixes):
    """Last-token logits of every prefix (one prefill chunk), all-gathered over the TP group."""
    got = []
    orig = eng._next_tokens

    def cap(hidden, out, temperature, seed, step):
        got.append(model.logits(hidden).float().clone())
        return orig(hidden, out, temperature, seed, step)
    eng._next_tokens = cap
    eng.lpt = False           # the captured rows in the caller's prompt order, not longest-first
    try:
        eng.generate(prefixes, 1, ignore_eos=True)
    finally:
        eng._next_tokens = orig
        eng.lpt = True
    assert len(got) in (1, 2)       # TP: the chunk may run as two overlapped halves, rows in order
    return torch.cat(got)


def _full_weights():
    from copilot_for_consensus_amd.models.decoder import DecoderWeights, get_config
    return DecoderWeights.random(get_config(CFG), "cpu", seed=11)


def _reference():
    from copilot_for_consensus_amd.models.decoder import DecoderModel
    m = DecoderModel(_full_weights())
    eng = _engine(m, m.w.kv_heads)
    toks = eng.generate(PROMPTS, N_NEW, ignore_eos=True).tokens
    prefixes = [p + t[:i] for p, t in zip(PROMPTS, toks) for i in range(N_NEW)]
    return toks, prefixes, _prefix_logits(eng, m, prefixes)


def _tp_rank(rank, world, port, prefixes, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import traceback
    try:
        from copilot_for_consensus_amd.models.decoder import DecoderModel
        from copilot_for_consensus_amd.parallel import init_distributed, make_groups
        from copilot_for_consensus_amd.parallel.tp import shard_weights
        env = init_distributed(backend="gloo")
        g = make_groups(env, tp=world)
        w = shard_weights(_full_weights(), g.tp_rank, g.tp_size)
        m = DecoderModel(w, tp_group=g.tp_group)
        eng = _engine(m, w.kv_heads)
        toks = eng.generate(PROMPTS, N_NEW, ignore_eos=True).tokens
        logits = _prefix_logits(eng, m, prefixes)
        q.put((rank, True, (w.kv_heads, w.heads, toks, logits)))
    except Exception:  # noqa: BLE001
        q.put((rank, False, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("tp", [4, 8])
def test_tp_wide_matches_tp1_70b_head_layout(tp):
    ref_toks, prefixes, ref_logits = _reference()
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_tp_rank, args=(r, tp, port, prefixes, q)) for r in range(tp)]
    for p in procs:
        p.start()
    try:
        res = {}
        deadline = time.time() + 300
        while len(res) < tp and time.time() < deadline:
            if not q.empty():
                r, ok, payload = q.get()
                assert ok, f"rank {r}:\n{payload}"
                res[r] = payload
            else:
                time.sleep(0.05)
        assert len(res) == tp, f"ranks answered: {sorted(res)}"
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    kvh, qh, toks, logits = res[0]
    assert (kvh, qh) == (8 // tp, 64 // tp)              # TP = 8: one kv head (and 8 q heads) per rank
    for r in range(1, tp):
        assert res[r][2] == toks and torch.equal(res[r][3], logits)   # every rank holds the same answer
    # prefill logits of every teacher-forced prefix
    err = float((logits - ref_logits).abs().max() / ref_logits.abs().max())
    assert err < 2e-2, err
    # greedy tokens: equal to TP = 1 up to the first near-tie
    V = ref_logits.shape[1]
    for s, (a, b) in enumerate(zip(toks, ref_toks)):
        for i, (x, y) in enumerate(zip(a, b)):
            if x != y:
                row = ref_logits[s * N_NEW + i]
                gap = float(row[y] - row[x])
                assert 0 <= gap < 4 * err * float(ref_logits.abs().max()) + 1e-3, (s, i, x, y, gap)
                break
        assert all(0 <= t < V for t in a)


# ------------------------------------------------------------------ services.main at TP = 4
_TP4_ENV = {"DOCUMENT_STORE_TYPE": "inmemory", "MESSAGE_BUS_TYPE": "inproc", "METRICS_TYPE": "noop",
            "LOG_TYPE": "silent", "ERROR_REPORTER_TYPE": "silent", "EMBEDDING_BACKEND_TYPE": "mock",
            "VECTOR_STORE_TYPE": "inmemory", "ARCHIVE_STORE_TYPE": "inmemory", "SECRET_PROVIDER_TYPE": "env",
            "LLM_BACKEND_TYPE": "hip", "LLM_MODEL_PRESET": CFG, "CFC_TP": "4", "LLM_DEVICE": "cpu",
            "LLM_MAX_NEW_TOKENS": "6", "LLM_KV_CACHE_TOKENS": "8192", "LLM_MAX_BATCH": "8",
            "SUMMARIZATION_CONTINUOUS_BATCHING": "true", "CFC_DIST_BACKEND": "gloo", "CUDA_VISIBLE_DEVICES": ""}


def _node_rank(rank, port, src_dir, q):
    os.environ.update(_TP4_ENV, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="4",
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    try:
        from copilot_for_consensus_amd.services import main as M
        ctx = M._distributed()
        if not ctx["serve"]:
            q.put((rank, "follower", M._model_rank(ctx)))
            return
        from copilot_for_consensus_amd.services.node import Node
        node = Node(env=_TP4_ENV, summarizer=ctx["summarizer"])
        node.start(threaded=True)
        try:
            ing = node.services["ingestion"]
            ing.create_source({"name": "tp4", "source_type": "local", "url": src_dir})
            ing.trigger_ingestion("tp4")
            deadline = time.time() + 240
            while time.time() < deadline and node.store.count_documents("summaries") < 2:
                time.sleep(0.1)
            sums = node.store.query_documents("summaries", {}, limit=10)
            engine = ctx["local"]._ce
            q.put((rank, "leader", len(sums), dict(engine.stats) if engine else None,
                   int(ctx["local"].engine.model.w.kv_heads)))
        finally:
            node.stop()
            M._close_distributed(ctx)
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def test_services_main_tp4_continuous_node_three_followers(tmp_path):
    """services.main roles at CFC_TP=4 with the 70B head layout: rank 0 runs the node and the TP
    leader's continuous engine, THREE followers replay every engine step; the fixture's threads
    are summarized and every rank exits cleanly."""
    src = tmp_path / "src"
    src.mkdir()
    shutil.copy(os.path.join(os.path.dirname(__file__), "fixtures", "sample.mbox"), src / "a.mbox")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_node_rank, args=(r, port, str(src), q)) for r in range(4)]
    for p in procs:
        p.start()
    try:
        got = {}
        for _ in procs:
            item = q.get(timeout=300)
            got[item[0]] = item
        assert got[0][1] == "leader", got
        assert got[0][2] == 2 and got[0][3]["admitted"] == 2 and got[0][3]["finished"] == 2, got
        assert got[0][4] == 2                                   # 8 kv heads over 4 ranks
        assert all(got[r][1] == "follower" and got[r][2] == 0 for r in (1, 2, 3)), got
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0, [p.exitcode for p in procs]
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
