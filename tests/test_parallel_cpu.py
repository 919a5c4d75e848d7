"""Multi-process (gloo, world_size 2) tests of the parallel layer: TP decoder == unsharded decoder,
sharded kNN == single index, DP sharding helpers."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from copilot_for_consensus_amd.parallel.dp import balanced_shard, gather_objects, hash_shard, owner_of


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(fn, world, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_entry, args=(fn, r, world, port, q, args)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    results = {}
    while not q.empty():
        r, ok, payload = q.get()
        results[r] = (ok, payload)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert len(results) == world, f"missing ranks: {results}"
    for r, (ok, payload) in sorted(results.items()):
        assert ok, f"rank {r} failed:\n{payload}"
    return [results[r][1] for r in range(world)]


def _entry(fn, rank, world, port, q, args):
    import traceback
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    try:
        from copilot_for_consensus_amd.parallel import init_distributed
        env = init_distributed(backend="gloo")
        out = fn(env, *args)
        q.put((rank, True, out))
    except Exception:
        q.put((rank, False, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


# ---------------------------------------------------------------- TP decoder
def _tp_generate(env, prompts, n_new):
    from copilot_for_consensus_amd.models.decoder import DecoderModel, DecoderWeights, get_config
    from copilot_for_consensus_amd.parallel import make_groups
    from copilot_for_consensus_amd.parallel.tp import shard_weights
    from copilot_for_consensus_amd.runtime.engine import LLMEngine
    from copilot_for_consensus_amd.runtime.kv_cache import PagedKVCache

    cfg = get_config("tiny")
    g = make_groups(env, tp=env.world)
    full = DecoderWeights.random(cfg, "cpu", seed=5)
    w = shard_weights(full, g.tp_rank, g.tp_size)
    m = DecoderModel(w, tp_group=g.tp_group)
    kv = PagedKVCache(cfg.layers, 64, w.kv_heads, cfg.head_dim, "cpu")
    return LLMEngine(m, kv).generate(prompts, n_new, ignore_eos=True).tokens


def test_tp2_decoder_matches_unsharded():
    from copilot_for_consensus_amd.models.decoder import DecoderModel, DecoderWeights, get_config
    from copilot_for_consensus_amd.runtime.engine import LLMEngine
    from copilot_for_consensus_amd.runtime.kv_cache import PagedKVCache

    prompts = [[1, 5, 9, 200, 17, 33], [1] + list(range(40, 110)), [1, 2]]
    cfg = get_config("tiny")
    ref = LLMEngine(DecoderModel(DecoderWeights.random(cfg, "cpu", seed=5)),
                    PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, "cpu")).generate(
        prompts, 8, ignore_eos=True).tokens
    outs = _run(_tp_generate, 2, prompts, 8)
    assert outs[0] == outs[1]
    # fp32-accumulated partial sums are reduced in a different order; greedy tokens must agree
    agree = sum(a == b for x, y in zip(outs[0], ref) for a, b in zip(x, y))
    assert agree >= 0.9 * sum(len(x) for x in ref), (outs[0], ref)


def _tp_prefill_overlap(env, prompts):
    """Last-token prefill hidden states of every prompt at TP = world, one pass vs two overlapped
    halves (async all-reduces interleaved with the other half's compute)."""
    from copilot_for_consensus_amd.models.decoder import DecoderModel, DecoderWeights, get_config
    from copilot_for_consensus_amd.parallel import make_groups
    from copilot_for_consensus_amd.parallel.tp import shard_weights
    from copilot_for_consensus_amd.runtime.engine import LLMEngine
    from copilot_for_consensus_amd.runtime.kv_cache import PagedKVCache

    cfg = get_config("tiny")
    g = make_groups(env, tp=env.world)
    m = DecoderModel(shard_weights(DecoderWeights.random(cfg, "cpu", seed=5), g.tp_rank, g.tp_size),
                     tp_group=g.tp_group)
    out = {}
    for overlap in (False, True):
        eng = LLMEngine(m, PagedKVCache(cfg.layers, 64, m.w.kv_heads, cfg.head_dim, "cpu"), prefix_cache=False)
        eng.tp_overlap, eng.lpt = overlap, False
        seen, calls = [], []
        orig_next, orig_ov = eng._next_tokens, m.forward_prefill_overlap

        def cap(hidden, o, t, s, st, orig_next=orig_next, seen=seen):
            seen.append(hidden.float().clone())
            return orig_next(hidden, o, t, s, st)

        def ov(*a, orig_ov=orig_ov, calls=calls, **k):
            calls.append(1)
            return orig_ov(*a, **k)
        eng._next_tokens, m.forward_prefill_overlap = cap, ov
        try:
            toks = eng.generate(prompts, 1, ignore_eos=True).tokens
        finally:
            m.forward_prefill_overlap = orig_ov
        out[overlap] = (torch.cat(seen).numpy(), toks, len(calls))    # by value: the rank exits first
    return out



class _EpochAR:
    """CPU stand-in of parallel.custom_ar.OneShotAllReduce with comm.hip's epoch bookkeeping: a sum
    call advances epochs[0:nb] (nb = min(ceil(n / 8 / 256), blocks)), a key-max call the last
    block; the reduction itself goes through gloo.  Two ranks whose call sequences differ end with
    different epoch arrays -- the desync that would make every later call of the lagging rank spin
    to its timeout."""

    def __init__(self, group, blocks: int = 32):
        self.group, self.blocks, self.enabled = group, blocks, True
        self.staging_bytes, self.key_rows = 8 << 20, 1024
        self.epochs = [0] * 64
        self.log = []
        self.busy = False

    def supports(self, x):
        return x.numel() % 8 == 0 and x.numel() * 2 <= self.staging_bytes

    def supports_keys(self, n):
        return 0 < n <= self.key_rows

    def _enter(self, tag, nb):
        assert not self.busy, "two one-shot all-reduces in flight at once on one rank"
        self.log.append((tag, nb))

    def __call__(self, x, out=None):
        nb = min(-(-(x.numel() // 8) // 256), self.blocks)
        self._enter("sum", nb)
        for b in range(63):          # every sum-type launch advances all 63 sum blocks' epochs
            self.epochs[b] += 1
        dist.all_reduce(x, group=self.group)
        return x if out is None else out.copy_(x)

    def supports_slabs(self, part):
        return part.shape[1] * part.shape[2] * 4 <= self.staging_bytes

    def residual_rmsnorm(self, part, residual, norm_w, eps):
        """The fused fp32 all-reduce + residual + RMSNorm (comm.hip oneshot_ar_residual_rmsnorm)."""
        from copilot_for_consensus_amd.ops import kernels as K
        self._enter("norm", min(part.shape[1], self.blocks))
        for b in range(63):
            self.epochs[b] += 1
        t = part.sum(0, keepdim=True)
        dist.all_reduce(t, group=self.group)
        return K.splitk_residual_rmsnorm(t, residual, norm_w, eps)

    def keymax(self, keys, out_ids):
        self._enter("keymax", 1)
        self.epochs[63] += 1
        dist.all_reduce(keys, op=dist.ReduceOp.MAX, group=self.group)
        return out_ids.copy_((0xFFFFFFFF - (keys & 0xFFFFFFFF)).to(torch.int32))


def _tp_overlap_epochs(env, batches):
    """Two batches through the engine with the overlapped TP prefill ON and greedy decode, the
    one-shot all-reduce replaced by _EpochAR: returns (log, epochs, calls inside the overlapped
    prefill, tokens) per rank."""
    from copilot_for_consensus_amd.models.decoder import DecoderModel, DecoderWeights, get_config
    from copilot_for_consensus_amd.parallel import make_groups
    from copilot_for_consensus_amd.parallel.tp import shard_weights
    from copilot_for_consensus_amd.runtime.engine import LLMEngine
    from copilot_for_consensus_amd.runtime.kv_cache import PagedKVCache

    cfg = get_config("tiny")
    g = make_groups(env, tp=env.world)
    ar = _EpochAR(g.tp_group)
    m = DecoderModel(shard_weights(DecoderWeights.random(cfg, "cpu", seed=5), g.tp_rank, g.tp_size),
                     tp_group=g.tp_group, custom_ar=ar)
    eng = LLMEngine(m, PagedKVCache(cfg.layers, 64, m.w.kv_heads, cfg.head_dim, "cpu"))
    eng.tp_overlap = True
    inside = []
    orig = m.forward_prefill_overlap

    def ov(*a, **k):
        n0 = len(ar.log)
        try:
            return orig(*a, **k)
        finally:
            inside.append(len(ar.log) - n0)
    m.forward_prefill_overlap = ov
    toks = [eng.generate(p, 6, ignore_eos=True).tokens for p in batches]
    return ar.log, ar.epochs, inside, toks


def test_tp2_overlapped_prefill_keeps_one_shot_allreduce_epochs_in_step():
    """The overlapped TP prefill runs its all-reduces on the process group, never on the one-shot
    kernel, and every rank makes the same one-shot calls (same order, same block counts) over two
    batches of prefill + greedy decode -- so the per-block epochs of comm.hip stay equal on all
    ranks (round-5 stall investigation: scripts/tp_rehearsal.sh with CFC_TP_PREFILL_OVERLAP=force
    CFC_AR_DEBUG=1 read the real counters on the GPU,
    errors 0 and identical epochs on both ranks after each batch, profiles/r06_tp2_overlap_gloo_1gpu.log)."""
    batches = [[[1, 5, 9, 200, 17, 33], [1] + list(range(40, 110)), [1, 2], [1] + [7] * 40],
               [[1, 3] * 20, [1, 9, 9], [1] + list(range(300, 340))]]
    outs = _run(_tp_overlap_epochs, 2, batches)
    (log0, ep0, in0, t0), (log1, ep1, in1, t1) = outs
    assert in0 == in1 and len(in0) == 2 and all(n == 0 for n in in0), (in0, in1)
    assert log0 == log1 and ep0 == ep1
    assert any(tag == "norm" for tag, _ in log0) and any(tag == "keymax" for tag, _ in log0)
    assert t0 == t1


def test_tp2_prefill_overlapped_halves_match_one_pass():
    prompts = [[1, 5, 9, 200, 17, 33], [1] + list(range(40, 110)), [1, 2], [1] + [7] * 40]
    outs = _run(_tp_prefill_overlap, 2, prompts)
    for r in outs:
        (h1, t1, c1), (h2, t2, c2) = r[False], r[True]
        h1, h2 = torch.from_numpy(h1), torch.from_numpy(h2)
        assert c1 == 0 and c2 == 1                       # the overlapped path ran (one chunk, two halves)
        assert h1.shape == h2.shape == (len(prompts), h1.shape[1])
        assert float((h1 - h2).abs().max()) <= 2e-2 * float(h1.abs().max()), float((h1 - h2).abs().max())
        assert t1 == t2


def test_shard_weights_reassemble():
    from copilot_for_consensus_amd.models.decoder import DecoderWeights, get_config
    from copilot_for_consensus_amd.parallel.tp import shard_weights
    cfg = get_config("tiny")
    full = DecoderWeights.random(cfg, "cpu", seed=1)
    s0, s1 = shard_weights(full, 0, 2), shard_weights(full, 1, 2)
    D, hq, hk = cfg.head_dim, cfg.heads // 2, cfg.kv_heads // 2
    q = torch.cat([s0.layers[0]["qkv"][:hq * D], s1.layers[0]["qkv"][:hq * D]])
    assert torch.equal(q, full.layers[0]["qkv"][:cfg.heads * D])
    k1 = s1.layers[0]["qkv"][hq * D:(hq + hk) * D]
    assert torch.equal(k1, full.layers[0]["qkv"][cfg.heads * D + hk * D:cfg.heads * D + 2 * hk * D])
    assert torch.equal(torch.cat([s0.layers[0]["down"], s1.layers[0]["down"]], 1), full.layers[0]["down"])
    assert torch.equal(torch.cat([s0.lm_head, s1.lm_head]), full.lm_head)


def test_random_sharded_replicates_embeddings():
    from copilot_for_consensus_amd.models.decoder import DecoderWeights, get_config
    cfg = get_config("tiny")
    a = DecoderWeights.random(cfg, "cpu", seed=3, tp_rank=0, tp_size=2)
    b = DecoderWeights.random(cfg, "cpu", seed=3, tp_rank=1, tp_size=2)
    assert torch.equal(a.embed, b.embed)
    assert not torch.equal(a.layers[0]["qkv"], b.layers[0]["qkv"])


# ---------------------------------------------------------------- sharded kNN
def _knn(env, X, ids, Q, k):
    from copilot_for_consensus_amd.parallel.knn import ShardedVectorIndex
    from copilot_for_consensus_amd.vectorstore import HipFlatIndex
    idx = ShardedVectorIndex(HipFlatIndex(X.shape[1], device="cpu", capacity=256))
    idx.add_embeddings(ids, X, [{"i": i} for i in range(len(ids))])
    res = idx.query_batch(Q, k)
    n_local = idx.local.count()
    got = idx.get(ids[7])
    return [[(r.id, round(r.score, 4), r.metadata["i"]) for r in q] for q in res], n_local, idx.count(), got.id


def test_sharded_knn_matches_single_index():
    from copilot_for_consensus_amd.vectorstore import HipFlatIndex
    g = torch.Generator().manual_seed(0)
    X = torch.randn(300, 32, generator=g)
    Q = torch.randn(5, 32, generator=g)
    ids = [f"c{i}" for i in range(300)]
    single = HipFlatIndex(32, device="cpu")
    single.add_embeddings(ids, X)
    ref = [[r.id for r in q] for q in single.query_batch(Q, 10)]
    outs = _run(_knn, 2, X, ids, Q, 10)
    assert outs[0][0] == outs[1][0]
    assert [[t[0] for t in q] for q in outs[0][0]] == ref
    assert outs[0][1] + outs[1][1] == 300 and 0 < outs[0][1] < 300
    assert outs[0][2] == 300 and outs[0][3] == "c7"


def _thread_rows(env, batches):
    """Each rank inserts ITS batch (rank-local threads) through add_thread_rows."""
    from copilot_for_consensus_amd.parallel.knn import ShardedVectorIndex
    from copilot_for_consensus_amd.vectorstore import HipFlatIndex
    idx = ShardedVectorIndex(HipFlatIndex(32, device="cpu", capacity=512))
    tids, ids, X = batches[env.rank]
    sc = idx.add_thread_rows(tids, ids, X)
    stored = {idx.local._tab.id_at(r): idx.local._tab.meta_at(r)["thread_id"] for r in range(idx.local._n)}
    return sc.tolist(), stored


def test_thread_owned_sharded_insert_and_relevance_matches_single_index():
    """DP data plane of the bench / orchestrator: every rank's rows land on the shard that owns
    their THREAD, and the relevance scores that come back equal the single-index computation
    (cosine of each row to its own thread's centroid) for every rank's batch."""
    from copilot_for_consensus_amd.parallel.dp import owner_of
    from copilot_for_consensus_amd.vectorstore import HipFlatIndex
    g = torch.Generator().manual_seed(3)
    batches = []
    for r in range(2):
        tids, ids = [], []
        for t in range(9):
            for c in range(1 + (t * 7 + r) % 4):
                tids.append(f"r{r}-thread-{t}")
                ids.append(f"r{r}-t{t}-c{c}")
        batches.append((tids, ids, torch.randn(len(ids), 32, generator=g)))
    outs = _run(_thread_rows, 2, batches)
    for r, (tids, ids, X) in enumerate(batches):
        single = HipFlatIndex(32, device="cpu")
        single.add_embeddings(ids, X)
        spans, a = [], 0
        for i in range(1, len(ids) + 1):
            if i == len(ids) or tids[i] != tids[a]:
                spans.append((a, i))
                a = i
        want = HipFlatIndex.span_centroid_scores(single._X, spans).tolist()
        assert outs[r][0] == pytest.approx(want, abs=1e-5)
    # every row is stored exactly once, on its thread's owner
    seen = {}
    for r, (_, stored) in enumerate(outs):
        for cid, tid in stored.items():
            assert owner_of(tid, 2) == r and cid not in seen
            seen[cid] = tid
    assert len(seen) == sum(len(b[1]) for b in batches)


# ---------------------------------------------------------------- DP helpers
def test_owner_and_hash_shard_are_stable_partitions():
    keys = [f"thread-{i}" for i in range(1000)]
    parts = [hash_shard(keys, r, 4) for r in range(4)]
    assert sorted(sum(parts, [])) == sorted(keys)
    assert all(150 < len(p) < 350 for p in parts)
    assert owner_of("abc", 4) == owner_of("abc", 4) and owner_of("abc", 1) == 0


def test_balanced_shard_lpt():
    costs = [10, 9, 8, 1, 1, 1, 1, 1]
    bins = balanced_shard(costs, 3)
    loads = sorted(sum(costs[i] for i in b) for b in bins)
    assert sorted(sum(bins, [])) == list(range(8))
    assert loads[-1] - loads[0] <= 2


def test_gather_objects_single_process():
    assert gather_objects({"a": 1}) == [{"a": 1}]


def _gather(env):
    return gather_objects({"rank": env.rank})


def test_gather_objects_two_ranks():
    outs = _run(_gather, 2)
    assert outs[0] == outs[1] == [{"rank": 0}, {"rank": 1}]


# ---------------------------------------------------------------- TP bench pipeline
def _tp_bench(env):
    from copilot_for_consensus_amd.parallel import make_groups
    from copilot_for_consensus_amd.pipeline.bench_pipeline import BenchPipeline
    g = make_groups(env, tp=2)
    p = BenchPipeline(model="tiny", encoder="tiny", device="cpu", threads_per_step=2, max_new_tokens=3,
                      prefill_tokens=4096, seed=5, index_prefill=0, tp=2, groups=g)
    p.prepare_sources([0, 1])
    res = p.run_steps([0, 1], overlap=True)
    return [(r.threads, r.generated_tokens, r.prompt_tokens) for r in res]


def test_tp2_bench_pipeline_leader_broadcasts_prompts():
    outs = _run(_tp_bench, 2)
    lead, fol = outs
    assert [t for t, _, _ in lead] == [2, 2] and [t for t, _, _ in fol] == [0, 0]
    assert [x[1:] for x in lead] == [x[1:] for x in fol]  # same prompts, same generation length


# ---------------------------------------------------------------- failure detection / recovery
def test_watchdog_detects_dead_rank_and_reclaims_work():
    from copilot_for_consensus_amd.parallel.resilience import Heartbeat, Watchdog, WorkLedger
    store = dist.HashStore()
    now = [1000.0]
    clock = lambda: now[0]  # noqa: E731
    hbs = [Heartbeat(store, r, clock=clock) for r in range(3)]
    for h in hbs:
        h.beat()
    ledger = WorkLedger(store)
    for r in range(3):
        ledger.assign(r, [f"t{r}-{i}" for i in range(4)])
    ledger.complete(1, ["t1-0"])
    wd = Watchdog(store, 3, timeout=10.0, stall_timeout=20.0, clock=clock)
    assert wd.dead_ranks() == []
    now[0] += 15.0                      # rank 1 stops beating (process died)
    hbs[0].beat(); hbs[2].beat()
    assert wd.dead_ranks() == [1]
    moved = wd.reclaim(ledger)
    assert sorted(i for v in moved.values() for i in v) == ["t1-1", "t1-2", "t1-3"]
    assert set(moved) <= {0, 2} and ledger.pending(1) == []
    assert set(ledger.pending(0)) >= {"t0-0"} and len(ledger.pending(0)) + len(ledger.pending(2)) == 11
    # hung-but-alive: heartbeat keeps coming, progress counter stuck -> declared dead after stall_timeout
    for _ in range(3):
        now[0] += 8.0
        hbs[0].tick(); hbs[0].beat(); hbs[2].beat()
    assert wd.status(2)["alive"] is False and "no progress" in wd.status(2)["reason"]
    assert wd.status(0)["alive"] is True


def test_heartbeat_thread_and_timeouts():
    import time as _t
    from copilot_for_consensus_amd.parallel.resilience import Heartbeat, Watchdog, configure_collective_timeouts
    store = dist.HashStore()
    hb = Heartbeat(store, 0, interval=0.05).start()
    _t.sleep(0.2)
    assert Watchdog(store, 1, timeout=1.0).dead_ranks() == []
    hb.stop()
    env = configure_collective_timeouts(120)
    assert os.environ["TORCH_NCCL_ASYNC_ERROR_HANDLING"] == "1" and env["collective_timeout_s"] == 120


def test_argmax_keys_reduce_equals_global_argmax():
    """TP greedy: MAX over the shards' packed (logit, -index) keys is the unsharded argmax,
    negative logits and exact ties (smallest index wins) included."""
    from copilot_for_consensus_amd.models.decoder import argmax_keys
    g = torch.Generator().manual_seed(0)
    for V, tp in ((512, 2), (1000, 4), (96, 8)):
        x = torch.randn(9, V, generator=g) * 5 - 3
        x[0] = -7.5                       # all equal, all negative: index 0
        x[1, V // 2] = x[1, V - 1] = 50.0  # tie across shards: the first one
        x = x.bfloat16()
        Vs = V // tp
        keys = torch.stack([argmax_keys(x[:, r * Vs:(r + 1) * Vs], r * Vs) for r in range(tp)]).max(0).values
        ids = (0xFFFFFFFF - (keys & 0xFFFFFFFF)).to(torch.int32)
        want = torch.tensor([int(torch.nonzero(row == row.max())[0]) for row in x.float()], dtype=torch.int32)
        assert torch.equal(ids, want), (ids, want)


def test_unshard_inverts_shard_and_random_sharded():
    """unshard_weights(shards) is the model whose shard_weights are those shards: exact on a full
    model, and it assembles per-rank random_sharded shards into the model a TP run computes."""
    from copilot_for_consensus_amd.models.decoder import DecoderWeights, get_config
    from copilot_for_consensus_amd.parallel.tp import random_sharded, shard_weights, unshard_weights
    cfg = get_config("tiny-70b-heads")
    full = DecoderWeights.random(cfg, "cpu", seed=2)
    back = unshard_weights([shard_weights(full, r, 4) for r in range(4)])
    for a, b in zip(full.layers, back.layers):
        assert all(torch.equal(a[k], b[k]) for k in a)
    assert torch.equal(full.lm_head, back.lm_head)
    shards = [random_sharded(cfg, "cpu", 9, r, 2) for r in range(2)]
    ref = [{k: v.clone() for k, v in sh.layers[1].items()} for sh in shards]
    u = unshard_weights(shards)
    for r in range(2):
        again = shard_weights(u, r, 2).layers[1]
        assert all(torch.equal(again[k], ref[r][k]) for k in again)
