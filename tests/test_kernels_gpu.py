"""Numerics of every HIP kernel vs the plain-PyTorch fp32 reference (ops/reference.py)."""
import math

import pytest
import torch

from copilot_for_consensus_amd.ops import kernels as K
from copilot_for_consensus_amd.ops import reference as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol, rtol=2e-2):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    assert torch.allclose(a, b, atol=atol, rtol=rtol), f"max abs err {err}"


@pytest.fixture(autouse=True)
def _native_loaded():
    from copilot_for_consensus_amd.ops import _native
    _native.kernels()  # must load: no silent fallback on a GPU box
    torch.manual_seed(0)


@pytest.mark.parametrize("dim", [384, 4096, 8192])
def test_rmsnorm(dim):
    x = torch.randn(37, dim, device=DEV).bfloat16()
    r = torch.randn(37, dim, device=DEV).bfloat16()
    w = (1 + 0.1 * torch.randn(dim, device=DEV)).bfloat16()
    ref_o, ref_r = R.rmsnorm(x.cpu(), w.cpu(), 1e-5, r.cpu())
    rr = r.clone()
    o = K.rmsnorm(x, w, 1e-5, residual=rr)
    _close(rr, ref_r, 1e-2)
    _close(o, ref_o, 3e-2)
    _close(K.rmsnorm(x, w, 1e-5), R.rmsnorm(x.cpu(), w.cpu(), 1e-5)[0], 3e-2)


@pytest.mark.parametrize("dim", [384, 768])
def test_layernorm_variants(dim):
    x = torch.randn(50, dim, device=DEV).bfloat16()
    res = torch.randn(50, dim, device=DEV).bfloat16()
    b = torch.randn(dim, device=DEV).bfloat16()
    g = (1 + 0.1 * torch.randn(dim, device=DEV)).bfloat16()
    be = (0.1 * torch.randn(dim, device=DEV)).bfloat16()
    _close(K.layernorm(x, g, be, 1e-12), R.layernorm(x.cpu(), g.cpu(), be.cpu(), 1e-12), 3e-2)
    _close(K.layernorm(x, g, be, 1e-12, bias=b, residual=res),
           R.layernorm(x.cpu(), g.cpu(), be.cpu(), 1e-12, b.cpu(), res.cpu()), 3e-2)
    V = 1000
    we, pe, te = (torch.randn(n, dim, device=DEV).bfloat16() for n in (V, 512, 2))
    ids = torch.randint(0, V, (50,), device=DEV, dtype=torch.int32)
    pos = torch.randint(0, 512, (50,), device=DEV, dtype=torch.int32)
    _close(K.embed_layernorm(ids, pos, we, pe, te, g, be, 1e-12),
           R.embed_layernorm(ids.cpu(), pos.cpu(), we.cpu(), pe.cpu(), te.cpu(), g.cpu(), be.cpu(), 1e-12), 3e-2)


def _kv_setup(Hkv, D, nblk):
    kc = torch.zeros(nblk, Hkv, R.KV_BLOCK, D, device=DEV).bfloat16()
    vc = torch.zeros(nblk, Hkv, D, R.KV_BLOCK, device=DEV).bfloat16()
    return kc, vc


def test_rope_kv_write():
    Hq, Hkv, D, T = 8, 2, 128, 45
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV).bfloat16()
    pos = torch.randint(0, 3000, (T,), device=DEV, dtype=torch.int32)
    slots = torch.randperm(20 * 32, device=DEV)[:T].to(torch.int32)
    cs = R.rope_cos_sin(4096, D, 1e6, device=DEV)
    kc, vc = _kv_setup(Hkv, D, 20)
    kc2, vc2 = kc.cpu().clone(), vc.cpu().clone()
    q = K.rope_kv_write(qkv, pos, slots, cs, kc, vc, Hq, Hkv, D)
    qr = R.rope_kv_write(qkv.cpu(), pos.cpu(), slots.cpu(), cs.cpu(), kc2, vc2, Hq, Hkv, D)
    _close(q, qr, 2e-2)
    _close(kc, kc2, 2e-2)
    _close(vc, vc2, 1e-6, 0)


def test_rope_kv_write_prefill_runs():
    """The prefill V path (whole-block runs, 16-B stores; partial runs per element) writes exactly
    what the per-token path writes and leaves the other slots of partially written blocks alone."""
    Hq, Hkv, D = 8, 2, 128
    # seq A continues at offset 5 of block 3 (prefix in cache) for 70 tokens; seq B: 40 tokens from 0
    slots = [3 * 32 + 5 + i for i in range(27)] + [9 * 32 + i for i in range(32)] + [4 * 32 + i for i in range(11)]
    slots += [12 * 32 + i for i in range(32)] + [1 * 32 + i for i in range(8)]
    T = len(slots)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV).bfloat16()
    pos = torch.arange(T, device=DEV, dtype=torch.int32)
    cs = R.rope_cos_sin(4096, D, 1e6, device=DEV)
    kc0 = torch.randn(16, Hkv, 32, D, device=DEV).bfloat16()
    vc0 = torch.randn(16, Hkv, D, 32, device=DEV).bfloat16()
    kc1, vc1, kc2, vc2 = kc0.clone(), vc0.clone(), kc0.clone(), vc0.clone()
    sl = torch.tensor(slots, dtype=torch.int32, device=DEV)
    runs_np = K.v_runs(slots)
    assert runs_np[:, 1].tolist() == [27, 32, 11, 32, 8]
    runs = torch.from_numpy(runs_np).to(DEV)
    q1 = K.rope_kv_write(qkv, pos, sl, cs, kc1, vc1, Hq, Hkv, D)
    q2 = K.rope_kv_write(qkv, pos, sl, cs, kc2, vc2, Hq, Hkv, D, runs=runs)
    torch.cuda.synchronize()
    assert torch.equal(q1, q2) and torch.equal(kc1, kc2) and torch.equal(vc1, vc2)
    untouched = [b for b in range(16) if b not in (1, 3, 4, 9, 12)]
    assert torch.equal(vc2[untouched], vc0[untouched])


def _fill_cache(ctx_lens, Hkv, D, extra_blocks=3):
    """Random K/V for every sequence, written through the reference writer; returns tables."""
    tables, nblk = [], 0
    for n in ctx_lens:
        nb = math.ceil(n / 32)
        tables.append(list(range(nblk, nblk + nb)))
        nblk += nb
    nblk += extra_blocks
    perm = torch.randperm(nblk).tolist()  # scatter blocks around the pool
    tables = [[perm[b] for b in t] for t in tables]
    kc = (torch.randn(nblk, Hkv, 32, D)).bfloat16()
    vc = (torch.randn(nblk, Hkv, D, 32)).bfloat16()
    maxb = max(len(t) for t in tables) + 2
    bt = torch.full((len(tables), maxb), 0, dtype=torch.int32)
    for i, t in enumerate(tables):
        bt[i, :len(t)] = torch.tensor(t, dtype=torch.int32)
    return kc, vc, bt


@pytest.mark.parametrize("G", [1, 4, 8])
@pytest.mark.parametrize("part_blocks", [4, 1000, -1, -2, -3, -7, -300])
def test_paged_decode(G, part_blocks):
    Hkv, D = 2, 128
    Hq = Hkv * G
    ctx = [1, 31, 32, 33, 100, 517, 2049, 64]
    kc, vc, bt = _fill_cache(ctx, Hkv, D)
    q = torch.randn(len(ctx), Hq, D).bfloat16()
    cl = torch.tensor(ctx, dtype=torch.int32)
    ref = R.paged_decode_attention(q, kc, vc, bt, cl, 1 / math.sqrt(D))
    out = K.paged_decode_attention(q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), cl.to(DEV), 1 / math.sqrt(D),
                                   part_blocks=part_blocks)
    _close(out, ref, 2e-2)


@pytest.mark.parametrize("shared", [0, 2, 5, 1000])
@pytest.mark.parametrize("fp8", [False, True])
def test_paged_decode_shared_prefix_blocks_read_cached_same_result(shared, fp8):
    """The leading `shared` blocks of every sequence are loaded through the caches (the batch's
    shared prefix), the rest nontemporal: a cache-policy change only -- bit-identical output."""
    Hkv, D, G = 8, 128, 4
    ctx = [300, 31, 2049, 64, 700] * 8          # 40 rows: the nontemporal path (B >= 32)
    kc, vc, bt = _fill_cache(ctx, Hkv, D)
    bt[:, :2] = bt[0, :2]                        # two physical prefix blocks shared by every row
    kw = {}
    if fp8:
        kc, vc = (kc.float() / 0.5).clamp(-448, 448).to(F8), (vc.float() / 0.25).clamp(-448, 448).to(F8)
        kw = dict(k_scale=0.5, v_scale=0.25)
    q = torch.randn(len(ctx), Hkv * G, D).bfloat16().to(DEV)
    args = (q, kc.to(DEV), vc.to(DEV), bt.to(DEV), torch.tensor(ctx, dtype=torch.int32, device=DEV), 1 / math.sqrt(D))
    a = K.paged_decode_attention(*args, part_blocks=-1, **kw)
    b = K.paged_decode_attention(*args, part_blocks=-1, shared_blocks=torch.tensor([shared], dtype=torch.int32,
                                                                                   device=DEV), **kw)
    assert torch.equal(a, b)


@pytest.mark.parametrize("G", [1, 4])
@pytest.mark.parametrize("part_blocks", [4, -1, -3])
@pytest.mark.parametrize("window", [1, 33, 100])
def test_paged_decode_sliding_window(G, part_blocks, window):
    Hkv, D = 2, 128
    Hq = Hkv * G
    ctx = [1, 31, 32, 33, 100, 517, 2049, 64]
    kc, vc, bt = _fill_cache(ctx, Hkv, D)
    q = torch.randn(len(ctx), Hq, D).bfloat16()
    cl = torch.tensor(ctx, dtype=torch.int32)
    ref = R.paged_decode_attention(q, kc, vc, bt, cl, 1 / math.sqrt(D), window=window)
    out = K.paged_decode_attention(q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), cl.to(DEV), 1 / math.sqrt(D),
                                   part_blocks=part_blocks, window=window)
    _close(out, ref, 2e-2)


@pytest.mark.parametrize("G", [1, 4, 8])
@pytest.mark.parametrize("window", [1, 40, 100])
def test_prefill_attention_sliding_window(G, window):
    Hkv, D = 2, 128
    Hq = Hkv * G
    seqs = [(1, 1), (17, 17), (200, 200), (70, 300), (129, 1000), (600, 600)]
    kc, vc, bt = _fill_cache([c for _, c in seqs], Hkv, D)
    cu = [0]
    for qn, _ in seqs:
        cu.append(cu[-1] + qn)
    q = torch.randn(cu[-1], Hq, D).bfloat16()
    cu_t = torch.tensor(cu, dtype=torch.int32)
    cl = torch.tensor([c for _, c in seqs], dtype=torch.int32)
    ref = R.prefill_attention(q, kc, vc, bt, cu_t, cl, 1 / math.sqrt(D), window=window)
    out = K.prefill_attention(q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), cu_t.to(DEV), cl.to(DEV),
                              1 / math.sqrt(D), window=window)
    _close(out, ref, 2e-2)


@pytest.mark.parametrize("G", [1, 2, 4, 8])
def test_prefill_attention(G):
    Hkv, D = 2, 128
    Hq = Hkv * G
    # (q_len, ctx_len): fresh prompts and chunked continuation (ctx > q_len), tile edges of every
    # G's tile height (256 / G rows) and a long prompt
    seqs = [(1, 1), (17, 17), (64, 64), (200, 200), (70, 300), (129, 1000), (256, 256), (33, 33), (1100, 1100)]
    kc, vc, bt = _fill_cache([c for _, c in seqs], Hkv, D)
    cu = [0]
    for qn, _ in seqs:
        cu.append(cu[-1] + qn)
    q = torch.randn(cu[-1], Hq, D).bfloat16()
    cu_t = torch.tensor(cu, dtype=torch.int32)
    cl = torch.tensor([c for _, c in seqs], dtype=torch.int32)
    ref = R.prefill_attention(q, kc, vc, bt, cu_t, cl, 1 / math.sqrt(D))
    out = K.prefill_attention(q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), cu_t.to(DEV), cl.to(DEV),
                              1 / math.sqrt(D))
    _close(out, ref, 2e-2)


@pytest.mark.parametrize("D", [32, 64])
def test_encoder_attention(D):
    H = 4
    lens = [1, 5, 31, 64, 130, 256]
    cu = [0]
    for n in lens:
        cu.append(cu[-1] + n)
    qkv = torch.randn(cu[-1], 3 * H * D).bfloat16()
    cu_t = torch.tensor(cu, dtype=torch.int32)
    ref = R.encoder_attention(qkv, cu_t, H, D, 1 / math.sqrt(D))
    out = K.encoder_attention(qkv.to(DEV), cu_t.to(DEV), H, D, 1 / math.sqrt(D), max(lens))
    _close(out, ref, 2e-2)


def test_silu_mul_and_gelu():
    gu = torch.randn(33, 2 * 1536, device=DEV).bfloat16()
    _close(K.silu_mul(gu), R.silu_mul(gu.cpu()), 2e-2)
    x = torch.randn(33, 1536, device=DEV).bfloat16()
    b = torch.randn(1536, device=DEV).bfloat16()
    _close(K.bias_gelu(x, b), R.bias_gelu(x.cpu(), b.cpu()), 2e-2)


def test_embedding_and_greedy_sample():
    table = torch.randn(1000, 256, device=DEV).bfloat16()
    ids = torch.randint(0, 1000, (17,), device=DEV, dtype=torch.int32)
    _close(K.embedding(table, ids), table.cpu()[ids.cpu().long()], 0, 0)
    logits = torch.randn(9, 32000, device=DEV).bfloat16()
    out = torch.empty(9, dtype=torch.int32, device=DEV)
    K.sample(logits, out)
    assert out.cpu().tolist() == R.sample_greedy(logits.cpu()).tolist()


def test_gumbel_sampling_distribution():
    # 4-way categorical at T=1: empirical frequencies match softmax
    probs = torch.tensor([0.1, 0.2, 0.3, 0.4])
    logits = probs.log().repeat(4096, 1).bfloat16().to(DEV)
    out = torch.empty(4096, dtype=torch.int32, device=DEV)
    step = torch.tensor([3], dtype=torch.int32, device=DEV)
    K.sample(logits, out, temperature=1.0, seed=11, step=step)
    freq = torch.bincount(out.cpu().long(), minlength=4).float() / 4096
    assert (freq - probs).abs().max() < 0.03, freq


@pytest.mark.parametrize("N,nq,k,metric", [(5000, 1, 10, "dot"), (3000, 16, 100, "l2"), (1024, 7, 1, "dot"),
                                           (70, 3, 20, "l2"), (40000, 16, 256, "dot"), (100000, 16, 150, "dot"),
                                           (70000, 2, 33, "l2"), (50000, 5, 256, "l2")])
def test_knn_topk_fused_matches_reference(N, nq, k, metric):
    """Fused scan + per-chunk radix select (+ candidate merge) vs torch.topk of fp32 scores of the
    same bf16 rows; dead rows and a row window excluded."""
    X = torch.nn.functional.normalize(torch.randn(N, 384, device=DEV), dim=1).bfloat16()
    Q = torch.nn.functional.normalize(torch.randn(nq, 384, device=DEV), dim=1).bfloat16()
    alive = torch.rand(N, device=DEV) > 0.1
    xn2 = X.float().pow(2).sum(1) if metric == "l2" else None
    qn2 = Q.float().pow(2).sum(1) if metric == "l2" else None
    lo = N // 7
    v, i = K.knn_topk(X, Q, k, xn2, qn2, alive, row_lo=lo, N=N)
    ref = R.knn_scores(X[lo:].float(), Q.float(), None if xn2 is None else xn2[lo:], qn2)
    ref = ref.masked_fill(~alive[lo:][None], float("-inf"))
    rv, ri = torch.topk(ref, min(k, N - lo), dim=1)
    assert v.shape == rv.shape
    assert torch.allclose(v, rv, atol=2e-3, rtol=1e-3), (v[:, :5], rv[:, :5])
    # the returned rows really have those scores
    got = torch.gather(ref, 1, (i - lo).clamp_min(0))
    assert torch.allclose(got, v, atol=2e-3, rtol=1e-3)
    assert bool((i >= lo).all()) and bool(alive[i].all())


def test_ivf_gpu_matches_flat_when_every_list_is_probed_and_recall():
    from copilot_for_consensus_amd.vectorstore import HipFlatIndex, HipIVFIndex
    g = torch.Generator(device=DEV).manual_seed(3)
    C = torch.nn.functional.normalize(torch.randn(40, 384, device=DEV, generator=g), dim=1)
    X = C[torch.randint(0, 40, (20000,), device=DEV, generator=g)] + 0.05 * torch.randn(20000, 384, device=DEV, generator=g)
    ids = [f"v{j}" for j in range(20000)]
    flat = HipFlatIndex(384, device=DEV, capacity=1 << 15)
    flat.add_embeddings(ids, X)
    ivf = HipIVFIndex(384, "cosine", nlist=32, nprobe=32, device=DEV, capacity=1 << 15)
    ivf.add_embeddings(ids, X)
    ivf.train(iters=6)
    Q = C[:16] + 0.05 * torch.randn(16, 384, device=DEV, generator=g)
    a = [[r.id for r in row] for row in ivf.query_batch(Q, top_k=10)]
    b = [[r.id for r in row] for row in flat.query_batch(Q, top_k=10)]
    assert a == b                                   # all lists probed: exactly the flat result
    ivf.nprobe = 4
    a = [[r.id for r in row] for row in ivf.query_batch(Q, top_k=10)]
    recall = sum(len(set(x) & set(y)) for x, y in zip(a, b)) / 160
    assert recall >= 0.95, recall
    # rows added after training (the unsorted tail) are found
    ivf.add_embedding("late", Q[0])
    assert ivf.query(Q[0], top_k=1)[0].id == "late"
    ivf.delete("late")
    assert ivf.query(Q[0], top_k=1)[0].id != "late"


def test_knn_scores_and_topk():
    N, dim = 50_000, 384
    X = torch.randn(N, dim, device=DEV).bfloat16()
    Xn = K.l2_normalize(X)
    _close(Xn[:100], R.l2_normalize(X[:100].cpu())[0], 1e-2)
    Q = K.l2_normalize(torch.randn(5, dim, device=DEV).bfloat16())
    s = K.knn_scores(Xn, Q)
    _close(s[:, :2000], R.knn_scores(Xn[:2000].cpu(), Q.cpu()), 1e-2)
    v, i = K.topk(s, 150)
    rv, ri = torch.topk(s, 150, dim=1)
    _close(v, rv, 1e-6, 0)
    # ids may differ only among exact ties
    assert (s.gather(1, i.to(DEV)) == v.to(DEV)).all()
    # squared-L2 mode
    n2 = torch.empty(N, device=DEV)
    K.l2_normalize(X, norms2=n2)
    qn2 = Q.float().pow(2).sum(1)
    s2 = K.knn_scores(X, Q, n2, qn2)
    _close(s2[:, :1000], R.knn_scores(X[:1000].cpu(), Q.cpu(), n2[:1000].cpu(), qn2.cpu()), 0.5, 1e-2)


def test_pool():
    lens = [3, 1, 40]
    cu = torch.tensor([0, 3, 4, 44], dtype=torch.int32)
    h = torch.randn(44, 384).bfloat16()
    for mode in ("mean", "cls"):
        _close(K.pool(h.to(DEV), cu.to(DEV), mode, True), R.pool(h, cu, mode, True), 1e-3)
    del lens


def test_silu_mul_interleaved():
    gu = torch.randn(33, 2 * 512, device=DEV).bfloat16()
    _close(K.silu_mul(gu, interleaved=True), R.silu_mul_interleaved(gu.cpu()), 2e-2)
    w = torch.randn(2 * 64, 16)
    assert torch.equal(R.deinterleave_gate_up(R.interleave_gate_up(w)), w)


def _ref_linear(x, w):
    return (x.float() @ w.float().T).cpu()


@pytest.mark.parametrize("M,N,Kd,split,bn", [(5, 6144, 4096, None, None), (8, 4096, 4096, 8, 64),
                                            (77, 1024, 512, 2, 128), (128, 4096, 14336, None, None),
                                            (128, 6144, 4096, 4, 96), (128, 28672, 512, 1, 112),
                                            (200, 512, 1024, 1, 128), (256, 768, 1024, 3, 96),
                                            (128, 32000, 4096, 1, 128), (300, 640, 256, 1, 64), (64, 448, 320, 5, 112)])
def test_dgemm_linear(M, N, Kd, split, bn):
    """Hand-written decode GEMM vs fp32 x @ w^T: every row tile (64 / 128 / 256, M > 256 over
    grid.y), every W tile width, split-K slabs + reduce, uneven K slices."""
    x = torch.randn(M, Kd, device=DEV).bfloat16()
    w = (torch.randn(N, Kd, device=DEV) * 0.02).bfloat16()
    y = K.dgemm_linear(x, w, split=split, bn=bn)
    _close(y, _ref_linear(x, w), 3e-2)


def test_dgemm_asymmetric_exact():
    """Small-integer operands (exact in bf16 and fp32): the output must match bit for bit, which
    catches any row/column or k-order mix-up an all-random check could hide."""
    M, N, Kd = 128, 256, 512
    x = torch.randint(-3, 4, (M, Kd), device=DEV).bfloat16()
    w = torch.randint(-2, 3, (N, Kd), device=DEV).bfloat16()
    w[:, :7] += torch.arange(N, device=DEV).bfloat16().unsqueeze(1) % 5   # asymmetric in n
    ref = (x.float() @ w.float().T)
    for bn in K.DGEMM_BNS:
        if N % bn == 0:
            part = K.dgemm(x, w, "part", 2, bn=bn)
            assert torch.equal(part.sum(0), ref), bn


@pytest.mark.parametrize("M,split", [(128, None), (5, None), (64, None), (128, 2), (130, 4), (256, None)])
def test_dgemm_swiglu(M, split):
    F, Kd = 1024, 512
    x = torch.randn(M, Kd, device=DEV).bfloat16()
    gu = (torch.randn(2 * F, Kd, device=DEV) * 0.05).bfloat16()
    wi = R.interleave_gate_up(gu)
    ref = R.silu_mul(_ref_linear(x, gu).bfloat16())
    _close(K.dgemm_swiglu(x, wi, split=split), ref, 3e-2)


@pytest.mark.parametrize("M,N,Kd,split", [(128, 4096, 4096, None), (5, 256, 512, 1), (128, 4096, 14336, 8),
                                         (256, 1024, 1024, None)])
def test_dgemm_residual_rmsnorm(M, N, Kd, split):
    x = torch.randn(M, Kd, device=DEV).bfloat16()
    w = (torch.randn(N, Kd, device=DEV) * 0.02).bfloat16()
    r = torch.randn(M, N, device=DEV).bfloat16()
    nw = (1 + 0.1 * torch.randn(N, device=DEV)).bfloat16()
    ref_o, ref_r = R.rmsnorm(_ref_linear(x, w).bfloat16(), nw.cpu(), 1e-5, r.cpu())
    rr = r.clone()
    o = K.dgemm_residual_rmsnorm(x, w, rr, nw, 1e-5, split=split)
    _close(rr, ref_r, 3e-2)
    _close(o, ref_o, 5e-2)


@pytest.mark.parametrize("bn", [64, 96, 112, 128])
def test_dgemm_pack_matches_reference_layout(bn):
    """The GPU pack kernel writes exactly the layout reference.pack_dgemm_weight describes."""
    N, Kd = (1280 if bn == 128 else 1344), 320
    w = torch.randn(N, Kd, device=DEV).bfloat16()
    pw = K.pack_dgemm_weight(w, bn)
    assert torch.equal(pw.data.cpu(), R.pack_dgemm_weight(w.cpu(), bn).reshape(-1))
    assert torch.equal(K._rowmajor(pw).cpu(), w.cpu())


@pytest.mark.parametrize("M,N,Kd,split,bn", [(128, 6144, 4096, None, 128), (5, 4096, 4096, 4, 64),
                                            (77, 1024, 512, 2, 128), (200, 512, 1024, 1, 128),
                                            (256, 768, 1024, 3, 96), (128, 28672, 512, 1, 112),
                                            (300, 640, 256, 1, 64), (64, 448, 320, 5, 112)])
def test_dgemm_packed_linear(M, N, Kd, split, bn):
    """Fragment-packed weights (buffer-load stream) vs fp32 x @ w^T, every row tile and W width."""
    x = torch.randn(M, Kd, device=DEV).bfloat16()
    w = (torch.randn(N, Kd, device=DEV) * 0.02).bfloat16()
    y = K.dgemm_linear(x, K.pack_dgemm_weight(w, bn), split=split)
    _close(y, _ref_linear(x, w), 3e-2)


def test_dgemm_packed_exact():
    M, N, Kd = 128, 448, 512
    x = torch.randint(-3, 4, (M, Kd), device=DEV).bfloat16()
    w = torch.randint(-2, 3, (N, Kd), device=DEV).bfloat16()
    w[:, :7] += torch.arange(N, device=DEV).bfloat16().unsqueeze(1) % 5
    ref = (x.float() @ w.float().T)
    for bn in K.DGEMM_BNS:
        if N % bn == 0:
            for split in (1, 3):
                part = K.dgemm(x, K.pack_dgemm_weight(w, bn), "part", split)
                assert torch.equal(part.sum(0), ref), (bn, split)


@pytest.mark.parametrize("M,N,Kd,split", [(128, 6144, 4096, 4), (128, 4096, 14336, 8), (77, 448, 512, 3)])
def test_dgemm_write_through_slabs_equal_plain(M, N, Kd, split, monkeypatch):
    """DG_PART_WT (sc1 slab stores, CFC_DGEMM_SLAB_WT=1) writes the same fp32 partials as the plain
    slab epilogue, bit for bit, and they sum to the fp32 reference."""
    x = torch.randn(M, Kd, device=DEV).bfloat16()
    w = (torch.randn(N, Kd, device=DEV) * 0.02).bfloat16()
    pw = K.pack_dgemm_weight(w)
    monkeypatch.setattr(K, "DGEMM_PART_MODE", 0)
    plain = K.dgemm(x, pw, "part", split).clone()
    monkeypatch.setattr(K, "DGEMM_PART_MODE", 3)
    wt = K.dgemm(x, pw, "part", split).clone()
    assert torch.equal(plain, wt)
    _close(wt.sum(0).bfloat16(), _ref_linear(x, w), 3e-2)


@pytest.mark.parametrize("M,split", [(128, None), (5, None), (128, 2), (256, None)])
def test_dgemm_packed_swiglu_and_norm(M, split):
    F, Kd = 1024, 512
    x = torch.randn(M, Kd, device=DEV).bfloat16()
    gu = (torch.randn(2 * F, Kd, device=DEV) * 0.05).bfloat16()
    ref = R.silu_mul(_ref_linear(x, gu).bfloat16())
    pw = K.pack_dgemm_weight(R.interleave_gate_up(gu), swiglu=True, m=M)
    _close(K.dgemm_swiglu(x, pw, split=split), ref, 3e-2)
    w = (torch.randn(Kd, F, device=DEV) * 0.02).bfloat16()
    a = torch.randn(M, F, device=DEV).bfloat16()
    r = torch.randn(M, Kd, device=DEV).bfloat16()
    nw = (1 + 0.1 * torch.randn(Kd, device=DEV)).bfloat16()
    ref_o, ref_r = R.rmsnorm(_ref_linear(a, w).bfloat16(), nw.cpu(), 1e-5, r.cpu())
    rr = r.clone()
    o = K.dgemm_residual_rmsnorm(a, K.pack_dgemm_weight(w, m=M), rr, nw, 1e-5, split=split)
    _close(rr, ref_r, 3e-2)
    _close(o, ref_o, 5e-2)


@pytest.mark.parametrize("M,N,Kd,epi", [(512, 512, 256, "bf16"), (300, 1152, 384, "bias"), (257, 1536, 384, "bias_gelu"),
                                       (1000, 768, 1536, "bf16"), (129, 2048, 512, "swiglu"), (64, 320, 128, "bf16"),
                                       (2048, 4096, 1024, "bf16"), (513, 640, 4096, "swiglu")])
@pytest.mark.parametrize("variant", ["ring5", "ring4", "stage2", "pp", "w4", "pps"])
def test_pgemm(M, N, Kd, epi, variant):
    """Prefill / encoder GEMM with its fused epilogue vs the fp32 reference of the same op: edge
    tiles in M and N (rows/cols past the edge never stored), bias, bias+GELU, SwiGLU."""
    x = (torch.rand(M, Kd, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(N, Kd, device=DEV) * 2 - 1) / Kd ** 0.5).bfloat16()
    b = (torch.rand(N, device=DEV) * 0.2 - 0.1).bfloat16()
    ref = _ref_linear(x, w)
    if epi in ("bias", "bias_gelu"):
        ref = ref + b.float().cpu()
    if epi == "bias_gelu":
        ref = torch.nn.functional.gelu(ref)
    if epi == "swiglu":
        gu = R.deinterleave_gate_up(w.cpu())      # the same weights in [gate; up] order
        ref = R.silu_mul(_ref_linear(x, gu.to(DEV)).bfloat16()).float()
    out = torch.full((M, N // 2 if epi == "swiglu" else N), float("nan"), device=DEV).bfloat16()
    y = K.pgemm(x, w, epi, bias=b, out=out, variant=variant)
    _close(y, ref, 3e-2)


@pytest.mark.parametrize("variant", ["ring5", "ring4", "stage2", "pp", "w4", "pps"])
def test_pgemm_exact_and_strided_out(variant):
    """Small-integer operands: bit-exact; output written into a wider buffer (ldo > N) leaves the
    other columns untouched."""
    M, N, Kd = 300, 320, 192
    x = torch.randint(-3, 4, (M, Kd), device=DEV).bfloat16()
    w = torch.randint(-2, 3, (N, Kd), device=DEV).bfloat16()
    w[:, :5] += torch.arange(N, device=DEV).bfloat16().unsqueeze(1) % 7
    buf = torch.zeros(M, N + 64, device=DEV).bfloat16()
    K.pgemm(x, w, out=buf[:, :N], variant=variant)
    assert torch.equal(buf[:, :N].float(), x.float() @ w.float().T)
    assert torch.equal(buf[:, N:], torch.zeros_like(buf[:, N:]))


@pytest.mark.parametrize("M,N,Kd,epi,bn", [(512, 768, 256, "bf16", 64), (300, 1152, 384, "bias", 96),
                                          (257, 1536, 448, "bias_gelu", 128), (129, 2240, 512, "swiglu", 112),
                                          (1000, 6144, 1024, "bf16", 96), (513, 1792, 2048, "swiglu", 64)])
@pytest.mark.parametrize("variant", ["pp", "w4", "pps", "ppp"])
def test_pgemm_packed_weight(M, N, Kd, epi, bn, variant):
    """The ping-pong prefill GEMM reading the decode GEMM's fragment-packed weight (one weight copy
    for prefill and decode) vs the fp32 reference, for every packing width bn; bit-identical to the
    same kernel on the row-major weight."""
    x = (torch.rand(M, Kd, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(N, Kd, device=DEV) * 2 - 1) / Kd ** 0.5).bfloat16()
    b = (torch.rand(N, device=DEV) * 0.2 - 0.1).bfloat16()
    ref = _ref_linear(x, w)
    if epi in ("bias", "bias_gelu"):
        ref = ref + b.float().cpu()
    if epi == "bias_gelu":
        ref = torch.nn.functional.gelu(ref)
    if epi == "swiglu":
        ref = R.silu_mul(_ref_linear(x, R.deinterleave_gate_up(w.cpu()).to(DEV)).bfloat16()).float()
    pw = K.pack_dgemm_weight(w, bn=bn)
    y = K.pgemm(x, pw, epi, bias=b, variant=variant)
    _close(y, ref, 3e-2)
    assert torch.equal(y, K.pgemm(x, w, epi, bias=b, variant=variant))


@pytest.mark.parametrize("variant", ["pp", "w4", "pps", "ppp"])
def test_pgemm_packed_exact(variant):
    """Small-integer operands through the packed weight: bit-exact."""
    M, N, Kd = 700, 576, 320
    x = torch.randint(-3, 4, (M, Kd), device=DEV).bfloat16()
    w = torch.randint(-2, 3, (N, Kd), device=DEV).bfloat16()
    w[:, :5] += torch.arange(N, device=DEV).bfloat16().unsqueeze(1) % 7
    y = K.pgemm(x, K.pack_dgemm_weight(w, bn=96), variant=variant)
    assert torch.equal(y.float(), x.float() @ w.float().T)


@pytest.mark.parametrize("epi", ["bf16", "swiglu"])
@pytest.mark.parametrize("M", [300, 512, 1000])
def test_pgemm_staged_epilogue_bit_identical(epi, M):
    """The LDS-staged epilogue (variant pps) writes exactly the bytes of the register epilogue (pp),
    partial row tiles and a strided output included; nothing outside the output columns."""
    N, Kd = 1536 if epi == "swiglu" else 768, 512
    x = (torch.rand(M, Kd, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(N, Kd, device=DEV) * 2 - 1) / Kd ** 0.5).bfloat16()
    pw = K.pack_dgemm_weight(w, swiglu=epi == "swiglu")
    oc = N // 2 if epi == "swiglu" else N
    a = torch.full((M, oc + 64), 7.0, device=DEV).bfloat16()
    b = a.clone()
    K.pgemm(x, pw, epi, out=a[:, :oc], variant="pp")
    K.pgemm(x, pw, epi, out=b[:, :oc], variant="pps")
    assert torch.equal(a, b)
    assert bool((b[:, oc:] == 7.0).all())


@pytest.mark.parametrize("epi,M,N,Kd", [("bf16", 8192, 8192, 256), ("bf16", 4100, 4352, 448),
                                       ("swiglu", 4097, 7168, 320), ("swiglu", 16384, 2240, 128),
                                       ("bf16", 300, 768, 64)])
def test_pgemm_persistent_bit_identical(epi, M, N, Kd):
    """The persistent ping-pong kernel (variant ppp: one workgroup per CU walking the tiles, the DMA
    stream running on across tile boundaries, epilogue stores left in flight) writes exactly the
    bytes of the one-tile-per-workgroup kernel (pp): up to 4 tiles per workgroup, odd K-tile
    counts (the LDS slot parity flips per tile), edge tiles in M and N (the drained epilogue),
    a strided output, and K = 64 (the non-persistent fallback)."""
    x = (torch.rand(M, Kd, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(N, Kd, device=DEV) * 2 - 1) / Kd ** 0.5).bfloat16()
    pw = K.pack_dgemm_weight(w, swiglu=epi == "swiglu")
    oc = N // 2 if epi == "swiglu" else N
    a = torch.full((M, oc + 64), 7.0, device=DEV).bfloat16()
    b = a.clone()
    K.pgemm(x, pw, epi, out=a[:, :oc], variant="pp")
    K.pgemm(x, pw, epi, out=b[:, :oc], variant="ppp")
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert bool((b[:, oc:] == 7.0).all())


@pytest.mark.parametrize("epi,M,N,Kd", [("bf16", 4100, 4352, 448), ("swiglu", 2049, 7168, 256)])
def test_pgemm_persistent_tile_orders_and_direct_stores_bit_identical(epi, M, N, Kd):
    """The persistent kernel through its probe entry: every tile-order group gm (M-tiles per N
    sweep) and the register-direct epilogue stores write the same bytes as the one-tile kernel."""
    x = (torch.rand(M, Kd, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(N, Kd, device=DEV) * 2 - 1) / Kd ** 0.5).bfloat16()
    pw = K.pack_dgemm_weight(w, swiglu=epi == "swiglu")
    oc = N // 2 if epi == "swiglu" else N
    ref = K.pgemm(x, pw, epi, variant="pp")
    for gm in (1, 2, 4, 8, 16):
        for direct in (False, True):
            y = torch.full((M, oc), 7.0, device=DEV).bfloat16()
            K.check(K.kernels().cfc_pgemm_ppp_probe(x.data_ptr(), pw.data.data_ptr(), y.data_ptr(), M, N, Kd,
                                                   (3 if epi == "swiglu" else 0) | (16 if direct else 0), oc,
                                                   pw.bn // 16, gm, K._stream(x)), "cfc_pgemm_ppp_probe")
            torch.cuda.synchronize()
            assert torch.equal(y, ref), (gm, direct)


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("N,Kd,bn", [(6144, 4096, 96), (1024, 1536, 64), (2240, 512, 112), (768, 448 + 64, 128)])
def test_gemv_packed_weight(M, N, Kd, bn):
    """The B <= 4 GEMV over the fragment-packed weight (packed-only decode) vs the fp32 reference and
    vs the row-major GEMV: fp32, bf16 and SwiGLU epilogues."""
    x = (torch.rand(M, Kd, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(N, Kd, device=DEV) * 2 - 1) / Kd ** 0.5).bfloat16()
    pw = K.pack_dgemm_weight(w, bn=bn)
    ref = _ref_linear(x, w)
    _close(K.gemv(x, pw, "f32"), ref, 1e-3)
    _close(K.gemv(x, pw, "bf16"), ref, 1e-2)
    torch.testing.assert_close(K.gemv(x, pw, "f32"), K.gemv(x, w, "f32"), rtol=1e-4, atol=1e-4)
    if N % 16 == 0:
        want = R.silu_mul(_ref_linear(x, R.deinterleave_gate_up(w.cpu()).to(DEV)).bfloat16()).float()
        _close(K.gemv(x, pw, "swiglu"), want, 3e-2)


@pytest.mark.parametrize("split", [1, 2, 5, 32])
@pytest.mark.parametrize("M,waves", [(1, 4), (1, 16), (3, 8)])
def test_gemv_packed_slabs(split, M, waves):
    """The packed GEMV's k-slice slab form (split 1 .. K / 32): the slabs sum to the product, the
    residual + RMSNorm reduce over them matches the row-major GEMV route, and repeated launches
    are bit-identical."""
    N, Kd, bn = 896, 1024, 112
    x = (torch.rand(M, Kd, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(N, Kd, device=DEV) * 2 - 1) / Kd ** 0.5).bfloat16()
    pw = K.pack_dgemm_weight(w, bn=bn)
    part = K.gemv_part(x, pw, split, waves).clone()
    assert part.shape == (split, M, N)
    _close(part.sum(0), _ref_linear(x, w), 1e-3)
    assert torch.equal(part, K.gemv_part(x, pw, split, waves))
    for epi in ("f32", "bf16", "swiglu"):      # split-1 epilogues at this wave count
        want = K.gemv(x, w, epi).float()
        torch.testing.assert_close(K.gemv(x, pw, epi, waves=waves).float(), want, rtol=2e-2, atol=2e-2)
    norm = torch.rand(N, device=DEV).bfloat16()
    r1 = (torch.rand(M, N, device=DEV) * 2 - 1).bfloat16()
    r2 = r1.clone()
    o1 = K.gemv_residual_rmsnorm(x, pw, r1, norm, 1e-5)
    o2 = K.gemv_residual_rmsnorm(x, w, r2, norm, 1e-5)
    torch.testing.assert_close(r1.float(), r2.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(o1.float(), o2.float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("N,Kd,bn,s_in", [(896, 5120, 112, 6), (768, 1024, 128, 1), (1536, 2048, 96, 8)])
def test_gemv_norm_equals_reduce_then_gemv(M, N, Kd, bn, s_in):
    """The residual + RMSNorm folded into the packed GEMV's prologue == splitk_residual_rmsnorm then
    the GEMV, bit for bit: the new residual, the slabs (split 1 and > 1) and the bf16 / SwiGLU
    epilogues; res_in is left untouched."""
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N)
    part = torch.randn(s_in, M, Kd, device=DEV, generator=g)
    res = torch.randn(M, Kd, device=DEV, generator=g).bfloat16()
    norm = (torch.rand(Kd, device=DEV, generator=g) + 0.5).bfloat16()
    w = ((torch.rand(N, Kd, device=DEV, generator=g) * 2 - 1) / Kd ** 0.5).bfloat16()
    pw = K.pack_dgemm_weight(w, bn=bn)
    r1 = res.clone()
    x = K.splitk_residual_rmsnorm(part, r1, norm, 1e-5)
    for waves in (4, 8):
        for split in (1, 3):
            r_in, r_out = res.clone(), torch.empty_like(res)
            got = K.gemv_norm(part, r_in, r_out, norm, 1e-5, pw, split=split, waves=waves).clone()
            assert torch.equal(r_out, r1) and torch.equal(r_in, res)
            assert torch.equal(got, K.gemv_part(x, pw, split, waves))
        for epi in ("bf16", "swiglu"):
            r_in, r_out = res.clone(), torch.empty_like(res)
            got = K.gemv_norm(part, r_in, r_out, norm, 1e-5, pw, epi, waves=waves)
            assert torch.equal(got, K.gemv(x, pw, epi, waves=waves)) and torch.equal(r_out, r1)
    with pytest.raises(ValueError):
        K.gemv_norm(part, res, res, norm, 1e-5, pw)


@pytest.mark.parametrize("split", [1, 3, 4])
def test_rope_kv_write_from_splitk_slabs_matches_reduce_then_rope(split):
    """rope_kv_write_part == splitk_reduce -> rope_kv_write, bit for bit (q, K cache, V cache)."""
    Hq, Hkv, D, T, nblk = 8, 2, 128, 5, 4
    N = (Hq + 2 * Hkv) * D
    part = torch.randn(split, T, N, device=DEV)
    cs = R.rope_cos_sin(256, D, 1e4, device=DEV)
    pos = torch.tensor([0, 3, 17, 100, 255], dtype=torch.int32, device=DEV)
    slots = torch.tensor([0, 5, 40, 63, 90], dtype=torch.int32, device=DEV)

    def caches():
        return (torch.zeros(nblk, Hkv, 32, D, device=DEV).bfloat16(), torch.zeros(nblk, Hkv, D, 32, device=DEV).bfloat16())
    k1, v1 = caches()
    q1 = K.rope_kv_write(K.splitk_reduce(part), pos, slots, cs, k1, v1, Hq, Hkv, D)
    k2, v2 = caches()
    q2 = K.rope_kv_write_part(part, pos, slots, cs, k2, v2, Hq, Hkv, D)
    assert torch.equal(q1, q2) and torch.equal(k1, k2) and torch.equal(v1, v2)
    # every V store mode (CFC_KV_VSTORE: plain, write-through, nontemporal) writes the same bytes
    orig = K._KV_VSTORE["mode"]
    try:
        for mode in (0, 1, 2):
            K.set_kv_vstore_mode(mode)
            k3, v3 = caches()
            q3 = K.rope_kv_write_part(part, pos, slots, cs, k3, v3, Hq, Hkv, D)
            k4, v4 = caches()
            K.rope_kv_write(K.splitk_reduce(part), pos, slots, cs, k4, v4, Hq, Hkv, D)
            assert torch.equal(q1, q3) and torch.equal(k1, k3) and torch.equal(v1, v3), mode
            assert torch.equal(k1, k4) and torch.equal(v1, v4), mode
    finally:
        K.set_kv_vstore_mode(orig)


@pytest.mark.parametrize("G", [1, 4, 8])
@pytest.mark.parametrize("part_blocks", [4, -1, -3])
@pytest.mark.parametrize("src", ["bf16", "slabs3"])
@pytest.mark.parametrize("kv", ["bf16", "fp8"])
@pytest.mark.parametrize("window", [0, 100])
def test_paged_decode_rope_attention_fused_matches_two_kernels(G, part_blocks, src, kv, window):
    """RoPE + KV write in the decode attention's prologue == rope_kv_write(_part) -> paged_decode_attention,
    bit for bit: output, K cache and V cache (one row with slot -1 writes nothing); and against the
    fp32 reference of the same step."""
    Hkv, D = 2, 128
    Hq = Hkv * G
    ctx = [1, 31, 32, 33, 100, 517, 2049, 64]
    kc, vc, bt = _fill_cache(ctx, Hkv, D)
    ks, vs = (0.5, 0.25) if kv == "fp8" else (1.0, 1.0)
    if kv == "fp8":
        kc = (kc.float() / ks).clamp(-448, 448).to(F8)
        vc = (vc.float() / vs).clamp(-448, 448).to(F8)
    B, N = len(ctx), (Hq + 2 * Hkv) * D
    pos = torch.tensor([n - 1 for n in ctx], dtype=torch.int32)
    slots = torch.tensor([int(bt[b, (n - 1) // 32]) * 32 + (n - 1) % 32 for b, n in enumerate(ctx)], dtype=torch.int32)
    slots[3] = -1
    cs = R.rope_cos_sin(4096, D, 1e6, device=DEV)
    if src == "bf16":
        qkv = torch.randn(B, N, device=DEV).bfloat16()
    else:
        qkv = torch.randn(3, B, N, device=DEV)
    args = (pos.to(DEV), slots.to(DEV), cs)
    bt_d, cl = bt.to(DEV), torch.tensor(ctx, dtype=torch.int32, device=DEV)
    k1, v1, k2, v2 = kc.to(DEV), vc.to(DEV), kc.to(DEV), vc.to(DEV)
    if src == "bf16":
        q = K.rope_kv_write(qkv, *args, k1, v1, Hq, Hkv, D, k_scale=ks, v_scale=vs)
    else:
        q = K.rope_kv_write_part(qkv, *args, k1, v1, Hq, Hkv, D, k_scale=ks, v_scale=vs)
    o1 = K.paged_decode_attention(q, k1, v1, bt_d, cl, 1 / math.sqrt(D), part_blocks=part_blocks, window=window,
                                  k_scale=ks, v_scale=vs)
    o2 = K.paged_decode_rope_attention(qkv, *args, k2, v2, bt_d, cl, 1 / math.sqrt(D), Hq, Hkv, D,
                                       part_blocks=part_blocks, window=window, k_scale=ks, v_scale=vs)
    torch.cuda.synchronize()
    assert torch.equal(k1.view(torch.uint8) if kv == "fp8" else k1, k2.view(torch.uint8) if kv == "fp8" else k2)
    assert torch.equal(v1.view(torch.uint8) if kv == "fp8" else v1, v2.view(torch.uint8) if kv == "fp8" else v2)
    assert torch.equal(o1, o2)
    # fp32 reference of the whole step
    kr, vr = kc.clone(), vc.clone()
    qb = (qkv.float().sum(0).bfloat16() if src != "bf16" else qkv).cpu()
    qr = R.rope_kv_write(qb, pos, slots, cs.cpu(), kr, vr, Hq, Hkv, D, ks, vs)
    ref = R.paged_decode_attention(qr, kr, vr, bt, torch.tensor(ctx, dtype=torch.int32), 1 / math.sqrt(D),
                                   window=window, k_scale=ks, v_scale=vs)
    _close(o2, ref, 3e-2 if kv == "fp8" else 2e-2)


def test_paged_decode_rope_attention_rejects_bad_shapes():
    Hq, Hkv, D = 8, 2, 128
    kc, vc, bt = _fill_cache([40, 70], Hkv, D)
    cs = R.rope_cos_sin(256, D, 1e4, device=DEV)
    pos = torch.tensor([39, 69], dtype=torch.int32, device=DEV)
    sl = torch.tensor([0, 1], dtype=torch.int32, device=DEV)
    cl = torch.tensor([40, 70], dtype=torch.int32, device=DEV)
    with pytest.raises(ValueError):     # wrong width
        K.paged_decode_rope_attention(torch.randn(2, 100, device=DEV).bfloat16(), pos, sl, cs, kc.to(DEV), vc.to(DEV),
                                      bt.to(DEV), cl, 0.1, Hq, Hkv, D)
    with pytest.raises(ValueError):     # B mismatch between qkv and the per-row tensors
        K.paged_decode_rope_attention(torch.randn(3, (Hq + 2 * Hkv) * D, device=DEV).bfloat16(), pos, sl, cs,
                                      kc.to(DEV), vc.to(DEV), bt.to(DEV), cl, 0.1, Hq, Hkv, D)


def test_dgemm_rejects_bad_shapes():
    x = torch.randn(8, 100, device=DEV).bfloat16()
    w = torch.randn(128, 100, device=DEV).bfloat16()
    with pytest.raises(ValueError):
        K.dgemm(x, w)
    x = torch.randn(8, 128, device=DEV).bfloat16()
    w = torch.randn(192, 128, device=DEV).bfloat16()
    with pytest.raises(RuntimeError):
        K.dgemm(x, w, bn=128)      # 192 rows do not tile by 128: the launcher refuses


@pytest.mark.parametrize("M,N,Kd,split", [(128, 4096, 14336, 8), (5, 256, 512, 2)])
def test_lib_splitk_linear_residual_rmsnorm(M, N, Kd, split):
    x = torch.randn(M, Kd, device=DEV).bfloat16()
    w = (torch.randn(N, Kd, device=DEV) * 0.02).bfloat16()
    r = torch.randn(M, N, device=DEV).bfloat16()
    nw = (1 + 0.1 * torch.randn(N, device=DEV)).bfloat16()
    ref_o, ref_r = R.rmsnorm(_ref_linear(x, w).bfloat16(), nw.cpu(), 1e-5, r.cpu())
    rr = r.clone()
    o = K.lib_splitk_linear_residual_rmsnorm(x, w, split, rr, nw, 1e-5)
    _close(rr, ref_r, 3e-2)
    _close(o, ref_o, 5e-2)


# ------------------------------------------------------------------ FP8 (e4m3fn) KV cache
F8 = torch.float8_e4m3fn


def _fill_cache_fp8(ctx_lens, Hkv, D, k_scale, v_scale):
    kc, vc, bt = _fill_cache(ctx_lens, Hkv, D)
    return ((kc.float() / k_scale).clamp(-448, 448).to(F8), (vc.float() / v_scale).clamp(-448, 448).to(F8), bt)


@pytest.mark.parametrize("scales", [(1.0, 1.0), (0.5, 0.25)])
def test_rope_kv_write_fp8_matches_reference_bytes(scales):
    """The kernel writes OCP e4m3fn bytes identical to torch's float8_e4m3fn of the same values
    (per-token and whole-block-run V paths)."""
    ks, vs = scales
    Hq, Hkv, D = 8, 2, 128
    slots = [3 * 32 + 5 + i for i in range(27)] + [9 * 32 + i for i in range(32)] + [4 * 32 + i for i in range(11)]
    T = len(slots)
    qkv = (torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV) * 3).bfloat16()
    pos = torch.arange(T, device=DEV, dtype=torch.int32)
    cs = R.rope_cos_sin(4096, D, 1e6, device=DEV)
    sl = torch.tensor(slots, dtype=torch.int32, device=DEV)
    kr, vr = torch.zeros(16, Hkv, 32, D, dtype=F8), torch.zeros(16, Hkv, D, 32, dtype=F8)
    qr = R.rope_kv_write(qkv.cpu(), pos.cpu(), sl.cpu(), cs.cpu(), kr, vr, Hq, Hkv, D, ks, vs)
    for runs in (None, torch.from_numpy(K.v_runs(slots)).to(DEV)):
        kc = torch.zeros(16, Hkv, 32, D, dtype=F8, device=DEV)
        vc = torch.zeros(16, Hkv, D, 32, dtype=F8, device=DEV)
        q = K.rope_kv_write(qkv, pos, sl, cs, kc, vc, Hq, Hkv, D, runs=runs, k_scale=ks, v_scale=vs)
        _close(q, qr, 2e-2)
        kb, kref = kc.cpu().view(torch.uint8), kr.view(torch.uint8)
        # K goes through the rotation in fp32 on both sides: allow a 1-ulp fp8 difference on a few values
        assert (kb.int() - kref.int()).abs().max() <= 1 and (kb != kref).float().mean() < 0.01
        assert torch.equal(vc.cpu().view(torch.uint8), vr.view(torch.uint8))


@pytest.mark.parametrize("G", [1, 4, 8])
@pytest.mark.parametrize("part_blocks", [4, -1, -3])
def test_paged_decode_fp8(G, part_blocks):
    Hkv, D = 2, 128
    Hq = Hkv * G
    ctx = [1, 31, 33, 100, 517, 2049]
    kc, vc, bt = _fill_cache_fp8(ctx, Hkv, D, 0.5, 0.25)
    q = torch.randn(len(ctx), Hq, D).bfloat16()
    cl = torch.tensor(ctx, dtype=torch.int32)
    ref = R.paged_decode_attention(q, kc, vc, bt, cl, 1 / math.sqrt(D), k_scale=0.5, v_scale=0.25)
    out = K.paged_decode_attention(q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), cl.to(DEV), 1 / math.sqrt(D),
                                   part_blocks=part_blocks, k_scale=0.5, v_scale=0.25)
    _close(out, ref, 2e-2)


@pytest.mark.parametrize("G", [1, 2, 4, 8])
def test_prefill_attention_fp8(G):
    Hkv, D = 2, 128
    Hq = Hkv * G
    seqs = [(1, 1), (17, 17), (200, 200), (70, 300), (129, 1000)]
    kc, vc, bt = _fill_cache_fp8([c for _, c in seqs], Hkv, D, 0.5, 2.0)
    cu = [0]
    for qn, _ in seqs:
        cu.append(cu[-1] + qn)
    q = torch.randn(cu[-1], Hq, D).bfloat16()
    cu_t = torch.tensor(cu, dtype=torch.int32)
    cl = torch.tensor([c for _, c in seqs], dtype=torch.int32)
    ref = R.prefill_attention(q, kc, vc, bt, cu_t, cl, 1 / math.sqrt(D), k_scale=0.5, v_scale=2.0)
    out = K.prefill_attention(q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), cu_t.to(DEV), cl.to(DEV),
                              1 / math.sqrt(D), k_scale=0.5, v_scale=2.0)
    _close(out, ref, 2e-2)


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("N,Kd", [(6144, 4096), (512, 11008), (258, 1000)])
def test_gemv_bf16_and_f32(M, N, Kd):
    """GEMV (gemm.hip: gemv_kernel) vs fp32 matmul; K not a multiple of the 512-wide chunk included."""
    x = torch.randn(M, Kd, device=DEV).bfloat16()
    w = (torch.randn(N, Kd, device=DEV) / math.sqrt(Kd)).bfloat16()
    ref = x.float() @ w.float().t()
    _close(K.gemv(x, w, "f32"), ref, atol=2e-3, rtol=1e-3)
    _close(K.gemv(x, w, "bf16"), ref, atol=2e-2)


@pytest.mark.parametrize("M", [1, 4])
def test_gemv_swiglu_interleaved(M):
    Kd, F = 4096, 1024
    x = torch.randn(M, Kd, device=DEV).bfloat16()
    gu = (torch.randn(2 * F, Kd, device=DEV) / math.sqrt(Kd)).bfloat16()
    y = (x.float() @ gu.float().t()).bfloat16().float()
    ref = torch.nn.functional.silu(y[:, :F]) * y[:, F:]
    _close(K.gemv(x, R.interleave_gate_up(gu), "swiglu"), ref, atol=2e-2)


def test_gemv_residual_rmsnorm_matches_reference():
    M, Kd, N = 2, 14336, 4096
    x = torch.randn(M, Kd, device=DEV).bfloat16()
    w = (torch.randn(N, Kd, device=DEV) / math.sqrt(Kd)).bfloat16()
    res = torch.randn(M, N, device=DEV).bfloat16()
    g = torch.rand(N, device=DEV).bfloat16() + 0.5
    r2 = res.clone()
    out = K.gemv_residual_rmsnorm(x, w, r2, g, 1e-5)
    ref_o, ref_r = R.rmsnorm((x.float() @ w.float().t()).bfloat16(), g, 1e-5, res)
    _close(r2, ref_r, atol=3e-2)
    _close(out, ref_o, atol=5e-2)


@pytest.mark.parametrize("V", [32000, 32003, 128256, 7])
def test_greedy_sample_vocab_sizes_and_ties(V):
    """1024-thread sampler: 4 loads in flight per thread, scalar tail when V % 8 != 0, lowest index on ties."""
    logits = torch.randn(5, V, device=DEV).bfloat16()
    logits[1] = 0.0                                   # all tied -> index 0
    logits[2, V - 1] = 100.0                          # maximum in the last (tail) element
    out = torch.empty(5, dtype=torch.int32, device=DEV)
    K.sample(logits, out)
    assert out.cpu().tolist() == R.sample_greedy(logits.cpu()).tolist()
    assert out[1].item() == 0 and out[2].item() == V - 1


@pytest.mark.parametrize("V", [32000, 517])
def test_sample_all_nan_row_stays_in_vocab(V):
    """A row of NaN logits matches no comparison; the sampler must still emit an index inside the
    vocabulary (the next embedding gather reads it)."""
    logits = torch.randn(3, V, device=DEV).bfloat16()
    logits[1] = float("nan")
    for t in (0.0, 0.7, K.SamplingParams(0.7, top_k=40, top_p=0.95, min_p=0.05)):
        out = torch.empty(3, dtype=torch.int32, device=DEV)
        K.sample(logits, out, temperature=t, seed=3)
        ids = out.cpu().tolist()
        assert all(0 <= i < V for i in ids), (t, ids)


@pytest.mark.parametrize("M,Kd", [(300, 384), (1000, 1536), (64, 384), (129, 768)])
def test_pgemm_ln(M, Kd):
    """Fused projection + bias + residual + LayerNorm (post-LN encoder sub-layer) vs the fp32
    reference of the unfused op (projection rounded to bf16 first, as the unfused path does);
    edge rows past M are never written."""
    N = 384
    x = (torch.rand(M, Kd, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(N, Kd, device=DEV) * 2 - 1) / Kd ** 0.5).bfloat16()
    b = (torch.rand(N, device=DEV) * 0.2 - 0.1).bfloat16()
    res = torch.randn(M, N, device=DEV).bfloat16()
    g = (1 + 0.1 * torch.randn(N, device=DEV)).bfloat16()
    be = (0.1 * torch.randn(N, device=DEV)).bfloat16()
    y = K.pgemm_ln(x, w, b, res, g, be, 1e-12)
    proj = _ref_linear(x, w).bfloat16()
    want = R.layernorm(proj, g.cpu(), be.cpu(), 1e-12, b.cpu(), res.cpu())
    _close(y, want.float(), 3e-2)
    # the same as the unfused kernels on the device
    unf = K.layernorm(K.pgemm(x, w), g, be, 1e-12, bias=b, residual=res)
    assert float((y.float() - unf.float()).abs().max()) <= 0.0625


@pytest.mark.parametrize("M,N,Kd,bn", [(300, 1024, 512, 128), (1000, 4096, 1024, 64), (257, 2048, 2048, 128)])
def test_pgemm_f32_epilogue_packed_and_rowmajor(M, N, Kd, bn):
    """The prefill GEMM's fp32 epilogue (a tensor-parallel row-parallel partial, all-reduced in fp32
    before its one bf16 rounding): the fp32 accumulators vs the fp32 reference within fp32
    summation-order error, rows past M never stored; the bf16 epilogue is exactly its rounding."""
    x = (torch.rand(M, Kd, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(N, Kd, device=DEV) * 2 - 1) / Kd ** 0.5).bfloat16()
    ref = _ref_linear(x, w)
    pw = K.pack_dgemm_weight(w, bn=bn)
    for wt in (pw, w):
        y = K.pgemm(x, wt, "f32")
        assert y.dtype == torch.float32 and y.shape == (M, N)
        err = float((y.cpu() - ref).abs().max())
        assert err <= 1e-4 * float(ref.abs().max()) + 1e-5, err
        assert torch.equal(y.bfloat16(), K.pgemm(x, wt, "bf16", variant="pp"))


def test_dgemm_tail_past_slice_loads_change_nothing():
    """The decode GEMM's ring refills past a k-slice's end are out-of-range buffer loads (zeros, no
    memory traffic): split-K slabs equal the round-5 re-reading tail's bit for bit, for slices that
    are whole multiples of the ring (qkv-like) and not (down-like: 28 stages)."""
    for (N, Kd, split, bn) in ((768, 4096, 4, 96), (512, 14336, 8, 128), (1024, 512, 1, 64)):
        x = (torch.rand(128, Kd, device=DEV) * 2 - 1).bfloat16()
        w = ((torch.rand(N, Kd, device=DEV) * 2 - 1) / Kd ** 0.5).bfloat16()
        pw = K.pack_dgemm_weight(w, bn=bn)
        a = K.dgemm(x, pw, "part", split).clone()
        b = torch.empty_like(a)
        K.check(K.kernels().cfc_dgemm_ablate(x.data_ptr(), pw.data.data_ptr(), 128, N, Kd, split, bn, 256,
                                             b.data_ptr(), K._stream(x)), "ablate")
        torch.cuda.synchronize()
        assert torch.equal(a, b), (N, Kd, split)
        _close(a.sum(0), _ref_linear(x, w), 1e-2)
