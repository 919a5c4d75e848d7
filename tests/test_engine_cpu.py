"""CPU path of the decoder/encoder (reference ops): engine plumbing, chunked prefill, stops."""
import torch

from copilot_for_consensus_amd.models.decoder import DecoderModel, DecoderWeights, get_config
from copilot_for_consensus_amd.models.encoder import EncoderModel
from copilot_for_consensus_amd.ops import reference as R
from copilot_for_consensus_amd.runtime.engine import LLMEngine
from copilot_for_consensus_amd.runtime.kv_cache import BlockPool, PagedKVCache


def _engine(seed=0, prefill=4096):
    cfg = get_config("tiny")
    m = DecoderModel(DecoderWeights.random(cfg, "cpu", seed=seed))
    kv = PagedKVCache(cfg.layers, 32, cfg.kv_heads, cfg.head_dim, "cpu")
    return LLMEngine(m, kv, max_prefill_tokens=prefill)


def test_generate_shapes_and_block_reuse():
    eng = _engine()
    free0 = eng.kv.pool.num_free()
    res = eng.generate([[1, 2, 3, 4], [1] * 50], max_new_tokens=5, ignore_eos=True)
    assert [len(t) for t in res.tokens] == [5, 5]
    # every block is back in the pool except the one full prompt block kept by the prefix cache
    assert eng.kv.pool.num_free() + eng.prefix_cache.cached_blocks() == free0 == 32


def test_chunked_prefill_equals_full_prefill():
    prompts = [[1] + list(range(3, 120)), [1, 7, 7, 7]]
    a = _engine(prefill=4096).generate(prompts, 4, ignore_eos=True).tokens
    b = _engine(prefill=50).generate(prompts, 4, ignore_eos=True).tokens
    assert a == b


def test_incremental_decode_matches_full_recompute():
    # token t+1 from decode == greedy from a fresh prefill of prompt + generated[:t]
    eng = _engine(seed=2)
    p = [1, 11, 12, 13, 14, 15]
    gen = eng.generate([p], 4, ignore_eos=True).tokens[0]
    for t in range(1, 4):
        again = eng.generate([p + gen[:t]], 1, ignore_eos=True).tokens[0]
        assert again[0] == gen[t]


def test_stop_tokens_truncate():
    eng = _engine(seed=1)
    full = eng.generate([[1, 2, 3]], 6, ignore_eos=True).tokens[0]
    stop = full[2]
    cut = eng.generate([[1, 2, 3]], 6, stop_ids=(stop,)).tokens[0]
    assert cut == full[:full.index(stop)]


def test_blockpool():
    bp = BlockPool(10)
    a = bp.alloc(4)
    b = bp.alloc(6)
    assert sorted(a + b) == list(range(10)) and bp.num_free() == 0
    try:
        bp.alloc(1)
        raise AssertionError("expected MemoryError")
    except MemoryError:
        pass
    bp.free(a)
    assert bp.num_free() == 4


def test_encoder_cpu_pooling_normalized():
    enc = EncoderModel.random("tiny", "cpu", seed=0)
    e = enc.encode_ids([[1, 2, 3], [4, 5, 6, 7, 8]])
    assert e.shape == (2, 64)
    assert torch.allclose(e.norm(dim=1), torch.ones(2), atol=1e-3)


def test_v_cache_slot_groups_layout_and_round_trip():
    """V tiles are stored [4 slot groups][D][8] (common.h kv_v_off): slot position p of row d at
    element (p // 8) * 8 D + 8 d + p % 8 of the tile, so one token's column spans D / 8 lines of
    128 B; the reference writes and gathers through that order."""
    Hq, Hkv, D, nblk = 4, 2, 16, 3
    torch.manual_seed(0)
    kc = torch.zeros(nblk, Hkv, R.KV_BLOCK, D)
    vc = torch.zeros(nblk, Hkv, D, R.KV_BLOCK)
    T = 40
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D)
    slots = torch.randperm(nblk * R.KV_BLOCK)[:T].int()
    cs = R.rope_cos_sin(64, D, 1e4)
    R.rope_kv_write(qkv, torch.arange(T, dtype=torch.int32), slots, cs, kc, vc, Hq, Hkv, D)
    v = qkv.view(T, Hq + 2 * Hkv, D)[:, Hq + Hkv:]
    perm = R.v_slot_perm()
    flat = vc.view(nblk, Hkv, -1)
    for t in range(T):
        blk, off = divmod(int(slots[t]), R.KV_BLOCK)
        p = int(perm[off])
        for d in (0, 5, D - 1):
            assert torch.equal(flat[blk, :, (p // 8) * 8 * D + 8 * d + p % 8], v[t, :, d])
    k_all, v_all = R.gather_kv(kc, vc, torch.arange(nblk, dtype=torch.int32), nblk * R.KV_BLOCK)
    for t in range(T):
        assert torch.equal(v_all[int(slots[t])], v[t])


def test_v_slot_perm_is_permutation():
    p = R.v_slot_perm()
    assert sorted(p.tolist()) == list(range(32))
    # slot 8g+j holds key perm(g, j) = j<4 ? 4g+j : 16+4g+j-4
    inv = {int(s): k for k, s in enumerate(p.tolist())}
    for g in range(4):
        for j in range(8):
            assert inv[8 * g + j] == (4 * g + j if j < 4 else 16 + 4 * g + j - 4)


def test_prefix_cache_reuse_matches_uncached():
    from copilot_for_consensus_amd.runtime.prefix_cache import PrefixCache
    system = [1] + list(range(20, 120))          # 101 shared tokens -> 3 shareable blocks
    prompts = [system + [5, 6, 7], system + list(range(200, 260)), system + [9]]
    cfg = get_config("tiny")
    w = DecoderWeights.random(cfg, "cpu", seed=4)
    ref = LLMEngine(DecoderModel(w), PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, "cpu"),
                    prefix_cache=False).generate(prompts, 5, ignore_eos=True)
    eng = LLMEngine(DecoderModel(w), PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, "cpu"))
    free0 = eng.kv.pool.num_free()
    a = eng.generate(prompts, 5, ignore_eos=True)
    assert a.tokens == ref.tokens
    assert a.cached_prompt_tokens == 2 * 3 * 32           # dedupe inside the first batch
    b = eng.generate(prompts[::-1], 5, ignore_eos=True)  # second batch: every prompt hits
    # prompt 2 (161 tokens) also hits its own 2 further full blocks
    assert b.tokens == ref.tokens[::-1] and b.cached_prompt_tokens == (3 * 3 + 2) * 32
    pc: PrefixCache = eng.prefix_cache
    assert pc.cached_blocks() == 3 + 2                   # system blocks + prompt 2's own full blocks
    # cached blocks are held back from the pool until an allocation needs them
    assert eng.kv.pool.num_free() == free0 - pc.cached_blocks()
    eng.generate([[1] + [3] * 1500], 2, ignore_eos=True)  # needs nearly the whole pool -> evicts
    assert eng.kv.pool.num_free() + pc.cached_blocks() == free0


def test_prefix_cache_invalidates_on_failure():
    eng = _engine()
    big = [[1] + [2] * 100] * 30                           # 30 x 4 blocks > 32-block cache
    try:
        eng.generate(big, 40, ignore_eos=True)
        raise AssertionError("expected MemoryError")
    except MemoryError:
        pass
    # nothing leaked, and no entry of the failed call (never prefilled) can be hit
    assert eng.kv.pool.num_free() == 32 and eng.prefix_cache.cached_blocks() == 0
    again = eng.generate([[1] + [2] * 100], 3, ignore_eos=True)
    assert again.cached_prompt_tokens == 0


def test_v_runs_split_on_block_and_offset_breaks():
    from copilot_for_consensus_amd.ops import kernels as K
    slots = [3 * 32 + 30, 3 * 32 + 31, 7 * 32, 7 * 32 + 1, 7 * 32 + 3, 2 * 32 + 0]
    assert K.v_runs(slots).tolist() == [[0, 2, 3, 30], [2, 2, 7, 0], [4, 1, 7, 3], [5, 1, 2, 0]]
    full = K.v_runs([5 * 32 + i for i in range(32)] + [6 * 32 + i for i in range(32)])
    assert full.tolist() == [[0, 32, 5, 0], [32, 32, 6, 0]]
    assert K.v_runs([]).shape == (0, 4)


def test_reference_sliding_window_is_attention_over_the_last_keys():
    import math

    from copilot_for_consensus_amd.ops import reference as R
    g = torch.Generator().manual_seed(0)
    q = torch.randn(5, 4, 16, generator=g)
    k = torch.randn(40, 2, 16, generator=g)
    v = torch.randn(40, 2, 16, generator=g)
    W = 7
    got = R._attend(q, k, v, 1 / math.sqrt(16), causal_offset=35, window=W)
    for i in range(5):
        p = 35 + i
        want = R._attend(q[i:i + 1], k[p - W + 1:p + 1], v[p - W + 1:p + 1], 1 / math.sqrt(16))
        assert torch.allclose(got[i:i + 1], want, atol=1e-5)
    # decode form: the last query sees the last W keys
    dec = R._attend(q[:1], k, v, 0.25, window=W)
    assert torch.allclose(dec, R._attend(q[:1], k[-W:], v[-W:], 0.25), atol=1e-5)


def test_fp8_reference_cache_round_trip():
    """float8_e4m3fn caches store value / scale (clamped to +-448) and gather scales back."""
    Hq, Hkv, D = 4, 2, 16
    T = 40
    qkv = (torch.randn(T, (Hq + 2 * Hkv) * D) * 4).bfloat16()
    cs = R.rope_cos_sin(128, D, 1e4)
    kc = torch.zeros(4, Hkv, 32, D, dtype=torch.float8_e4m3fn)
    vc = torch.zeros(4, Hkv, D, 32, dtype=torch.float8_e4m3fn)
    kb, vb = torch.zeros(4, Hkv, 32, D).bfloat16(), torch.zeros(4, Hkv, D, 32).bfloat16()
    slots = torch.arange(T, dtype=torch.int32) + 32
    pos = torch.arange(T, dtype=torch.int32)
    R.rope_kv_write(qkv, pos, slots, cs, kc, vc, Hq, Hkv, D, k_scale=0.25, v_scale=2.0)
    R.rope_kv_write(qkv, pos, slots, cs, kb, vb, Hq, Hkv, D)
    bt = torch.tensor([1, 2], dtype=torch.int32)
    k8, v8 = R.gather_kv(kc, vc, bt, T, 0.25, 2.0)
    k16, v16 = R.gather_kv(kb, vb, bt, T)
    # e4m3: 3 mantissa bits -> relative error <= 2^-4 (plus the clamp, not reached here)
    assert torch.allclose(k8, k16.float(), rtol=0.07, atol=0.25 * 2 ** -9)
    assert torch.allclose(v8, v16.float(), rtol=0.07, atol=2.0 * 2 ** -9)
    try:
        from copilot_for_consensus_amd.runtime.kv_cache import PagedKVCache as P
        P(1, 2, 1, 16, "cpu", dtype=torch.float16)
        raise AssertionError("fp16 cache accepted")
    except ValueError:
        pass


def test_llama2_presets_match_published_parameter_counts():
    # HF Llama-2 checkpoints: 6,738,415,616 and 13,015,864,320 parameters
    assert get_config("llama-2-7b").num_params() == 6_738_415_616
    assert get_config("llama-2-13b").num_params() == 13_015_864_320
    assert get_config("llama-2-13b").kv_heads == get_config("llama-2-13b").heads   # MHA, G = 1


def test_mha_incremental_decode_matches_full_recompute():
    """Multi-head attention (kv_heads == heads, the Llama-2 layout) through the paged engine."""
    cfg = get_config("tiny-mha")
    m = DecoderModel(DecoderWeights.random(cfg, "cpu", seed=4))
    eng = LLMEngine(m, PagedKVCache(cfg.layers, 32, cfg.kv_heads, cfg.head_dim, "cpu"))
    p = [1] + list(range(20, 60))
    gen = eng.generate([p], 4, ignore_eos=True).tokens[0]
    for t in range(1, 4):
        assert eng.generate([p + gen[:t]], 1, ignore_eos=True).tokens[0][0] == gen[t]


def test_packed_decode_weights_round_trip():
    """DecoderWeights.pack_decode: every projection's packed copy unpacks to the row-major weight
    (CPU reference packer), tiled with the decode GEMM's choice for a 128-row batch."""
    from copilot_for_consensus_amd.ops import kernels as K
    cfg = get_config("tiny")
    w = DecoderWeights.random(cfg, "cpu").pack_decode()
    for layer, packed in zip(w.layers, w.packed):
        for name, p in packed.items():
            assert isinstance(p, K.PackedWeight) and p.shape == tuple(layer[name].shape)
            assert torch.equal(K._rowmajor(p), layer[name]), name
    assert w.packed_bytes() == sum(p.nbytes() for layer in w.packed for p in layer.values()) + \
        w.packed_lm_head.nbytes()
    x = torch.randn(3, cfg.hidden).bfloat16()
    assert torch.equal(K.dgemm_linear(x, w.packed[0]["qkv"]), torch.nn.functional.linear(x, w.layers[0]["qkv"]))


def test_pack_layout_fragment_order():
    """Packed element [nb, kb, t, lane, j] = W[nb*bn + 16t + lane%16, 32kb + 8(lane//16) + j]."""
    bn, N, Kd = 64, 128, 96
    w = torch.arange(N * Kd, dtype=torch.float32).view(N, Kd)
    p = R.pack_dgemm_weight(w, bn)
    assert p.shape == (N // bn, Kd // 32, bn // 16, 64, 8)
    for nb, kb, t, lane, j in [(0, 0, 0, 0, 0), (1, 2, 3, 63, 7), (0, 1, 2, 17, 5), (1, 0, 1, 40, 3)]:
        assert p[nb, kb, t, lane, j] == w[nb * bn + 16 * t + lane % 16, 32 * kb + 8 * (lane // 16) + j]
    assert torch.equal(R.unpack_dgemm_weight(p), w)


def test_gemv_packed_config_fills_the_chip_and_keeps_whole_steps():
    """The packed GEMV's (split, waves): slab form -> at most one workgroup per CU (tiles x split <=
    256 unless one tile already exceeds it), every wave >= one whole step of U kg; in-kernel
    epilogues take split 1 (16 waves only at M = 1)."""
    from copilot_for_consensus_amd.ops import kernels as K
    shapes = [(6144, 4096, 6), (4096, 4096, 4), (28672, 4096, 7), (4096, 14336, 8), (15360, 5120, 8),
              (5120, 5120, 4), (27648, 5120, 8), (5120, 13824, 8), (768, 512, 8), (1024, 1536, 4)]
    for N, Kd, nw in shapes:
        tiles, kg = N // (16 * nw), Kd // 32
        for M in (1, 2, 3, 4):
            u = 2 if M > 2 else (3 if nw >= 7 else 4)
            split, waves = K.gemv_packed_config(N, Kd, nw, M)
            assert 1 <= split <= kg and waves in (4, 8)
            assert tiles * split <= max(256, tiles)
            assert split == 1 or kg // split >= waves * u
            s1, w1 = K.gemv_packed_config(N, Kd, nw, M, slab=False)
            assert s1 == 1 and w1 in ((4, 8, 16) if M == 1 else (4, 8))
    # the measured points the rule was fitted to (profiles/r04_gemv_grid.jsonl)
    assert K.gemv_packed_config(6144, 4096, 6) == (4, 8)
    assert K.gemv_packed_config(4096, 14336, 8) == (8, 8)
    assert K.gemv_packed_config(5120, 13824, 8) == (6, 8)


def test_prefill_routes_short_chunks_to_the_decode_gemm():
    """_dgemm_faster: fewer than 96 pgemm tiles -> the decode GEMM (profiles/r04_prefill_small_m.jsonl)."""
    from copilot_for_consensus_amd.models.decoder import DecoderModel
    m = DecoderModel.__new__(DecoderModel)
    assert m._dgemm_faster(512, 6144, 4096) and m._dgemm_faster(1024, 4096, 14336)
    assert not m._dgemm_faster(1024, 6144, 4096) and not m._dgemm_faster(16384, 4096, 4096)
    assert not m._dgemm_faster(512, 28672, 4096)


def test_longest_first_slots_return_caller_order(monkeypatch):
    """CFC_DECODE_LPT=1 fills the decode slots longest prompt first; tokens and prompt lengths come
    back in the caller's order, equal to the default slot order's."""
    prompts = [[1, 5], [1] + list(range(3, 90)), [1, 9, 9, 9, 9], [1] + list(range(40, 70))]
    monkeypatch.setenv("CFC_DECODE_LPT", "0")
    ref = _engine().generate(prompts, 5, ignore_eos=True)
    monkeypatch.setenv("CFC_DECODE_LPT", "1")
    eng = _engine()
    assert eng.lpt
    got = eng.generate(prompts, 5, ignore_eos=True)
    assert got.tokens == ref.tokens and got.prompt_lens == ref.prompt_lens == [len(p) for p in prompts]


def test_prefill_tile_order_groups_sequences_by_l2_budget_heaviest_first_inside():
    """The prefill attention's tile order (ops.kernels.prefill_tiles with ctx_lens): consecutive
    sequences in groups of at most PREFILL_GROUP_CTX context tokens, groups in order, each group's
    tiles heaviest-first (most keys under the causal mask); every tile exactly once."""
    from copilot_for_consensus_amd.ops import kernels as K
    lens = [2800, 2600, 3000, 700, 700, 700, 9000, 64]
    ctx = [n + (128 if i % 2 else 0) for i, n in enumerate(lens)]     # some with cached prefix keys
    cu = [0]
    for n in lens:
        cu.append(cu[-1] + n)
    seqs, q0 = K.prefill_tiles(cu, 64, ctx)
    want = {(s, r) for s, n in enumerate(lens) for r in range(0, n, 64)}
    assert sorted(zip(seqs, q0)) == sorted(want)
    # the groups the order must follow
    groups, acc, g = [], 0, 0
    for c in ctx:
        if acc and acc + c > K.PREFILL_GROUP_CTX:
            g, acc = g + 1, 0
        acc += c
        groups.append(g)
    order_groups = [groups[s] for s in seqs]
    assert order_groups == sorted(order_groups)
    keys = [ctx[s] - lens[s] + min(r + 64, lens[s]) for s, r in zip(seqs, q0)]
    for g in set(groups):
        ks = [k for k, og in zip(keys, order_groups) if og == g]
        assert ks == sorted(ks, reverse=True)
    assert len(set(groups)) > 2          # the 6144-token budget splits this batch
    # without ctx_lens: plain sequence order (encoder / bidirectional use)
    s2, r2 = K.prefill_tiles(cu, 64)
    assert list(zip(s2, r2)) == [(s, r) for s, n in enumerate(lens) for r in range(0, n, 64)]
