"""End-to-end decoder/encoder on the GPU vs the same model run through the CPU reference ops."""
import pytest
import torch

from copilot_for_consensus_amd.models.decoder import DecoderModel, DecoderWeights, get_config
from copilot_for_consensus_amd.models.encoder import EncoderModel
from copilot_for_consensus_amd.runtime.engine import LLMEngine
from copilot_for_consensus_amd.runtime.kv_cache import PagedKVCache

pytestmark = pytest.mark.gpu


def _to_cpu_fp32_model(w: DecoderWeights):
    c = DecoderWeights(w.cfg, "cpu")
    c.layers = [{k: v.cpu() for k, v in w.rowmajor_layer(i).items()} for i in range(w.cfg.layers)]
    c.embed, c.final_norm, c.lm_head = w.embed.cpu(), w.final_norm.cpu(), w.lm_head.cpu()
    c.gate_up_interleaved = w.gate_up_interleaved
    return c


def test_decoder_prefill_logits_match_reference():
    cfg = get_config("tiny")
    w = DecoderWeights.random(cfg, "cuda", seed=3)
    m = DecoderModel(w)
    mc = DecoderModel(_to_cpu_fp32_model(w))
    prompts = [[1] + list(range(5, 5 + 90)), [1, 9, 8, 7]]
    outs = []
    for model, dev in ((m, "cuda"), (mc, "cpu")):
        kv = PagedKVCache(cfg.layers, 16, cfg.kv_heads, cfg.head_dim, dev)
        eng = LLMEngine(model, kv, max_prefill_tokens=64, use_graph=(dev == "cuda"))  # 64 => chunked prefill
        outs.append(eng.generate(prompts, max_new_tokens=6, ignore_eos=True).tokens)
    # greedy tokens agree except for rare bf16 near-ties; require the first token exact
    assert [t[0] for t in outs[0]] == [t[0] for t in outs[1]]
    agree = sum(a == b for x, y in zip(*outs) for a, b in zip(x, y))
    assert agree >= 10, outs


def test_fp8_kv_engine_matches_reference_fp8_engine():
    """The opt-in FP8 (e4m3fn) KV cache end to end: GPU engine (fp8 kernels, hipGraph decode) vs the
    CPU reference engine over the same fp8 cache semantics."""
    cfg = get_config("tiny")
    w = DecoderWeights.random(cfg, "cuda", seed=3)
    prompts = [[1] + list(range(5, 5 + 90)), [1, 9, 8, 7], [1] + list(range(300, 371))]
    outs = []
    for model, dev in ((DecoderModel(w), "cuda"), (DecoderModel(_to_cpu_fp32_model(w)), "cpu")):
        kv = PagedKVCache(cfg.layers, 24, cfg.kv_heads, cfg.head_dim, dev, dtype=torch.float8_e4m3fn,
                          k_scale=0.5, v_scale=0.5)
        eng = LLMEngine(model, kv, max_prefill_tokens=64, use_graph=(dev == "cuda"))
        outs.append(eng.generate(prompts, max_new_tokens=8, ignore_eos=True).tokens)
    assert [t[0] for t in outs[0]] == [t[0] for t in outs[1]]
    agree = sum(a == b for x, y in zip(*outs) for a, b in zip(x, y))
    assert agree >= 0.8 * sum(len(x) for x in outs[1]), outs


def test_graph_and_eager_decode_agree():
    cfg = get_config("tiny")
    w = DecoderWeights.random(cfg, "cuda", seed=5)
    m = DecoderModel(w)
    res = []
    for g in (True, False):
        kv = PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, "cuda")
        res.append(LLMEngine(m, kv, use_graph=g).generate([[1, 2, 3] * 30, [4, 5] * 70], 40, ignore_eos=True).tokens)
    assert res[0] == res[1]


PROMPTS8 = [[1, 2, 3] * 30, [4, 5] * 70, [1, 7], [9] * 17, [3, 1, 4, 1, 5] * 9, [2, 6] * 33, [8] * 5, [7, 7, 1] * 21]


@pytest.mark.parametrize("mode", ["splitk", "dgemm"])
def test_decode_gemm_modes_match_library(mode, monkeypatch):
    cfg = get_config("tiny")
    res = []
    for m in (mode, "lib"):
        monkeypatch.setenv("CFC_DECODE_GEMM", m)
        # fresh weights per model: the dgemm model keeps only the packed copy of the projections
        model = DecoderModel(DecoderWeights.random(cfg, "cuda", seed=11))
        assert model.decode_gemm == m
        kv = PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, "cuda")
        # 8 sequences: decode batches above the GEMV's 4 rows take the mode's GEMMs
        res.append(LLMEngine(model, kv).generate(PROMPTS8, 24, ignore_eos=True).tokens)
    agree = sum(a == b for x, y in zip(*res) for a, b in zip(x, y))
    # different fp32 summation orders: a bf16 near-tie can flip one greedy token, after which that
    # sequence continues differently; first tokens must agree exactly, the bulk must agree
    assert [t[0] for t in res[0]] == [t[0] for t in res[1]] and agree >= 0.75 * 8 * 24, res


def test_fused_decode_matches_unfused():
    cfg = get_config("tiny")
    res = []
    for fused in (True, False):
        m = DecoderModel(DecoderWeights.random(cfg, "cuda", seed=7), fused_decode=fused)
        assert m.fused_decode == fused
        kv = PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, "cuda")
        res.append(LLMEngine(m, kv).generate(PROMPTS8, 24, ignore_eos=True).tokens)
    agree = sum(a == b for x, y in zip(*res) for a, b in zip(x, y))
    assert [t[0] for t in res[0]] == [t[0] for t in res[1]] and agree >= 0.9 * 8 * 24, res


def test_encoder_gpu_vs_cpu():
    enc = EncoderModel.random("tiny", "cuda", seed=1)
    cpu = EncoderModel("tiny", "cpu")
    cpu.p = {k: v.cpu() for k, v in enc.p.items()}
    cpu.layers = [{k: v.cpu() for k, v in layer.items()} for layer in enc.layers]
    batch = [[1, 2, 3, 4, 5], [7] * 100, [9, 8]]
    a = enc.encode_ids(batch).cpu()
    b = cpu.encode_ids(batch)
    assert torch.allclose(a, b, atol=3e-2), (a - b).abs().max()


def test_long_context_generation_matches_reference():
    """A 7k-token prompt (multi-chunk prefill, ~220 KV blocks per sequence, split-KV decode) on
    the GPU engine vs the CPU reference engine of the same weights."""
    cfg = get_config("small")
    w = DecoderWeights.random(cfg, "cuda", seed=11)
    g = torch.Generator().manual_seed(2)
    prompts = [[1] + torch.randint(3, cfg.vocab_size, (7000,), generator=g).tolist(),
               [1] + torch.randint(3, cfg.vocab_size, (300,), generator=g).tolist()]
    outs = []
    for model, dev in ((DecoderModel(w), "cuda"), (DecoderModel(_to_cpu_fp32_model(w)), "cpu")):
        kv = PagedKVCache(cfg.layers, 260, cfg.kv_heads, cfg.head_dim, dev)
        eng = LLMEngine(model, kv, max_prefill_tokens=4096, use_graph=(dev == "cuda"))
        outs.append(eng.generate(prompts, max_new_tokens=8, ignore_eos=True).tokens)
    assert [t[0] for t in outs[0]] == [t[0] for t in outs[1]]
    agree = sum(a == b for x, y in zip(*outs) for a, b in zip(x, y))
    assert agree >= 12, outs


def test_mha_generation_matches_reference():
    """Llama-2 layout (kv_heads == heads: G = 1 in the GQA-packed prefill kernel, one query head per
    kv-head in split-KV decode) on the GPU engine vs the CPU reference engine."""
    cfg = get_config("tiny-mha")
    w = DecoderWeights.random(cfg, "cuda", seed=7)
    prompts = [[1] + list(range(5, 5 + 300)), [1, 9, 8, 7], [1] + list(range(100, 171))]
    outs = []
    for model, dev in ((DecoderModel(w), "cuda"), (DecoderModel(_to_cpu_fp32_model(w)), "cpu")):
        kv = PagedKVCache(cfg.layers, 40, cfg.kv_heads, cfg.head_dim, dev)
        eng = LLMEngine(model, kv, max_prefill_tokens=128, use_graph=(dev == "cuda"))
        outs.append(eng.generate(prompts, max_new_tokens=8, ignore_eos=True).tokens)
    assert [t[0] for t in outs[0]] == [t[0] for t in outs[1]]
    agree = sum(a == b for x, y in zip(*outs) for a, b in zip(x, y))
    assert agree >= 0.8 * sum(len(x) for x in outs[1]), outs


def test_gemv_decode_matches_splitk_decode(monkeypatch):
    """B <= 4 decode on the GEMV kernel (over the packed-only weights) vs the decode GEMM, same weights."""
    cfg = get_config("small")
    w = DecoderWeights.random(cfg, "cuda", seed=13)
    res = []
    for flag in ("1", "0"):
        monkeypatch.setenv("CFC_DECODE_GEMV", flag)
        model = DecoderModel(w)
        assert model.decode_gemv == (flag == "1")
        kv = PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, "cuda")
        res.append(LLMEngine(model, kv).generate([[1, 2, 3] * 100, [1, 7]], 24, ignore_eos=True).tokens)
    agree = sum(a == b for x, y in zip(*res) for a, b in zip(x, y))
    assert [t[0] for t in res[0]] == [t[0] for t in res[1]] and agree >= 0.75 * 48, res


def test_small_graph_survives_workspace_growth():
    """A B=2 hipGraph (GEMV decode, fp32 partials in the shared split-K workspace) captured before a
    large batch grows the workspace must still be correct when replayed afterwards (the superseded
    buffer stays allocated)."""
    from copilot_for_consensus_amd.ops import kernels as K

    cfg = get_config("small")
    w = DecoderWeights.random(cfg, "cuda", seed=17)
    m = DecoderModel(w)
    small = [[1, 2, 3] * 40, [1, 9, 4] * 11]
    kv = PagedKVCache(cfg.layers, 1024, cfg.kv_heads, cfg.head_dim, "cuda")
    eng = LLMEngine(m, kv, use_graph=True)
    first = eng.generate(small, 16, ignore_eos=True).tokens
    g = torch.Generator().manual_seed(4)
    big = [[1] + torch.randint(3, cfg.vocab_size, (200,), generator=g).tolist() for _ in range(64)]
    eng.generate(big, 4, ignore_eos=True)
    grown = 0
    for key, ws in list(K._workspaces.items()):       # every stream's: force a growth past anything captured
        K._retired_workspaces.append(ws)
        K._workspaces[key] = torch.empty(4 * ws.numel(), device=ws.device)
        grown = max(grown, ws.numel())
    junk = torch.full((grown,), float("nan"), device="cuda")   # likely reuses freed memory
    again = eng.generate(small, 16, ignore_eos=True).tokens
    del junk
    kv2 = PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, "cuda")
    eager = LLMEngine(m, kv2, use_graph=False).generate(small, 16, ignore_eos=True).tokens
    assert again == first == eager


def test_odd_vocab_lm_head_single_stream():
    """An odd vocabulary (e.g. 32001-token fine-tunes) keeps the lm_head off the row-pair GEMV."""
    from copilot_for_consensus_amd.models.decoder import DecoderConfig

    cfg = DecoderConfig("tiny-odd", 517, 256, 2, 4, 2, 128, 512, rope_theta=1e4, max_positions=4096)
    w = DecoderWeights.random(cfg, "cuda", seed=21)
    prompts = [[1] + list(range(5, 60))]
    outs = []
    for model, dev in ((DecoderModel(w), "cuda"), (DecoderModel(_to_cpu_fp32_model(w)), "cpu")):
        kv = PagedKVCache(cfg.layers, 16, cfg.kv_heads, cfg.head_dim, dev)
        outs.append(LLMEngine(model, kv, use_graph=(dev == "cuda")).generate(prompts, 8, ignore_eos=True).tokens)
    assert all(0 <= t < cfg.vocab_size for t in outs[0][0])
    assert outs[0][0][0] == outs[1][0][0]
    assert sum(a == b for a, b in zip(outs[0][0], outs[1][0])) >= 6, outs


@pytest.mark.parametrize("mode", ["hip", "lib"])
def test_prefill_gemm_modes_match_reference_logits(mode, monkeypatch):
    """Prefill projections on the hand-written pgemm (SwiGLU fused into gate/up) or the library:
    the last-token logits of each prompt against the fp32 CPU reference model."""
    cfg = get_config("tiny")

    def _prefill_logits(model, cfg, dev, prompts):
        kv = PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, dev)
        eng = LLMEngine(model, kv, max_prefill_tokens=512, use_graph=False)
        seen = []
        orig_logits = model.logits
        model.logits = lambda h: seen.append(orig_logits(h)) or seen[-1]
        try:
            eng.generate(prompts, max_new_tokens=1, ignore_eos=True)
        finally:
            model.logits = orig_logits
        return seen[0].float().cpu()

    w = DecoderWeights.random(cfg, "cuda", seed=11)
    monkeypatch.setenv("CFC_PREFILL_GEMM", mode)
    m = DecoderModel(w)
    m.PGEMM_MIN_ROWS = 64
    m.PGEMM_MIN_TILES = 0           # tiny shapes: pgemm even where the decode GEMM would be faster
    assert m.prefill_gemm == mode
    prompts = [[1] + list(range(7, 7 + 150)), [1] + list(range(40, 40 + 130)), [1, 5, 9] * 20]
    calls = []
    if mode == "hip":
        from copilot_for_consensus_amd.ops import kernels as K
        orig = K.pgemm
        K.pgemm = lambda *a, **k: calls.append(1) or orig(*a, **k)
    try:
        got = _prefill_logits(m, cfg, "cuda", prompts)
    finally:
        if mode == "hip":
            K.pgemm = orig
    want = _prefill_logits(DecoderModel(_to_cpu_fp32_model(w)), cfg, "cpu", prompts)
    rel = float((got - want).abs().max() / want.abs().max())
    assert rel < 5e-2 and torch.equal(got.argmax(-1), want.argmax(-1)), rel
    assert (len(calls) > 0) == (mode == "hip")
    assert m.w.packed_only == (mode == "hip")       # the hip prefill + dgemm decode keep one weight copy


def test_prefill_beside_decode_on_cu_partitions_matches_generate():
    """Batch B prefilled on half the CUs (worker thread, its own decode state slot) while batch A
    decodes on the other half and widens to the whole GPU when B's prefill is done: both batches'
    tokens equal their plain generate() (greedy)."""
    import concurrent.futures as cf

    from copilot_for_consensus_amd.runtime.cu_partition import partition_streams
    cfg = get_config("tiny")
    w = DecoderWeights.random(cfg, "cuda", seed=7)
    m = DecoderModel(w)
    kv = PagedKVCache(cfg.layers, 160, cfg.kv_heads, cfg.head_dim, "cuda")
    eng = LLMEngine(m, kv, max_prefill_tokens=128)
    A = [[1] + list(range(3, 3 + 70)), [1, 4, 9] * 15, [1] + list(range(100, 160))]
    Bp = [[1] + list(range(200, 290)), [1, 7] * 30, [1] + list(range(11, 51))]
    want_a = eng.generate(A, 24, ignore_eos=True).tokens
    want_b = eng.generate(Bp, 24, ignore_eos=True).tokens
    sp, sd = partition_streams()
    full = torch.cuda.current_stream()
    ja = eng.start(A, 24, ignore_eos=True, slot=0)

    def start_b():
        with torch.cuda.stream(sp):
            return eng.start(Bp, 24, ignore_eos=True, slot=1, stream_sync=True)
    with cf.ThreadPoolExecutor(1) as pool:
        fut = pool.submit(start_b)
        with torch.cuda.stream(sd):
            got_a = eng.finish(ja, switch=lambda: full if fut.done() else None).tokens
        jb = fut.result()
    got_b = eng.finish(jb).tokens
    assert got_a == want_a and got_b == want_b


@pytest.mark.parametrize("use_graph", [False, True])
def test_single_stream_fused_norm_decode_bit_identical(use_graph):
    """B <= 4 decode over packed weights with the residual + RMSNorm reduces folded into the next
    GEMV (K.gemv_norm, two buffers alternating) == the unfused reduce-then-GEMV path, token for token."""
    cfg = get_config("small")
    w = DecoderWeights.random(cfg, "cuda", seed=23)
    m = DecoderModel(w)
    assert m.w.packed_only
    prompts = [[1] + list(range(40, 140)), [1, 5, 9] * 30, [1] + list(range(900, 960))]
    toks = []
    for fused in (True, False):
        m.gemv_norm_fused = fused
        kv = PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, "cuda")
        toks.append(LLMEngine(m, kv, use_graph=use_graph).generate(prompts, 24, ignore_eos=True).tokens)
    assert toks[0] == toks[1]


def test_longest_first_slots_give_every_prompt_the_same_tokens():
    """The engine's longest-first slot order (decode attention list scheduling) is a placement
    only: each prompt's greedy tokens are bit-identical to the caller-order run (the decode GEMMs,
    attention and sampler are row-independent), and come back in the caller's order."""
    cfg = get_config("tiny")
    m = DecoderModel(DecoderWeights.random(cfg, "cuda", seed=5))
    prompts = PROMPTS8 + [[1] + list(range(10, 10 + n)) for n in (3, 90, 41, 160, 12, 77, 5, 120)]
    out = {}
    for lpt in (False, True):
        eng = LLMEngine(m, PagedKVCache(cfg.layers, 128, cfg.kv_heads, cfg.head_dim, "cuda"), max_prefill_tokens=8192)
        eng.lpt = lpt
        r = eng.generate(prompts, 24, ignore_eos=True)
        out[lpt] = (r.tokens, r.prompt_lens)
    assert out[True] == out[False]
    assert out[True][1] == [len(p) for p in prompts]
