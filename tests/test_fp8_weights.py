"""Opt-in W8A8 FP8 projections (OCP e4m3fn on gfx950's MFMA FP8 path): the per-token activation
quantisation kernel against its fp32 reference, linear_fp8 against an fp32 GEMM, and a decoder
whose projections run in FP8 against the same decoder in bf16 (CPU reference path + MI355X)."""
from __future__ import annotations

import pytest
import torch

from copilot_for_consensus_amd.models.decoder import DecoderModel, DecoderWeights, get_config
from copilot_for_consensus_amd.ops import kernels as K
from copilot_for_consensus_amd.ops import reference as ref
from copilot_for_consensus_amd.runtime.engine import LLMEngine
from copilot_for_consensus_amd.runtime.kv_cache import PagedKVCache


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


def test_fp8_reference_and_linear_cpu():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(33, 256, generator=g).bfloat16()
    x8, s = ref.quant_fp8_rows(x)
    assert x8.dtype == torch.float8_e4m3fn and s.shape == (33, 1)
    assert float(x8.float().abs().amax(1).min()) == 448.0           # every row uses the full range
    assert _rel(x8.float() * s, x) < 0.04
    w = torch.randn(96, 256, generator=g).bfloat16()
    w8, ws = K.quant_fp8_weight(w)
    assert ws.shape == (1, 96)
    y = K.linear_fp8(x, w8, ws)
    assert y.dtype == torch.bfloat16 and _rel(y, x.float() @ w.float().T) < 0.06


def test_fused_quant_ops_cpu():
    g = torch.Generator().manual_seed(4)
    x = torch.randn(6, 512, generator=g).bfloat16()
    w = (1 + 0.1 * torch.randn(512, generator=g)).bfloat16()
    r1, r2 = torch.randn(6, 512, generator=g).bfloat16(), None
    r2 = r1.clone()
    x8, s = K.rmsnorm_fp8(x, w, 1e-5, residual=r1)
    e8, es = ref.quant_fp8_rows(K.rmsnorm(x, w, 1e-5, residual=r2))
    assert torch.equal(r1, r2) and torch.equal(s, es) and torch.equal(x8.float(), e8.float())
    gu = torch.randn(6, 2 * 256, generator=g).bfloat16()
    a8, sa = K.silu_mul_fp8(gu, interleaved=True)
    b8, sb = ref.quant_fp8_rows(K.silu_mul(gu, interleaved=True))
    assert torch.equal(sa, sb) and torch.equal(a8.float(), b8.float())
    wl = torch.randn(64, 512, generator=g).bfloat16()
    wq, ws = K.quant_fp8_weight(wl)
    assert torch.equal(K.linear_fp8((x8, s), wq, ws), K.linear_fp8((e8, es), wq, ws))


def _models(device, seed=3):
    cfg = get_config("tiny")
    wb = DecoderWeights.random(cfg, device, seed=seed)
    w8 = DecoderWeights.random(cfg, device, seed=seed).to_fp8()
    assert all(layer["qkv"] is None for layer in w8.layers) and w8.nbytes() < wb.nbytes()
    return cfg, DecoderModel(wb), DecoderModel(w8)


def _prefill_logits(cfg, model, device):
    kv = PagedKVCache(cfg.layers, 64, model.w.kv_heads, cfg.head_dim, device)
    eng = LLMEngine(model, kv, prefix_cache=False)
    prompt = [1] + [(7 * i) % 500 + 3 for i in range(90)]
    res = eng.generate([prompt], 6, temperature=0.0, ignore_eos=True)
    return res.tokens[0]


def test_fp8_decoder_cpu():
    cfg, mb, m8 = _models("cpu")
    assert m8.fp8 and m8.decode_gemm == "lib" and not m8.decode_gemv
    # prefill hidden states close to bf16; generation runs end to end
    ids = torch.tensor([1, 5, 9, 13, 17, 21, 25, 29], dtype=torch.int32)
    hb = mb.w.embed[ids]
    assert hb.shape[0] == 8
    assert len(_prefill_logits(cfg, m8, "cpu")) == 6


@pytest.mark.gpu
def test_quant_fp8_rows_kernel_matches_reference():
    g = torch.Generator(device="cuda").manual_seed(1)
    for M, Kd in ((1, 4096), (128, 4096), (77, 14336), (3, 28672), (5, 8)):
        x = (torch.randn(M, Kd, device="cuda", generator=g) * 3).bfloat16()
        x[0, 0] = 0.0
        x8, s = K.quant_fp8_rows(x)
        r8, rs = ref.quant_fp8_rows(x)
        torch.testing.assert_close(s, rs, rtol=1e-6, atol=0)
        # x * (1/s) vs x / s can round one fp8 step apart on a tie; nothing more
        diff = (x8.float() - r8.float()).abs()
        step = r8.float().abs().clamp_min(2 ** -6) / 8
        assert bool((diff <= step + 1e-6).all()) and float((diff > 0).float().mean()) < 0.01
    z8, zs = K.quant_fp8_rows(torch.zeros(2, 64, device="cuda", dtype=torch.bfloat16))
    assert float(zs.min()) == 1.0 and float(z8.float().abs().max()) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("rows,dim", [(1, 4096), (128, 4096), (37, 8192), (4, 64), (200, 5120)])
def test_rmsnorm_fp8_kernel_matches_unfused(rows, dim):
    g = torch.Generator(device="cuda").manual_seed(rows)
    x = torch.randn(rows, dim, device="cuda", generator=g).bfloat16()
    w = (1 + 0.1 * torch.randn(dim, device="cuda", generator=g)).bfloat16()
    res = torch.randn(rows, dim, device="cuda", generator=g).bfloat16()
    r1, r2 = res.clone(), res.clone()
    x8, s = K.rmsnorm_fp8(x, w, 1e-5, residual=r1)
    e8, es = K.quant_fp8_rows(K.rmsnorm(x, w, 1e-5, residual=r2))
    assert torch.equal(r1, r2)
    torch.testing.assert_close(s, es, rtol=1e-6, atol=0)
    assert float((x8.float() != e8.float()).float().mean()) < 1e-3
    # and against the fp32 reference of the whole op
    rn, _ = ref.rmsnorm(x.float(), w.float(), 1e-5, res.float())
    assert _rel(x8.float() * s, rn) < 0.04
    n8, ns = K.rmsnorm_fp8(x, w, 1e-5)
    f8, fs = K.quant_fp8_rows(K.rmsnorm(x, w, 1e-5))
    torch.testing.assert_close(ns, fs, rtol=1e-6, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("T,F,inter", [(1, 14336, True), (128, 14336, True), (33, 4096, False), (3, 28672, False)])
def test_silu_mul_fp8_kernel_matches_unfused(T, F, inter):
    g = torch.Generator(device="cuda").manual_seed(T + F)
    gu = (torch.randn(T, 2 * F, device="cuda", generator=g) * 2).bfloat16()
    a8, s = K.silu_mul_fp8(gu, interleaved=inter)
    b8, sb = K.quant_fp8_rows(K.silu_mul(gu, interleaved=inter))
    torch.testing.assert_close(s, sb, rtol=1e-6, atol=0)
    assert float((a8.float() != b8.float()).float().mean()) < 1e-3
    want = ref.silu_mul_interleaved(gu.float()) if inter else ref.silu_mul(gu.float())
    assert _rel(a8.float() * s, want) < 0.04


@pytest.mark.gpu
def test_linear_fp8_gpu_vs_fp32():
    g = torch.Generator(device="cuda").manual_seed(2)
    for M, N, Kd in ((128, 6144, 4096), (1000, 512, 1024), (4, 28672, 4096)):
        x = torch.randn(M, Kd, device="cuda", generator=g).bfloat16()
        w = (torch.randn(N, Kd, device="cuda", generator=g) * 0.02).bfloat16()
        w8, ws = K.quant_fp8_weight(w)
        y = K.linear_fp8(x, w8, ws)
        assert _rel(y, x.float() @ w.float().T) < 0.05


@pytest.mark.gpu
def test_fp8_decoder_gpu_tracks_bf16():
    cfg, mb, m8 = _models("cuda")
    kvb = PagedKVCache(cfg.layers, 64, mb.w.kv_heads, cfg.head_dim, "cuda")
    kv8 = PagedKVCache(cfg.layers, 64, m8.w.kv_heads, cfg.head_dim, "cuda")
    prompt = [1] + [(11 * i) % 500 + 3 for i in range(150)]
    eb = LLMEngine(mb, kvb, prefix_cache=False)
    e8 = LLMEngine(m8, kv8, prefix_cache=False)
    rb = eb.generate([prompt, prompt[:70]], 8, temperature=0.0, ignore_eos=True)
    r8 = e8.generate([prompt, prompt[:70]], 8, temperature=0.0, ignore_eos=True)
    assert [len(t) for t in r8.tokens] == [8, 8]
    # decode logits of the same context: FP8 projections stay close to bf16
    ids = torch.tensor(prompt[:64], dtype=torch.int32, device="cuda")
    xb = mb.logits(_hidden(mb, kvb, ids)).float()
    x8 = m8.logits(_hidden(m8, kv8, ids)).float()
    assert _rel(x8, xb) < 0.12


def _hidden(model, kv, ids):
    T = ids.shape[0]
    dev = ids.device
    bt = torch.arange(4, dtype=torch.int32, device=dev)[None]
    slots = torch.arange(T, dtype=torch.int32, device=dev)
    pos = torch.arange(T, dtype=torch.int32, device=dev)
    cu = torch.tensor([0, T], dtype=torch.int32, device=dev)
    ctx = torch.tensor([T], dtype=torch.int32, device=dev)
    return model.forward_prefill(ids, pos, slots, cu, ctx, bt, kv, last_idx=torch.tensor([T - 1], device=dev))
