"""Decoding controls: llama.cpp's default truncation chain (top-k -> top-p -> min-p -> temperature,
what the reference's llama.cpp /completion call runs with), string stop sequences, greedy.  The
CPU reference defines the semantics; the GPU kernel (elementwise.hip: sample_topk_kernel) must
pick only tokens the reference keeps and draw them with the reference's probabilities."""
from __future__ import annotations

import math

import pytest
import torch

from copilot_for_consensus_amd.ops import kernels as K
from copilot_for_consensus_amd.ops import reference as R


def test_truncation_keep_semantics():
    v = torch.tensor([3.0, 2.0, 1.0, 0.0, -1.0])
    p = torch.softmax(v, -1)
    assert R.truncation_keep(v, 1.0, 0.0) == 5
    assert R.truncation_keep(v, float(p[0]) - 1e-6, 0.0) == 1            # top-p reached by the first token
    assert R.truncation_keep(v, float(p[:2].sum()) - 1e-6, 0.0) == 2
    assert R.truncation_keep(v, 1.0, math.exp(-1.5)) == 2                 # min-p: logit >= 3 + ln(min_p) = 1.5
    assert R.truncation_keep(v, 1e-9, 0.9) == 1


def test_reference_sampler_respects_topk():
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(64, 100, generator=g)
    top5 = logits.topk(5, dim=1).indices
    for seed in range(5):
        ids = R.sample_truncated(logits, 1.5, 5, 1.0, 0.0, torch.Generator().manual_seed(seed))
        assert all(int(i) in set(top5[r].tolist()) for r, i in enumerate(ids))
    assert torch.equal(R.sample_truncated(logits, 0.0, 5, 0.9, 0.05), logits.argmax(1).to(torch.int32))


def test_sampling_params_and_cpu_dispatch():
    sp = K.SamplingParams(0.7, 40, 0.95, 0.05)
    assert sp.truncated and not K.SamplingParams(0.0, 40).truncated and K.SamplingParams.of(0.5) == K.SamplingParams(0.5)
    logits = torch.randn(3, 50).bfloat16()
    out = torch.empty(3, dtype=torch.int32)
    K.sample(logits, out, K.SamplingParams(0.7, 1), seed=1, step=torch.zeros(1, dtype=torch.int32))
    assert torch.equal(out, logits.float().argmax(1).to(torch.int32))


def test_engine_topk1_equals_greedy():
    from copilot_for_consensus_amd.models.decoder import DecoderModel, DecoderWeights, get_config
    from copilot_for_consensus_amd.runtime.engine import LLMEngine
    from copilot_for_consensus_amd.runtime.kv_cache import PagedKVCache
    cfg = get_config("tiny")
    eng = LLMEngine(DecoderModel(DecoderWeights.random(cfg, "cpu", seed=3)),
                    PagedKVCache(cfg.layers, 32, cfg.kv_heads, cfg.head_dim, "cpu"))
    p = [[1, 5, 9, 11], [1, 2]]
    greedy = eng.generate(p, 6, ignore_eos=True).tokens
    assert eng.generate(p, 6, temperature=1.3, top_k=1, ignore_eos=True).tokens == greedy


def test_stop_sequences_cut_text():
    from copilot_for_consensus_amd.summarization import HipLLMSummarizer
    s = HipLLMSummarizer.__new__(HipLLMSummarizer)
    s.stop_sequences = ("</s>", "\n\n\n")
    assert s.apply_stops("summary line\n\n\nrambling") == "summary line"
    assert s.apply_stops("a</s>b\n\n\nc") == "a"
    assert s.apply_stops("clean") == "clean"


# ------------------------------------------------------------------ GPU kernel
@pytest.mark.gpu
@pytest.mark.parametrize("V", [50, 32000, 128256])
def test_gpu_truncated_sampler_support(V):
    g = torch.Generator().manual_seed(V)
    logits = (torch.randn(16, V, generator=g) * 3).bfloat16()
    dev = logits.cuda()
    out = torch.empty(16, dtype=torch.int32, device="cuda")
    step = torch.zeros(1, dtype=torch.int32, device="cuda")
    lf = logits.float()
    # top_k = 1 and a tiny top_p collapse to argmax (lowest index among equal maxima)
    for sp in (K.SamplingParams(1.0, 1), K.SamplingParams(1.0, 0, 1e-6)):
        K.sample(dev, out, sp, seed=3, step=step)
        assert torch.equal(out.cpu(), lf.argmax(1).to(torch.int32)), sp
    # min_p = 1 keeps exactly the tokens tied at the maximum (p >= 1.0 * p_max), as llama.cpp does
    K.sample(dev, out, K.SamplingParams(1.0, 0, 1.0, 1.0), seed=3, step=step)
    assert all(lf[r, int(out[r])] == lf[r].max() for r in range(16))
    # sampled ids always inside the reference's kept set
    for seed in range(8):
        sp = K.SamplingParams(1.2, 40, 0.95, 0.05)
        K.sample(dev, out, sp, seed=seed, step=step)
        for r in range(16):
            vals, idx = torch.sort(lf[r], descending=True, stable=True)
            keep = R.truncation_keep(vals[:40], 0.95, 0.05)
            assert int(out[r]) in set(idx[:keep].tolist())


@pytest.mark.gpu
def test_gpu_truncated_sampler_distribution():
    V, rows = 64, 8192
    base = torch.linspace(2.0, -2.0, V)
    logits = base.repeat(rows, 1).bfloat16().cuda()   # same distribution on every row, row index salts the RNG
    out = torch.empty(rows, dtype=torch.int32, device="cuda")
    sp = K.SamplingParams(0.8, 8, 0.9, 0.0)
    K.sample(logits, out, sp, seed=11, step=torch.zeros(1, dtype=torch.int32, device="cuda"))
    vals = base.bfloat16().float()
    keep = R.truncation_keep(vals[:8], 0.9, 0.0)
    want = torch.softmax(vals[:keep] / 0.8, -1)
    counts = torch.bincount(out.cpu().long(), minlength=V).float() / rows
    assert counts[keep:].sum() == 0
    assert float((counts[:keep] - want).abs().max()) < 0.02, (counts[:keep], want)


@pytest.mark.gpu
def test_gpu_truncated_sampler_ties_take_lowest_indices():
    logits = torch.zeros(4, 32000, dtype=torch.bfloat16, device="cuda")
    logits[1, 31999] = 1.0        # one strictly larger element at the very end
    out = torch.empty(4, dtype=torch.int32, device="cuda")
    for seed in range(6):
        K.sample(logits, out, K.SamplingParams(1.0, 40, 1.0, 0.0), seed=seed,
                 step=torch.zeros(1, dtype=torch.int32, device="cuda"))
        o = out.cpu().tolist()
        assert o[0] < 40 and o[2] < 40 and o[3] < 40, o
        assert o[1] == 31999 or o[1] < 39, o   # the larger one + the 39 lowest-index ties
