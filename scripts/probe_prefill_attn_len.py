#!/usr/bin/env python3
"""Prefill attention efficiency vs sequence length at a fixed token count (nseq x L = 16800, the
headline's 16k-token chunks hold ~6 sequences of ~2.7k): hipGraph timing, causal TF/s.  A
persistent-kernel estimate: if per-workgroup overhead dominates at short L, TF/s falls with L."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402
from bench_pgemm import timed  # noqa: E402

Hq, Hkv, D = 32, 8, 128
for nseq, L in ((24, 700), (12, 1400), (6, 2800), (3, 5600), (1, 16800)):
    nb_per = math.ceil(L / 32)
    nblk = nseq * nb_per + 4
    kc = torch.randn(nblk, Hkv, 32, D, device="cuda").bfloat16()
    vc = torch.randn(nblk, Hkv, D, 32, device="cuda").bfloat16()
    bt = torch.randperm(nblk - 4, device="cuda").int().view(nseq, nb_per)
    cu = torch.arange(0, nseq + 1, device="cuda", dtype=torch.int32) * L
    ctx = torch.full((nseq,), L, device="cuda", dtype=torch.int32)
    q = torch.randn(nseq * L, Hq, D, device="cuda").bfloat16()
    seqs, q0 = K.prefill_tiles(cu.tolist(), K.prefill_rows(Hq, Hkv), ctx.tolist())
    tiles = (torch.tensor(seqs, dtype=torch.int32, device="cuda"), torch.tensor(q0, dtype=torch.int32, device="cuda"))
    out = torch.empty_like(q)
    t = timed(lambda: K.prefill_attention(q, kc, vc, bt, cu, ctx, 1 / math.sqrt(D), tiles=tiles, out=out))
    flops = 2.0 * nseq * L * L * D * Hq
    print(f"nseq={nseq} L={L}: {t * 1e6:.1f} us  {flops / t / 1e12:.0f} TF/s  tiles={len(seqs)}", flush=True)
