#!/usr/bin/env python3
"""Decode attention at the headline's shape (B = 128 sequences, ~2.9k-token contexts, Mistral-7B
heads, bf16 KV, one KV partition per sequence as the engine picks at B = 128) for a rocprofv3 PMC
pass: how many bytes the kernel fetches from memory (FETCH_SIZE) against its duration."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402

if __name__ == "__main__":
    B, L, Hq, Hkv, D = 128, 2900, 32, 8, 128
    nb_per = math.ceil(L / 32) + 1
    nblk = B * nb_per
    kc = torch.randn(nblk, Hkv, 32, D, device="cuda").bfloat16()
    vc = torch.randn(nblk, Hkv, D, 32, device="cuda").bfloat16()
    bt = torch.randperm(nblk, device="cuda").int().view(B, nb_per)
    ctx = torch.full((B,), L, device="cuda", dtype=torch.int32)
    q = torch.randn(B, Hq, D, device="cuda").bfloat16()
    out = torch.empty_like(q)
    ws = torch.empty(B * Hq * 1 * (D + 2), device="cuda")
    for _ in range(6):
        K.paged_decode_attention(q, kc, vc, bt, ctx, 1 / math.sqrt(D), out=out, part_blocks=-1, workspace=ws)
    torch.cuda.synchronize()
    print("kv bytes per call", B * L * Hkv * D * 2 * 2, flush=True)
