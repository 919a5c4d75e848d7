#!/usr/bin/env python3
"""Time the prefill and decode attention kernels on Mistral-7B shapes (random data)."""
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402


def prefill_case(nseq=6, L=2800, Hq=32, Hkv=8, D=128, iters=10, fp8=False):
    nb_per = math.ceil(L / 32)
    nblk = nseq * nb_per + 4
    kc = torch.randn(nblk, Hkv, 32, D, device="cuda").bfloat16()
    vc = torch.randn(nblk, Hkv, D, 32, device="cuda").bfloat16()
    if fp8:
        kc, vc = kc.to(torch.float8_e4m3fn), vc.to(torch.float8_e4m3fn)
    perm = torch.randperm(nblk - 4, device="cuda").int()
    bt = perm.view(nseq, nb_per)
    cu = torch.arange(0, nseq + 1, device="cuda", dtype=torch.int32) * L
    ctx = torch.full((nseq,), L, device="cuda", dtype=torch.int32)
    q = torch.randn(nseq * L, Hq, D, device="cuda").bfloat16()
    seqs, q0 = K.prefill_tiles(cu.tolist(), K.prefill_rows(Hq, Hkv), ctx.tolist())
    tiles = (torch.tensor(seqs, dtype=torch.int32, device="cuda"), torch.tensor(q0, dtype=torch.int32, device="cuda"))
    out = torch.empty_like(q)
    for _ in range(2):
        K.prefill_attention(q, kc, vc, bt, cu, ctx, 1 / math.sqrt(D), tiles=tiles, out=out)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        K.prefill_attention(q, kc, vc, bt, cu, ctx, 1 / math.sqrt(D), tiles=tiles, out=out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / iters
    flops = nseq * 4 * (L * (L + 1) / 2) * D * Hq
    print(f"prefill{' fp8-KV' if fp8 else ''} nseq={nseq} L={L}: {dt*1e3:.3f} ms  {flops/dt/1e12:.1f} TFLOP/s "
          "(causal flops)", flush=True)


def decode_case(B=128, L=2900, Hq=32, Hkv=8, D=128, iters=20, fp8=False, pbs=(8, 16, 26, 64)):
    nb_per = math.ceil(L / 32) + 1
    nblk = B * nb_per
    kc = torch.randn(nblk, Hkv, 32, D, device="cuda").bfloat16()
    vc = torch.randn(nblk, Hkv, D, 32, device="cuda").bfloat16()
    if fp8:
        kc, vc = kc.to(torch.float8_e4m3fn), vc.to(torch.float8_e4m3fn)
    bt = torch.randperm(nblk, device="cuda").int().view(B, nb_per)
    ctx = torch.full((B,), L, device="cuda", dtype=torch.int32)
    q = torch.randn(B, Hq, D, device="cuda").bfloat16()
    out = torch.empty_like(q)
    for pb in pbs:
        P = -pb if pb < 0 else math.ceil(nb_per / pb)
        ws = torch.empty(B * Hq * P * (D + 2), device="cuda")
        for _ in range(2):
            K.paged_decode_attention(q, kc, vc, bt, ctx, 1 / math.sqrt(D), out=out, part_blocks=pb, workspace=ws)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(iters):
            K.paged_decode_attention(q, kc, vc, bt, ctx, 1 / math.sqrt(D), out=out, part_blocks=pb, workspace=ws)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / iters
        byts = B * L * Hkv * D * 2 * kc.element_size()
        print(f"decode{' fp8-KV' if fp8 else ''} B={B} L={L} part_blocks={pb}: {dt*1e6:.1f} us  "
              f"{byts/dt/1e12:.2f} TB/s", flush=True)


if __name__ == "__main__":
    prefill_case()
    prefill_case(nseq=1, L=16384)
    decode_case()
    decode_case(B=8)
    if "--fp8" in sys.argv:
        prefill_case(fp8=True)
        prefill_case(nseq=1, L=16384, fp8=True)
        decode_case(fp8=True, pbs=(-1, -2, 26))
        decode_case(B=8, fp8=True, pbs=(-4, -8, 26))
