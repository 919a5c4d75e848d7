#!/usr/bin/env python3
"""Paged decode attention bandwidth study (Mistral-7B shapes, B=128): random vs sequential block
tables, part_blocks sweep.  Run twice (CFC_DECODE_NT=0/1) to compare plain and nontemporal loads."""
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402


def case(B=128, L=2650, Hq=32, Hkv=8, D=128, iters=30, seq=False, pbs=(26, 44, -1, -2, -3, -4)):
    nb_per = math.ceil(L / 32) + 1
    nblk = B * nb_per
    kc = torch.randn(nblk, Hkv, 32, D, device="cuda").bfloat16()
    vc = torch.randn(nblk, Hkv, D, 32, device="cuda").bfloat16()
    ids = torch.arange(nblk, device="cuda") if seq else torch.randperm(nblk, device="cuda")
    bt = ids.int().view(B, nb_per)
    ctx = torch.full((B,), L, device="cuda", dtype=torch.int32)
    q = torch.randn(B, Hq, D, device="cuda").bfloat16()
    out = torch.empty_like(q)
    res = []
    for pb in pbs:
        P = -pb if pb < 0 else math.ceil(nb_per / pb)
        ws = torch.empty(B * Hq * P * (D + 2), device="cuda")
        for _ in range(3):
            K.paged_decode_attention(q, kc, vc, bt, ctx, 1 / math.sqrt(D), out=out, part_blocks=pb, workspace=ws)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(iters):
            K.paged_decode_attention(q, kc, vc, bt, ctx, 1 / math.sqrt(D), out=out, part_blocks=pb, workspace=ws)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / iters
        byts = B * L * Hkv * D * 2 * 2
        res.append(f"pb={pb}:{dt*1e6:.0f}us/{byts/dt/1e12:.2f}TB/s")
    print(f"NT={os.environ.get('CFC_DECODE_NT', '1')} {'seq' if seq else 'rand'} B={B} L={L}: " + "  ".join(res),
          flush=True)


if __name__ == "__main__":
    case(seq=False)
    case(seq=True)
    case(B=64, L=2650, seq=False)
    case(B=8, L=2650, seq=False, pbs=(26, -4, -8, -16, -32))
