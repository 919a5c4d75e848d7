#!/usr/bin/env python3
"""Does a block-table prefix shared by every sequence already come from the caches?

Paged decode attention at the headline shape (B=128, ~2.8k context, Mistral-7B heads) with the
first S blocks of every block table pointing at the SAME physical blocks (what the prefix cache
produces for the common system prompt) against fully distinct tables.  If the shared rows were
served from the Infinity Cache the kernel time would drop by ~S/blocks; if not, a cascade
(shared-prefix-once) decode kernel has that fraction to win.
"""
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402


def run(B=128, L=2830, shared=0, Hq=32, Hkv=8, D=128, iters=40, layers=4):
    nb = math.ceil(L / 32)
    nblk = B * nb + 8
    # several "layers" of cache so consecutive calls do not re-read the same bytes
    kcs = [torch.randn(nblk, Hkv, 32, D, device="cuda").bfloat16() for _ in range(layers)]
    vcs = [torch.randn(nblk, Hkv, D, 32, device="cuda").bfloat16() for _ in range(layers)]
    ids = torch.randperm(nblk, device="cuda")[: B * nb].int().view(B, nb)
    if shared:
        ids[:, :shared] = ids[0, :shared]
    ctx = torch.full((B,), L, device="cuda", dtype=torch.int32)
    q = torch.randn(B, Hq, D, device="cuda").bfloat16()
    out = torch.empty_like(q)
    ws = torch.empty(B * Hq * 1 * (D + 2), device="cuda")
    for i in range(3):
        K.paged_decode_attention(q, kcs[i % layers], vcs[i % layers], ids, ctx, 1 / math.sqrt(D), out=out,
                                 part_blocks=-1, workspace=ws)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(iters):
        K.paged_decode_attention(q, kcs[i % layers], vcs[i % layers], ids, ctx, 1 / math.sqrt(D), out=out,
                                 part_blocks=-1, workspace=ws)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / iters
    byts = B * L * Hkv * D * 4
    uniq = B * (L - 32 * shared) * Hkv * D * 4 + shared * 32 * Hkv * D * 4
    print(f"B={B} L={L} shared_blocks={shared}/{nb}: {dt * 1e6:.1f} us  "
          f"{byts / dt / 1e12:.2f} TB/s logical  {uniq / dt / 1e12:.2f} TB/s unique", flush=True)
    return dt


if __name__ == "__main__":
    base = run(shared=0)
    for s in (10, 20, 40):
        d = run(shared=s)
        print(f"  -> {100 * (1 - d / base):.1f}% faster than distinct (ideal {100 * s / math.ceil(2830 / 32):.1f}%)")
