#!/usr/bin/env python3
"""Decode RoPE + paged K/V write at the headline shape (128 tokens, Mistral-7B heads), hipGraph
timing of 64 back-to-back calls: from the qkv split-K slabs (split 4, the decode path), from bf16
qkv, and a one-element kernel as the launch floor."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402
from copilot_for_consensus_amd.ops import reference as R  # noqa: E402


def timed(fn, calls=64, reps=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(calls):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) / calls)
    return sorted(ts)[len(ts) // 2] * 1e6


if __name__ == "__main__":
    T, Hq, Hkv, D, split = 128, 32, 8, 128, 4
    nblk = T * 100
    kc = torch.zeros(nblk, Hkv, 32, D, device="cuda").bfloat16()
    vc = torch.zeros(nblk, Hkv, D, 32, device="cuda").bfloat16()
    pos = torch.randint(2000, 3000, (T,), device="cuda", dtype=torch.int32)
    slots = (torch.randperm(nblk, device="cuda")[:T].int() * 32 + pos % 32).int()
    cs = R.rope_cos_sin(8192, D, 1e6).cuda()
    part = torch.randn(split, T, (Hq + 2 * Hkv) * D, device="cuda")
    qkv = part.sum(0).bfloat16()
    one = torch.zeros(1, device="cuda")
    res = {"part_split4_us": timed(lambda: K.rope_kv_write_part(part, pos, slots, cs, kc, vc, Hq, Hkv, D)),
           "bf16_qkv_us": timed(lambda: K.rope_kv_write(qkv, pos, slots, cs, kc, vc, Hq, Hkv, D)),
           "launch_floor_us": timed(lambda: one.add_(1))}
    print({k: round(v, 2) for k, v in res.items()}, flush=True)
