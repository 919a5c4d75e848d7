#!/usr/bin/env python3
"""Decode beside prefill on DISJOINT CU sets (hipExtStreamCreateWithCUMask).

Plain two-stream concurrency of decode steps (HBM-bound: paged attention + M=128 weight-streaming
GEMMs) and prefill GEMMs (MFMA-bound, M=4096) is slower than running them back to back
(bench_overlap.py: 31 ms vs 15.2 + 9.7).  Here each phase gets its own CU partition, so the GEMM
workgroups cannot occupy the CUs the attention kernel streams KV through.  For each split the probe
times decode alone / prefill alone on their partitions and both together.
"""
import ctypes
import json
import math
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def masked_stream(cus: list[int], n_cu: int) -> torch.cuda.ExternalStream:
    words = (n_cu + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in cus:
        mask[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    err = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    assert err == 0, f"hipExtStreamCreateWithCUMask -> {err}"
    return torch.cuda.ExternalStream(s.value)


def main():
    torch.cuda.init()
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    B, L, Hq, Hkv, D = 128, 2900, 32, 8, 128
    nb_per = math.ceil(L / 32) + 1
    kc = torch.randn(B * nb_per, Hkv, 32, D, device="cuda").bfloat16()
    vc = torch.randn(B * nb_per, Hkv, D, 32, device="cuda").bfloat16()
    bt = torch.randperm(B * nb_per, device="cuda").int().view(B, nb_per)
    ctx = torch.full((B,), L, device="cuda", dtype=torch.int32)
    q = torch.randn(B, Hq, D, device="cuda").bfloat16()
    ao = torch.empty_like(q)
    ws = torch.empty(B * Hq * 4 * (D + 2), device="cuda")
    shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
    # distinct weights per layer would not fit the point; 4 layers' worth rotate through the caches
    Ws = [[torch.randn(n, k, device="cuda").bfloat16() for n, k in shapes] for _ in range(4)]
    xd = [torch.randn(128, k, device="cuda").bfloat16() for _, k in shapes]
    xp = [torch.randn(4096, k, device="cuda").bfloat16() for _, k in shapes]

    def dec(layers=32):
        for li in range(layers):
            for x, w in zip(xd, Ws[li % 4]):
                F.linear(x, w)
            K.paged_decode_attention(q, kc, vc, bt, ctx, 1 / math.sqrt(D), out=ao, part_blocks=-1, workspace=ws)

    def pre(layers=8):
        for li in range(layers):
            for x, w in zip(xp, Ws[li % 4]):
                F.linear(x, w)

    def timed(*jobs):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for fn, st in jobs:
            with torch.cuda.stream(st):
                fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3

    full = torch.cuda.Stream()
    for fn in (dec, pre):
        timed((fn, full))
    res = {"n_cu": n_cu, "decode_full_ms": round(min(timed((dec, full)) for _ in range(3)), 2),
           "prefill_full_ms": round(min(timed((pre, full)) for _ in range(3)), 2)}
    res["sequential_ms"] = round(res["decode_full_ms"] + res["prefill_full_ms"], 2)
    print(json.dumps(res), flush=True)
    # partitions: two layouts per fraction, in case CU ids are XCD-major or XCD-interleaved
    parts = {"1/8 mod": lambda c: c % 8 == 0, "1/8 blk": lambda c: (c // 8) % 8 == 0,
             "1/4 mod": lambda c: c % 4 == 0, "1/4 blk": lambda c: (c // 8) % 4 == 0,
             "3/8 mod": lambda c: c % 8 in (0, 3, 5), "1/2 mod": lambda c: c % 2 == 0,
             "1/2 blk": lambda c: (c // 8) % 2 == 0}
    for label, sel in parts.items():
        pre_cus = [c for c in range(n_cu) if sel(c)]
        dec_cus = [c for c in range(n_cu) if c not in set(pre_cus)]
        sd, sp = masked_stream(dec_cus, n_cu), masked_stream(pre_cus, n_cu)
        timed((dec, sd), (pre, sp))
        r = {"split": label, "prefill_cus": len(pre_cus), "decode_cus": len(dec_cus),
             "decode_alone_ms": round(min(timed((dec, sd)) for _ in range(2)), 2),
             "prefill_alone_ms": round(min(timed((pre, sp)) for _ in range(2)), 2)}
        # concurrent: as many prefill rounds as fit beside one decode pass, measured as a rate
        r["both_ms"] = round(min(timed((dec, sd), (pre, sp)) for _ in range(3)), 2)
        r["saved_vs_sequential_ms"] = round(res["sequential_ms"] - r["both_ms"], 2)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
