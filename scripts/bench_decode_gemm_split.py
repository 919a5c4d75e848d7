#!/usr/bin/env python3
"""Decode-shape (M = batch) library GEMMs on MI355X: one GEMM vs strided-batched split-K with fp32
partials, for every Mistral-7B projection.  Prints us and the weight-stream rate (TB/s)."""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from copilot_for_consensus_amd.runtime.gemm_tuning import enable_tuned_gemms  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (32000, 4096)}


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    enable_tuned_gemms()
    res = {}
    for M in (128,):
        for name, (N, K) in SHAPES.items():
            # enough weight copies (>= 1 GB) that consecutive calls stream from HBM, not the 256 MB MALL
            nc = max(4, int(1e9 // (N * K * 2)) + 1)
            ws = [torch.randn(N, K, device="cuda").bfloat16() for _ in range(nc)]
            x = torch.randn(M, K, device="cuda").bfloat16()
            i = [0]

            def lin(nc=nc):
                i[0] = (i[0] + 1) % nc
                return F.linear(x, ws[i[0]])
            row = {"lib_us": timeit(lin)}
            for s in (2, 4, 8):
                if K % s or K // s < 512:
                    continue
                part = torch.empty(s, M, N, device="cuda", dtype=torch.float32)
                Ks = K // s

                def bmm(s=s, Ks=Ks, part=part, nc=nc):
                    i[0] = (i[0] + 1) % nc
                    torch.bmm(x.view(M, s, Ks).permute(1, 0, 2), ws[i[0]].view(N, s, Ks).permute(1, 2, 0),
                              out_dtype=torch.float32, out=part)
                row[f"split{s}_us"] = timeit(bmm)
            best = min(v for v in row.values())
            row["lib_TBs"] = N * K * 2 / row["lib_us"] / 1e6
            row["best_TBs"] = N * K * 2 / best / 1e6
            res[f"{name}_M{M}"] = {k: round(v, 2) for k, v in row.items()}
            print(name, M, res[f"{name}_M{M}"], flush=True)
            del ws
    print(json.dumps(res))


if __name__ == "__main__":
    main()
