#!/usr/bin/env python3
"""Decode/prefill GEMM shapes of Mistral-7B: hipBLASLt vs rocBLAS (and TunableOp when enabled)."""
import json
import sys
import time

import os

import torch
import torch.nn.functional as F

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (32000, 4096)}


def bench(M, N, K, iters=50):
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16() * 0.02
    for _ in range(5):
        F.linear(x, w)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            F.linear(x, w)
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / iters
    return dt * 1e6, N * K * 2 / dt / 1e12, 2 * M * N * K / dt / 1e12


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else "default"
    Ms = [int(a) for a in sys.argv[2:]] or [1, 8, 32, 64, 128, 256, 16384]
    if lib in ("cublas", "cublaslt"):
        torch.backends.cuda.preferred_blas_library(lib)
    res = {}
    for M in Ms:
        for name, (N, K) in SHAPES.items():
            us, tbs, tf = bench(M, N, K, iters=20 if M > 1000 else 50)
            res[f"{name}_M{M}"] = (round(us, 1), round(tbs, 2), round(tf, 1))
            print(f"{lib:8s} M={M:5d} {name:8s} {us:9.1f} us  {tbs:5.2f} TB/s(w)  {tf:7.1f} TF", flush=True)
    json.dump(res, open(f"gpurun_out/gemm_{lib}.json", "w"))


if __name__ == "__main__":
    main()
