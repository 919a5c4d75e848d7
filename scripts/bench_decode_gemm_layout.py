#!/usr/bin/env python3
"""Decode GEMM (M = 128) weight layout probe: y = x @ W^T with W stored [N, K] (the engine's
layout, "TN") vs W^T stored [K, N] ("NN"), each with TunableOp searching every hipBLASLt/rocBLAS
solution for the shape.  Prints us and weight-stream TB/s; weights rotate over >= 1 GB of copies so
every call streams from HBM."""
import json
import os
import sys
import time

os.environ.setdefault("PYTORCH_TUNABLEOP_ENABLED", "1")
os.environ.setdefault("PYTORCH_TUNABLEOP_TUNING", "1")
os.environ.setdefault("PYTORCH_TUNABLEOP_FILENAME", "gpurun_out/tunableop_layout_probe.csv")
os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS", "300")

import torch  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def graph_us(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    M = 128
    res = {}
    for name, (N, K) in SHAPES.items():
        nc = max(4, int(1e9 // (N * K * 2)) + 1)
        x = torch.randn(M, K, device="cuda").bfloat16()
        w_nk = [torch.randn(N, K, device="cuda").bfloat16() for _ in range(nc)]
        i = [0]

        def tn():
            i[0] = (i[0] + 1) % nc
            return x @ w_nk[i[0]].t()
        row = {"TN_us": graph_us(tn, 4 * nc)}
        del w_nk
        w_kn = [torch.randn(K, N, device="cuda").bfloat16() for _ in range(nc)]

        def nn():
            i[0] = (i[0] + 1) % nc
            return x @ w_kn[i[0]]
        row["NN_us"] = graph_us(nn, 4 * nc)
        del w_kn
        for k in ("TN", "NN"):
            row[f"{k}_TBs"] = N * K * 2 / row[f"{k}_us"] / 1e6
        res[name] = {k: round(v, 2) for k, v in row.items()}
        print(name, res[name], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
