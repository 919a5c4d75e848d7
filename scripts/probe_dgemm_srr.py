#!/usr/bin/env python3
"""Decode o / down projection + split-K residual-RMSNorm reduce, in place, per (W rows per
workgroup, split-K) choice: is the cost model's pick (ops/kernels.py dgemm_config) the fastest
PAIR of kernels once the reduce's slab reads are timed where they run?

One config per process (argv: proj bn split, e.g. ``down 128 8``), hipGraph of 24 x [512 MB HBM
sweep (stands in for attention / the next GEMMs) -> dgemm "part" -> splitk_residual_rmsnorm];
run it under ``rocprofv3 --kernel-trace --stats`` (scripts/prof_dgemm_srr.sh) and read the two
kernels' averages.  Without rocprofv3 it prints the graph time per repetition."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402

SHAPES = {"o": (4096, 4096), "down": (4096, 14336), "qkv": (6144, 4096)}
REPS = 24


def main():
    proj, bn, split = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    N, Kd = SHAPES[proj]
    M = 128
    assert N % bn == 0 and (Kd // 64) % split == 0, (N, bn, Kd, split)
    x = (torch.randn(M, Kd, device="cuda") * 0.05).bfloat16()
    w = K.pack_dgemm_weight((torch.randn(N, Kd, device="cuda") * 0.02).bfloat16(), bn=bn)
    part = torch.empty(split, M, N, device="cuda")
    res = torch.randn(M, N, device="cuda").bfloat16()
    nw = torch.ones(N, device="cuda").bfloat16()
    src = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)

    def body():
        dst.copy_(src)
        K.dgemm(x, w, "part", split, part=part)
        K.splitk_residual_rmsnorm(part, res, nw, 1e-5)

    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(REPS):
            body()
    ts = []
    for _ in range(8):
        t = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) / REPS * 1e6)
    print(json.dumps({"proj": proj, "bn": bn, "split": split, "blocks": N // bn * split,
                      "model_pick": K.dgemm_config(M, N, Kd), "graph_us_per_rep": round(sorted(ts)[4], 2)}),
          flush=True)


if __name__ == "__main__":
    main()
