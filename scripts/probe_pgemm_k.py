#!/usr/bin/env python3
"""Per-tile fixed cost of the prefill GEMM: time the kernel (packed W) at one (M, N) over several K
and fit t = a + b * K -- the intercept a is what every workgroup's prologue (first DMA round trip),
epilogue (store tail) and the launch cost per dispatch, the slope the K loop.  Random operands,
hipGraph timing, interleaved rounds.  One JSON line per (shape, variant, K) and one fit per
(shape, variant).   Usage: probe_pgemm_k.py OUT.jsonl [variant,variant,...]   (default pps)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402
from bench_pgemm import timed  # noqa: E402

KS = (1024, 2048, 4096, 8192)


def fit(rows):
    """least squares t = a + b K over [(K, t)]"""
    n = len(rows)
    sx = sum(k for k, _ in rows)
    sy = sum(t for _, t in rows)
    sxx = sum(k * k for k, _ in rows)
    sxy = sum(k * t for k, t in rows)
    b = (n * sxy - sx * sy) / (n * sxx - sx * sx)
    return (sy - b * sx) / n, b


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pgemm_k.jsonl"
    variants = sys.argv[2].split(",") if len(sys.argv) > 2 else ["pps"]
    fh = open(out, "a")

    def emit(r):
        print(json.dumps(r), flush=True)
        fh.write(json.dumps(r) + "\n")
    torch.manual_seed(0)
    for name, M, N, epi in (("qkv", 16384, 6144, "bf16"), ("gate_up", 16384, 28672, "swiglu")):
        fns = {}
        for Kd in KS:
            x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
            w = ((torch.rand(N, Kd, device="cuda") * 2 - 1) / Kd ** 0.5).bfloat16()
            pw = K.pack_dgemm_weight(w, swiglu=epi == "swiglu")
            del w
            for v in variants:
                fns[(v, Kd)] = (lambda x=x, pw=pw, v=v: K.pgemm(x, pw, epi, variant=v))
        ts = {k: [] for k in fns}
        for _ in range(3):
            for k, fn in fns.items():
                ts[k].append(timed(fn))
        tiles = ((M + 255) // 256) * ((N + 255) // 256)
        for var in variants:
            rows = []
            for Kd in KS:
                t = sorted(ts[(var, Kd)])[1]
                rows.append((Kd, t))
                emit({"shape": name, "variant": var, "M": M, "N": N, "K": Kd, "us": round(t * 1e6, 1),
                      "TFs": round(2.0 * M * N * Kd / t / 1e12, 1)})
            a, b = fit(rows)
            emit({"shape": name, "variant": var, "fit_intercept_us": round(a * 1e6, 1),
                  "slope_us_per_1k": round(b * 1e9, 1), "tile_waves": round(tiles / 256, 2),
                  "intercept_per_tile_wave_us": round(a * 1e6 / (tiles / 256), 2),
                  "K_loop_TFs_from_slope": round(2.0 * M * N / b / 1e12, 1)})
        del fns
        torch.cuda.empty_cache()
