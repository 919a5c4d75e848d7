#!/usr/bin/env python3
"""Decode-shaped projections of Mistral-7B: skinny split-K MFMA GEMM (+ fused epilogues) vs the
library GEMM (hipBLASLt/rocBLAS via F.linear, TunableOp table on).  hipGraph-timed, per call."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from copilot_for_consensus_amd.ops import kernels as K
from copilot_for_consensus_amd.ops import reference as R
from copilot_for_consensus_amd.runtime.gemm_tuning import enable_tuned_gemms

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (32000, 4096)}


def timed(fn, iters=50):
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
    enable_tuned_gemms()
    Ms = [int(a) for a in sys.argv[1:]] or [1, 8, 32, 64, 128, 256]
    res = {}
    for M in Ms:
        for name, (N, Kd) in SHAPES.items():
            x = torch.randn(M, Kd, device="cuda").bfloat16()
            w = (torch.randn(N, Kd, device="cuda") * 0.02).bfloat16()
            wbytes = N * Kd * 2
            lib = timed(lambda: F.linear(x, w))
            row = {"lib_us": round(lib, 1), "lib_TBs": round(wbytes / lib / 1e6, 2)}
            splits = sorted({1, 2, 4, 8, 16, K.skinny_split(M, N, Kd)})
            for s in splits:
                if (Kd // 64) % s:
                    continue
                us = timed(lambda: K.skinny_linear(x, w, split=s))
                row[f"s{s}_us"] = round(us, 1)
            if name == "gate_up":
                wi = R.interleave_gate_up(w)
                row["swiglu_us"] = round(timed(lambda: K.skinny_swiglu(x, wi)), 1)
                row["lib_plus_silu_us"] = round(timed(lambda: K.silu_mul(F.linear(x, wi), interleaved=True)), 1)
            if name in ("o", "down"):
                r = torch.randn(M, N, device="cuda").bfloat16()
                nw = torch.ones(N, device="cuda").bfloat16()
                row["fused_norm_us"] = round(timed(lambda: K.skinny_linear_residual_rmsnorm(x, w, r, nw, 1e-5)), 1)
                row["lib_plus_norm_us"] = round(timed(lambda: K.rmsnorm(F.linear(x, w), nw, 1e-5, residual=r)), 1)
            for S in (2, 4, 8):
                if Kd % S:
                    continue
                Ks = Kd // S
                xa = x.view(M, S, Ks).permute(1, 0, 2)          # [S, M, Ks]
                wb = w.view(N, S, Ks).permute(1, 2, 0)          # [S, Ks, N] (column-major slices)
                part = torch.empty(S, M, N, device="cuda", dtype=torch.float32)
                outb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)

                def bmm_split():
                    torch.bmm(xa, wb, out_dtype=torch.float32, out=part)
                    K.kernels().cfc_splitk_reduce(part.data_ptr(), S, M, N, 0, outb.data_ptr(), N,
                                                  torch.cuda.current_stream().cuda_stream)
                try:
                    row[f"bmm_s{S}_us"] = round(timed(bmm_split), 1)
                    if S == 4:
                        ref = F.linear(x, w).float()
                        row["bmm_err"] = round(float((outb.float() - ref).abs().max()), 4)
                except Exception as e:  # out_dtype / out= combination unsupported
                    row[f"bmm_s{S}_err"] = repr(e)[:80]
            best = min(v for k, v in row.items() if k.startswith("s") and k.endswith("_us"))
            row["best_skinny_TBs"] = round(wbytes / best / 1e6, 2)
            res[f"{name}_M{M}"] = row
            print(f"{name:8s} M={M:4d} {row}", flush=True)
    with open("gpurun_out/skinny_gemm.json", "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
