#!/usr/bin/env python3
"""Prefill projections at short chunk lengths: pgemm (256 x 256 tiles) vs the decode GEMM
(dgemm, one W pass per 256-row tile) on the packed Mistral-7B weights, M = 256 .. 16384 --
microseconds per call, to fit DecoderModel._dgemm_faster."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402
from bench_gemv import timeit  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def main():
    for name, (N, Kd) in SHAPES.items():
        sw = name == "gate_up"
        pw = K.pack_dgemm_weight(torch.randn(N, Kd, device="cuda").bfloat16() / Kd ** 0.5, swiglu=sw)
        for M in (256, 512, 1024, 2048, 4096, 8192, 16384):
            x = torch.randn(M, Kd, device="cuda").bfloat16()
            tp = timeit(lambda: K.pgemm(x, pw, "swiglu" if sw else "bf16", variant="pps"), 20)
            td = timeit(lambda: K.dgemm_swiglu(x, pw) if sw else K.dgemm_linear(x, pw), 20)
            fl = 2 * M * N * Kd
            print(json.dumps({"shape": name, "M": M, "pgemm_us": round(tp, 1), "dgemm_us": round(td, 1),
                              "pgemm_TFs": round(fl / tp / 1e6, 1), "dgemm_TFs": round(fl / td / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
