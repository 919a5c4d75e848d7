#!/usr/bin/env python3
"""GEMV (gemm.hip: gemv_kernel) vs hipBLASLt (F.linear) on the Mistral-7B / Llama-2-13B decode
projections at M = 1..4: microseconds per call and achieved weight-stream bandwidth; plus the
packed-weight GEMV (gemv_tile_kernel, the layout the model keeps) at several workgroup targets."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "13b_qkv": (15360, 5120), "13b_gate_up": (27648, 5120), "13b_down": (5120, 13824)}


def timeit(fn, iters=200):
    for _ in range(10):
        fn()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters


def main():
    # one weight set per shape, several copies so consecutive calls do not hit the 256 MB MALL
    for name, (N, Kd) in SHAPES.items():
        copies = max(2, int(1e9 // (N * Kd * 2)))
        ws = [torch.randn(N, Kd, device="cuda").bfloat16() for _ in range(copies)]
        ps = [K.pack_dgemm_weight(w, swiglu="gate_up" in name) for w in ws]
        for M in (1, 2, 4):
            x = torch.randn(M, Kd, device="cuda").bfloat16()
            it = iter(range(1 << 30))
            lib = timeit(lambda: torch.nn.functional.linear(x, ws[next(it) % copies]))
            epi = "swiglu" if "gate_up" in name else "bf16"
            gv = timeit(lambda: K.gemv(x, ws[next(it) % copies], epi))
            tb = N * Kd * 2 / 1e6
            rec = {"shape": name, "N": N, "K": Kd, "M": M, "lib_us": round(lib, 1), "gemv_us": round(gv, 1),
                   "lib_TB_s": round(tb / lib, 2), "gemv_TB_s": round(tb / gv, 2)}
            # packed weight (the copy the model keeps): split 1 with the epilogue in-kernel at 4 / 8 / 16
            # waves per workgroup, and the k-slice slab form over (split, waves) plus its consumer (the
            # residual + RMSNorm reduce, one workgroup per row, as o / down run it)
            nw = ps[0].bn // 16
            for wv in ((4, 8, 16) if M == 1 else (4, 8)):
                pv = timeit(lambda: K.gemv(x, ps[next(it) % copies], epi, waves=wv))
                rec[f"s1w{wv}_us"] = round(pv, 1)
            auto = K.gemv_packed_config(N, Kd, nw, M)
            rec["auto"] = auto
            cfgs = {auto, (auto[0] * 2, 4), (auto[0] * 2, auto[1]), (max(1, auto[0] // 2), min(auto[1] * 2, 16 if M == 1 else 8))}
            res = torch.zeros(M, N, device="cuda").bfloat16()
            nrm = torch.ones(N, device="cuda").bfloat16()
            for sp, wv in sorted(cfgs):
                if sp > Kd // 32:
                    continue
                pv = timeit(lambda: K.gemv_part(x, ps[next(it) % copies], sp, wv))
                part = K.gemv_part(x, ps[0], sp, wv)
                if epi == "swiglu" or N // 8 > 1024:   # qkv-like: the slab RoPE reads them instead
                    red = timeit(lambda: K.splitk_reduce(part, swiglu=epi == "swiglu"))
                else:
                    red = timeit(lambda: K.splitk_residual_rmsnorm(part, res, nrm, 1e-5))
                rec[f"slab_s{sp}w{wv}"] = [round(pv, 1), round(red, 1)]
            print(json.dumps(rec), flush=True)
        del ws, ps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
