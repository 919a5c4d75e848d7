#!/usr/bin/env python3
"""Quantized GEMV probe (csrc/kernels/quant.hip): times the Mistral-7B decode projections at M = 1
for prebuilt variants of the kernel library (scripts/probes/build/libquant_<VARIANT>.so, e.g. the
QG_MEMONLY build that keeps the loads and drops the dequant arithmetic), weights rotated over
> 1 GB so every call streams from HBM.

    python scripts/probes/qgemv_probe.py [--variants BASE MEMONLY]
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from copilot_for_consensus_amd.ops.kernels import QWeight  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
SHAPES = [("swiglu", 12, 14336, 4096), ("q", 12, 4096, 4096), ("o_f32", 12, 4096, 4096),
          ("down_q4k_f32", 12, 4096, 14336), ("down_q6k_f32", 14, 4096, 14336), ("lm_head_q6k", 14, 32000, 4096)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="+", default=["BASE", "MEMONLY"])
    ap.add_argument("--configs", nargs="+", default=["0x0"],
                    help="RxKS pairs for cfc_qgemv_config (rows per wave x K split); 0x0 = automatic")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    P, I = ctypes.c_void_p, ctypes.c_int
    x = torch.randn(1, 14336, device="cuda").bfloat16()
    for name, qt, N, K in SHAPES:
        nb = N * (K // 256) * (144 if qt == 12 else 224) * (2 if name == "swiglu" else 1)
        ncopy = max(2, (1 << 30) // nb + 1)
        ws = [(QWeight.random(qt, N, K, "cuda"), QWeight.random(qt, N, K, "cuda") if name == "swiglu" else None)
              for _ in range(ncopy)]
        out = torch.empty(1, N, dtype=torch.float32, device="cuda")
        epi = 2 if name == "swiglu" else (0 if name.endswith("f32") else 1)
        row = {"shape": name, "N": N, "K": K, "MB": round(nb / 1e6, 1)}
        for v, cfgs in [(v, c) for v in a.variants for c in a.configs]:
            lib = ctypes.CDLL(os.path.join(HERE, "build", f"libquant_{v}.so"))
            rr, kk = (int(t) for t in cfgs.split("x"))
            if hasattr(lib, "cfc_qgemv_config"):
                lib.cfc_qgemv_config(rr, kk)
            tag = v if cfgs == "0x0" else f"{v}_{cfgs}"
            fn = lib.cfc_qgemv
            fn.argtypes = [P, I, I, I, I, P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, I, P, P, I, P]
            st = torch.cuda.current_stream().cuda_stream

            def call(i):
                w, w2 = ws[i % ncopy]
                o = tuple(w.offs) + (0,) * 4
                rc = fn(x.data_ptr(), 1, N, K, qt, w.buf.data_ptr(), w2.buf.data_ptr() if w2 is not None else None,
                        o[1], o[2], o[3], epi, out.data_ptr() if epi == 0 else None, out.data_ptr() if epi else None,
                        N, st)
                if rc != 0:
                    raise RuntimeError(rc)
            try:
                call(0)
            except RuntimeError:
                continue
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(a.iters):
                call(i)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.iters
            row[tag + "_us"] = round(us, 2)
            row[tag + "_TBs"] = round(nb / us / 1e6, 2)
        print(json.dumps(row), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
