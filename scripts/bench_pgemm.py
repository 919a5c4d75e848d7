#!/usr/bin/env python3
"""Prefill / encoder GEMM (csrc/kernels/pgemm.hip) vs the library path on the headline's shapes.

numerics against an fp32 reference, then hipGraph timing (median of 5 replays of 8 calls) of:
  <variant>_*   the hand-written kernel (each K-loop variant) with its fused epilogue;
  lib_*  F.linear (hipBLASLt, TunableOp table when present) + the separate elementwise kernel.
Random [-1, 1)-scale operands (guide §5.4 rule 25: never zero-filled).
Writes one JSON line per shape to gpurun_out/pgemm.jsonl.
"""
import argparse
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

# name: (M, N, K, epi)
SHAPES = {
    "qkv": (16384, 6144, 4096, "bf16"), "o": (16384, 4096, 4096, "bf16"),
    "gate_up": (16384, 28672, 4096, "swiglu"), "down": (16384, 4096, 14336, "bf16"),
    "minilm_qkv": (32768, 1152, 384, "bias"), "minilm_o": (32768, 384, 384, "bf16"),
    "minilm_up": (32768, 1536, 384, "bias_gelu"), "minilm_down": (32768, 384, 1536, "bf16"),
    "bge_qkv": (32768, 2304, 768, "bias"), "bge_up": (32768, 3072, 768, "bias_gelu"),
    "bge_down": (32768, 768, 3072, "bf16"),
}


def timed(fn, calls=8, reps=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(calls):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) / calls)
    return sorted(ts)[len(ts) // 2]


def rel_err(a, ref):
    return float((a.float() - ref.float()).abs().max() / ref.float().abs().max().clamp_min(1e-6))


def lib_fn(x, w, b, epi):
    if epi == "bf16":
        return lambda: F.linear(x, w)
    if epi == "bias":
        return lambda: F.linear(x, w, b)
    if epi == "bias_gelu":
        return lambda: K.bias_gelu(F.linear(x, w), b)
    return lambda: K.silu_mul(F.linear(x, w), interleaved=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="*", default=list(SHAPES))
    ap.add_argument("--m", type=int, default=None, help="override M")
    ap.add_argument("--out", default="gpurun_out/pgemm.jsonl")
    ap.add_argument("--variants", nargs="*", default=["stage2", "pp", "packed"],
                    help="row-major K loops (stage2 / ring5 / ring4 / pp / w4) and 'packed' / 'packed_w4' = "
                         "the ping-pong / 4-wave kernel on the decode GEMM's fragment-packed weight")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    enable_tuned_gemms()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    fh = open(args.out, "a")
    torch.manual_seed(0)
    for name in args.shapes:
        M, N, Kd, epi = SHAPES[name]
        M = args.m or M
        x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
        w = ((torch.rand(N, Kd, device="cuda") * 2 - 1) / Kd ** 0.5).bfloat16()
        b = (torch.rand(N, device="cuda") * 0.2 - 0.1).bfloat16()
        row = {"shape": name, "M": M, "N": N, "K": Kd, "epi": epi}
        # numerics on the first 512 rows (fp32 reference of the same op), every variant
        xs = x[:512].contiguous()
        ref = xs.float() @ w.float().t()
        if epi in ("bias", "bias_gelu"):
            ref = ref + b.float()
        if epi == "bias_gelu":
            ref = F.gelu(ref)
        if epi == "swiglu":
            ref = R.silu_mul_interleaved(ref.bfloat16()).float()
        flops = 2.0 * M * N * Kd
        fns = {"lib": lib_fn(x, w, b, epi)}
        pw = (K.pack_dgemm_weight(w, swiglu=epi == "swiglu") if any(v.startswith("packed") for v in args.variants)
              else None)

        def run(v, xx):
            if v.startswith("packed"):      # packed = ping-pong, packed_w4 = the 4-wave kernel
                return K.pgemm(xx, pw, epi, bias=b, variant=v[7:] or "pp")
            return K.pgemm(xx, w, epi, bias=b, variant=v)
        for v in args.variants:
            row[f"err_{v}"] = rel_err(run(v, xs), ref)
            fns[v] = (lambda v=v: run(v, x))
        # whole-matrix agreement of each variant with the 2-stage kernel (same fp32 sums per tile)
        y0 = K.pgemm(x, w, epi, bias=b, variant="stage2")
        for v in args.variants:
            if v != "stage2":
                row[f"maxdiff_{v}_vs_stage2"] = float((run(v, x).float() - y0.float()).abs().max())
        del y0
        ts = {k: [] for k in fns}
        for _ in range(args.rounds):          # interleaved rounds in one process (guide rule 24)
            for k, fn in fns.items():
                ts[k].append(timed(fn))
        for k, v in ts.items():
            t = sorted(v)[len(v) // 2]
            row[f"{k}_us"] = round(t * 1e6, 1)
            row[f"{k}_TFs"] = round(flops / t / 1e12, 1)
        best = min(args.variants, key=lambda v: row[f"{v}_us"])
        row["best"] = best
        row["speedup_best_vs_lib"] = round(row["lib_us"] / row[f"{best}_us"], 3)
        print(json.dumps(row), flush=True)
        fh.write(json.dumps(row) + "\n")
        fh.flush()
        del x, w, pw
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
