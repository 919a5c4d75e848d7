#!/usr/bin/env python3
"""Mid-M GEMM probe: what one weight pass over (decode rows + a prefill chunk) costs on the
existing kernels, against the decode GEMM at M = 128 plus the prefill GEMM at M = chunk.

For every Mistral-7B projection (packed weights, rotated over enough copies that each call reads
its weight from HBM, as a decode step does) this times, in hipGraphs interleaved over rounds in one
process (guide §5.4 rule 24):
  dg<M>   the decode GEMM (dgemm.hip) with the decoder's split / epilogue choice,
  pg<M>   the prefill GEMM (pgemm.hip, "pps"),
  lib<M>  the library GEMM on a row-major copy (reference for what the chip does at that M).
One JSON line per (shape, kernel, M) to gpurun_out/mixed_m.jsonl.
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

SHAPES = {"qkv": (6144, 4096, "bf16"), "o": (4096, 4096, "bf16"), "gate_up": (28672, 4096, "swiglu"),
          "down": (4096, 14336, "bf16")}


def timed(fns, calls=8, reps=5):
    """median seconds per call of the rotating call list ``fns`` replayed from one graph"""
    for f in fns:
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(calls):
            fns[i % len(fns)]()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) / calls)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="*", default=list(SHAPES))
    ap.add_argument("--ms", type=int, nargs="*", default=[128, 256, 512, 640, 768, 896, 1024, 1280, 2048])
    ap.add_argument("--kernels", nargs="*", default=["dg", "pg", "lib"])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/mixed_m.jsonl")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    fh = open(args.out, "a")
    torch.manual_seed(0)
    for name in args.shapes:
        N, Kd, epi = SHAPES[name]
        wbytes = N * Kd * 2
        copies = max(2, -(-600_000_000 // wbytes))
        ws = [((torch.rand(N, Kd, device="cuda") * 2 - 1) / Kd ** 0.5).bfloat16() for _ in range(copies)]
        pws = [K.pack_dgemm_weight(w, swiglu=epi == "swiglu") for w in ws]
        if "lib" not in args.kernels:
            del ws
            ws = None
        xmax = (torch.rand(max(args.ms), Kd, device="cuda") * 2 - 1).bfloat16()
        fns = {}
        for M in args.ms:
            x = xmax[:M]
            if "dg" in args.kernels:
                bn, split = K.dgemm_config(M, N, Kd, swiglu=epi == "swiglu", bn=pws[0].bn)
                if epi == "swiglu":
                    fns[("dg", M)] = [lambda p=p, x=x: K.dgemm(x, p, "swiglu") for p in pws]
                else:
                    fns[("dg", M)] = [lambda p=p, x=x, s=split: K.dgemm(x, p, "part", s) for p in pws]
            if "pg" in args.kernels and M >= 256:
                fns[("pg", M)] = [lambda p=p, x=x: K.pgemm(x, p, epi, variant="pps") for p in pws]
            if "lib" in args.kernels:
                if epi == "swiglu":
                    fns[("lib", M)] = [lambda w=w, x=x: K.silu_mul(F.linear(x, w), interleaved=True) for w in ws]
                else:
                    fns[("lib", M)] = [lambda w=w, x=x: F.linear(x, w) for w in ws]
        ts = {k: [] for k in fns}
        for _ in range(args.rounds):
            for k, f in fns.items():
                ts[k].append(timed(f))
        for (kern, M), v in ts.items():
            t = sorted(v)[len(v) // 2]
            row = {"shape": name, "kernel": kern, "M": M, "N": N, "K": Kd, "us": round(t * 1e6, 1),
                   "TFs": round(2.0 * M * N * Kd / t / 1e12, 1), "W_TBs": round(wbytes / t / 1e12, 2)}
            if kern == "dg":
                row["bn_split"] = K.dgemm_config(M, N, Kd, swiglu=epi == "swiglu", bn=pws[0].bn)
            print(json.dumps(row), flush=True)
            fh.write(json.dumps(row) + "\n")
        fh.flush()
        del pws, ws, xmax, fns
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
