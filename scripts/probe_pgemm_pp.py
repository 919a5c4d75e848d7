#!/usr/bin/env python3
"""Ping-pong prefill GEMM probes (csrc/kernels/pgemm.hip cfc_pgemm_probe): priority schemes and the
tile-order group size, A/B against the library in interleaved rounds in one process (guide §5.4 rule
24), random operands (rule 25), packed weights.  One JSON line per shape to --out.

    python scripts/probe_pgemm_pp.py                 # timing
    python scripts/probe_pgemm_pp.py --pmc qkv       # a few dispatches for rocprofv3 --pmc passes
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402
from copilot_for_consensus_amd.ops._native import kernels  # noqa: E402
from copilot_for_consensus_amd.runtime.gemm_tuning import enable_tuned_gemms  # noqa: E402

SHAPES = {"qkv": (16384, 6144, 4096), "o": (16384, 4096, 4096), "gate_up": (16384, 28672, 4096),
          "down": (16384, 4096, 14336)}
PROBES = {"pf0_g8": (0, 8), "pf1_g8": (1, 8), "w1e_g8": (33, 8), "stg_g8": (97, 8), "pf2_g8": (2, 8), "pf0_g4": (0, 4), "pf0_g16": (0, 16),
          # ablations (wrong results by construction; timing only): no DMA / no ds_read / no MFMA
          "abl_nodma": (5, 8), "abl_noread": (9, 8), "abl_mfma_only": (13, 8), "abl_nomfma": (17, 8),
          "abl_read_only": (21, 8)}
ABLATIONS = {k for k in PROBES if k.startswith("abl_")}


def probe(x, pw, out, pf, gm):
    M, Kd = x.shape
    rc = kernels().cfc_pgemm_probe(x.data_ptr(), pw.data.data_ptr(), out.data_ptr(), M, pw.N, Kd, pw.bn // 16, pf, gm,
                                   ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    if rc:
        raise RuntimeError(f"cfc_pgemm_probe rc={rc}")


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="*", default=list(SHAPES))
    ap.add_argument("--probes", nargs="*", default=list(PROBES))
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--pmc", default=None, help="shape: run 3 dispatches of each probe + the library, no timing")
    ap.add_argument("--out", default="gpurun_out/pgemm_probe.jsonl")
    args = ap.parse_args()
    enable_tuned_gemms()
    torch.manual_seed(0)
    for name in ([args.pmc] if args.pmc else args.shapes):
        M, N, Kd = SHAPES[name]
        x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
        w = ((torch.rand(N, Kd, device="cuda") * 2 - 1) / Kd ** 0.5).bfloat16()
        pw = K.pack_dgemm_weight(w)
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        ref = F.linear(x, w)
        fns = {"lib": lambda: F.linear(x, w)}
        row = {"shape": name, "M": M, "N": N, "K": Kd, "bn": pw.bn}
        for p in args.probes:
            pf, gm = PROBES[p]
            out.zero_()
            probe(x, pw, out, pf, gm)
            if p not in ABLATIONS:
                row[f"maxdiff_{p}"] = float((out.float() - ref.float()).abs().max())
            fns[p] = (lambda pf=pf, gm=gm: probe(x, pw, out, pf, gm))
        if args.pmc:
            for fn in fns.values():
                for _ in range(3):
                    fn()
            torch.cuda.synchronize()
            print("pmc probe done", flush=True)
            return
        ts = {k: [] for k in fns}
        for _ in range(args.rounds):
            for k, fn in fns.items():
                ts[k].append(timed(fn))
        flops = 2.0 * M * N * Kd
        for k, v in ts.items():
            t = sorted(v)[len(v) // 2]
            row[f"{k}_us"] = round(t * 1e6, 1)
            row[f"{k}_TFs"] = round(flops / t / 1e12, 1)
        print(json.dumps(row), flush=True)
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "a") as fh:
            fh.write(json.dumps(row) + "\n")
        del x, w, pw, out, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
