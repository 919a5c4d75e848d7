#!/usr/bin/env python3
"""Persistent prefill GEMM probes (cfc_pgemm_ppp_probe), A/B interleaved in one process on the
headline's four 16k-row shapes (random operands, hipGraph timing): the tile-order group gm (M-tiles
per N sweep; "s<gm>" = the same with register-direct instead of LDS-staged epilogue stores).
Usage: probe_ppp_gm.py OUT.jsonl 2,4,8,16 | 8,s8 ...   One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402
from bench_pgemm import SHAPES, timed  # noqa: E402

if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ppp_gm.jsonl"
    gms = (sys.argv[2] if len(sys.argv) > 2 else "2,4,8,16").split(",")
    fh = open(out, "a")
    torch.manual_seed(0)
    for name in ("qkv", "o", "gate_up", "down"):
        M, N, Kd, epi = SHAPES[name]
        x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
        w = ((torch.rand(N, Kd, device="cuda") * 2 - 1) / Kd ** 0.5).bfloat16()
        pw = K.pack_dgemm_weight(w, swiglu=epi == "swiglu")
        del w
        oc = N // 2 if epi == "swiglu" else N
        y = torch.empty(M, oc, device="cuda", dtype=torch.bfloat16)
        ref = K.pgemm(x, pw, epi, variant="ppp").clone()

        def run(gm):
            direct = gm.startswith("s")
            K.check(K.kernels().cfc_pgemm_ppp_probe(x.data_ptr(), pw.data.data_ptr(), y.data_ptr(), M, N, Kd,
                                                   (3 if epi == "swiglu" else 0) | (16 if direct else 0), oc,
                                                   pw.bn // 16, int(gm.lstrip("s")), K._stream(x)),
                    "cfc_pgemm_ppp_probe")
        row = {"shape": name, "M": M, "N": N, "K": Kd, "tiles_n": (N + 255) // 256}
        for gm in gms:
            run(gm)
            torch.cuda.synchronize()
            row[f"maxdiff_gm{gm}"] = float((y.float() - ref.float()).abs().max())
        ts = {gm: [] for gm in gms}
        for _ in range(3):
            for gm in gms:
                ts[gm].append(timed(lambda gm=gm: run(gm)))
        for gm in gms:
            row[f"gm{gm}_us"] = round(sorted(ts[gm])[1] * 1e6, 1)
        print(json.dumps(row), flush=True)
        fh.write(json.dumps(row) + "\n")
        del x, pw, y, ref
        torch.cuda.empty_cache()
