#!/usr/bin/env python3
"""Packed GEMV (gemv_tile_kernel) over a (k-slices, waves per workgroup) grid on the Mistral-7B /
Llama-2-13B decode projections: microseconds per call of the slab form, to fit gemv_packed_config."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402
from bench_gemv import SHAPES, timeit  # noqa: E402


def main():
    for name, (N, Kd) in SHAPES.items():
        copies = max(2, int(1e9 // (N * Kd * 2)))
        ps = [K.pack_dgemm_weight(torch.randn(N, Kd, device="cuda").bfloat16(), swiglu="gate_up" in name)
              for _ in range(copies)]
        nw = ps[0].bn // 16
        for M in (1, 4):
            x = torch.randn(M, Kd, device="cuda").bfloat16()
            it = iter(range(1 << 30))
            rec = {"shape": name, "N": N, "K": Kd, "M": M, "tiles": N // ps[0].bn, "auto": K.gemv_packed_config(N, Kd, nw, M)}
            for sp in (1, 2, 3, 4, 6, 8, 12, 16, 24):
                for wv in ((4, 8, 16) if M == 1 else (4, 8)):
                    if sp > Kd // 32:
                        continue
                    rec[f"s{sp}w{wv}"] = round(timeit(lambda: K.gemv_part(x, ps[next(it) % copies], sp, wv), 100), 1)
            print(json.dumps(rec), flush=True)
        del ps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
