#!/usr/bin/env python3
"""One decode-GEMM shape at M = 128 through the ablation entry (cfc_dgemm_ablate), for rocprofv3 PMC
passes: 4 calls on 4 distinct packed weight copies (cold, as in decode).
Usage: pmc_dgemm_abl.py SHAPE ABL   (SHAPE in qkv o gate_up down; ABL 0 = full kernel, 1 = no X DMA)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}

if __name__ == "__main__":
    name, abl = sys.argv[1], int(sys.argv[2])
    N, Kd = SHAPES[name]
    M = 128
    bn, split = K.dgemm_config(M, N, Kd)
    x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
    ws = [K.pack_dgemm_weight(((torch.rand(N, Kd, device="cuda") * 2 - 1) / Kd ** 0.5).bfloat16(), bn=bn)
          for _ in range(4)]
    part = torch.empty(split, M, N, device="cuda", dtype=torch.float32)
    torch.cuda.synchronize()
    for w in ws:
        K.check(K.kernels().cfc_dgemm_ablate(x.data_ptr(), w.data.data_ptr(), M, N, Kd, split, bn, abl,
                                             part.data_ptr(), K._stream(x)), "ablate")
    torch.cuda.synchronize()
    print(name, "bn", bn, "split", split, "abl", abl, flush=True)
