#!/usr/bin/env python3
"""Decode GEMM (dgemm.hip) at the headline's M = 128 on fragment-packed weights, for a rocprofv3
PMC pass: qkv, o, gate_up (+SwiGLU), down, each 3 calls on 3 distinct weight copies (decode reads
every layer's weights once per step and 32 layers do not fit the Infinity Cache, so no call may be
served from a warm copy)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402

SHAPES = {"qkv": (6144, 4096, "part"), "o": (4096, 4096, "part"), "gate_up": (28672, 4096, "swiglu"),
          "down": (4096, 14336, "part")}

if __name__ == "__main__":
    M = 128
    x = {k: (torch.rand(M, kd, device="cuda") * 2 - 1).bfloat16() for k, (n, kd, _) in SHAPES.items()}
    for name, (N, Kd, epi) in SHAPES.items():
        bn, split = K.dgemm_config(M, N, Kd, swiglu=epi == "swiglu")
        ws = [K.pack_dgemm_weight(((torch.rand(N, Kd, device="cuda") * 2 - 1) / Kd ** 0.5).bfloat16(), bn=bn)
              for _ in range(3)]
        torch.cuda.synchronize()
        for w in ws:
            if epi == "swiglu":
                K.dgemm(x[name], w, "swiglu", bn=bn)
            else:
                K.dgemm(x[name], w, "part", split, bn=bn)
        torch.cuda.synchronize()
        print(name, "bn", bn, "split", split, "weight MB", N * Kd * 2 / 1e6, flush=True)
        del ws
    print("pmc_dgemm done")
