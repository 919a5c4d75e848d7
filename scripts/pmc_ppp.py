#!/usr/bin/env python3
"""Dispatches for rocprofv3 PMC passes of the prefill GEMM at the headline's qkv and gate_up shapes
(16k rows, random operands): the persistent kernel ("ppp"), the one-tile ping-pong kernel ("pps")
and the library GEMM (F.linear on a row-major copy), three dispatches each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402

if __name__ == "__main__":
    for N, epi in ((6144, "bf16"), (28672, "swiglu")):
        M, Kd = 16384, 4096
        x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
        w = ((torch.rand(N, Kd, device="cuda") * 2 - 1) / Kd ** 0.5).bfloat16()
        pw = K.pack_dgemm_weight(w, swiglu=epi == "swiglu")
        for v in ("ppp", "pps"):
            for _ in range(3):
                K.pgemm(x, pw, epi, variant=v)
        for _ in range(3):
            F.linear(x, w)
        torch.cuda.synchronize()
        del x, w, pw
        torch.cuda.empty_cache()
    print("pmc_ppp done", flush=True)
