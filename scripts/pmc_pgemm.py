#!/usr/bin/env python3
"""A few dispatches of each prefill-GEMM K-loop variant and the library GEMM at the headline's
gate/up shape (16384 x 28672 x 4096, random operands), for rocprofv3 PMC passes
(scripts/pmc_summary.py averages the counters per kernel)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402

if __name__ == "__main__":
    M, N, Kd = int(os.environ.get("PMC_M", 16384)), 28672, 4096
    x = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
    w = ((torch.rand(N, Kd, device="cuda") * 2 - 1) / Kd ** 0.5).bfloat16()
    for v in ("ring5", "stage2"):
        for _ in range(3):
            K.pgemm(x, w, "bf16", variant=v)
    for _ in range(3):
        F.linear(x, w)
    torch.cuda.synchronize()
    print("pmc_pgemm done")
