#!/usr/bin/env python3
"""A few dispatches of each hand-written attention kernel at the headline shapes, for rocprofv3
PMC passes (scripts/pmc_summary.py turns the counter CSVs into profiles/pmc_attention_r01.txt)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench_attn  # noqa: E402  (scripts/bench_attn.py: prefill_case / decode_case)

if __name__ == "__main__":
    bench_attn.prefill_case(iters=3)
    bench_attn.decode_case(iters=3, pbs=(-1,))
