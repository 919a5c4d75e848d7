#!/usr/bin/env python3
"""Where rope_kv's 10.9 us in the decode step goes (~5 us alone).

Each variant is a hipGraph of 24 repetitions of [HBM sweep (stands in for the attention kernel
that evicts L2 / MALL between layers) -> qkv decode GEMM -> rope_kv variant]; a variant's cost is
its graph time minus the graph without the rope_kv launch, i.e. its marginal time in a step.

  part        : the decode path (fp32 split-K slabs in, RoPE, K and V cache writes)
  part_noKV   : same reads and q writes, slots = -1 (no cache writes)
  bf16        : bf16 qkv in (the GEMM's bf16 epilogue instead of slabs), K and V writes
  bf16_noV    : bf16 qkv in, K writes only (V skipped)
  bf16_noKV   : bf16 qkv in, no cache writes
  part_vwt / part_vnt : the decode path with write-through / nontemporal V stores
Prints one JSON line per variant; argv: run only the named variants (one per process under rocprofv3,
whose per-kernel durations cannot tell two calls of one kernel apart)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402
from copilot_for_consensus_amd.ops import reference as R  # noqa: E402

REPS = 24


def graph_us(body, reps=5):
    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(REPS):
            body()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) / REPS)
    return sorted(ts)[len(ts) // 2] * 1e6


def main():
    T, Hq, Hkv, D, Kd = 128, 32, 8, 128, 4096
    N = (Hq + 2 * Hkv) * D
    nblk = T * 100
    kc = torch.zeros(nblk, Hkv, 32, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.zeros(nblk, Hkv, D, 32, device="cuda", dtype=torch.bfloat16)
    pos = torch.randint(2000, 3000, (T,), device="cuda", dtype=torch.int32)
    slots = (torch.randperm(nblk, device="cuda")[:T].int() * 32 + pos % 32).int()
    noslots = torch.full_like(slots, -1)
    cs = R.rope_cos_sin(8192, D, 1e6).cuda()
    x = (torch.randn(T, Kd, device="cuda") * 0.05).bfloat16()
    w = K.pack_dgemm_weight((torch.randn(N, Kd, device="cuda") * 0.02).bfloat16())
    bn, split = K.dgemm_config(T, N, Kd, bn=w.bn)
    part = torch.empty(split, T, N, device="cuda")
    qkv = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
    q_out = torch.empty(T, Hq, D, device="cuda", dtype=torch.bfloat16)
    src = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    no_runs = torch.zeros(0, 4, dtype=torch.int32, device="cuda")

    def sweep():
        dst.copy_(src)

    def gemm_part():
        K.dgemm(x, w, "part", split, part=part)

    def gemm_bf16():
        K.dgemm(x, w, "bf16", out=qkv)

    variants = {
        "part": (gemm_part, lambda: K.rope_kv_write_part(part, pos, slots, cs, kc, vc, Hq, Hkv, D)),
        "part_noKV": (gemm_part, lambda: K.rope_kv_write_part(part, pos, noslots, cs, kc, vc, Hq, Hkv, D)),
        "bf16": (gemm_bf16, lambda: K.rope_kv_write(qkv, pos, slots, cs, kc, vc, Hq, Hkv, D, q_out=q_out)),
        "bf16_noV": (gemm_bf16, lambda: K.rope_kv_write(qkv, pos, slots, cs, kc, vc, Hq, Hkv, D, q_out=q_out,
                                                       runs=no_runs)),
        "bf16_noKV": (gemm_bf16, lambda: K.rope_kv_write(qkv, pos, noslots, cs, kc, vc, Hq, Hkv, D, q_out=q_out)),
    }
    variants["part_vwt"] = variants["part_vnt"] = variants["part"]
    modes = {"part_vwt": 1, "part_vnt": 2}
    base = {}
    only = sys.argv[1:]
    for name, (gemm, rope) in variants.items():
        if only and name not in only:
            continue
        K.set_kv_vstore_mode(modes.get(name, 0))
        key = gemm.__name__
        if key not in base:
            base[key] = graph_us(lambda: (sweep(), gemm()))
        tot = graph_us(lambda: (sweep(), gemm(), rope()))
        alone = graph_us(rope) if not only else float("nan")     # profiled: in-step calls only
        print(json.dumps({"variant": name, "split": split, "bn": bn, "base_us": round(base[key], 2),
                          "with_rope_us": round(tot, 2), "rope_marginal_us": round(tot - base[key], 2),
                          "rope_alone_us": round(alone, 2)}), flush=True)


if __name__ == "__main__":
    main()
