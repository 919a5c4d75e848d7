#!/usr/bin/env python3
"""Can a prefill chunk (compute-bound GEMMs) run beside decode steps (HBM-bound attention + weight
streaming) on a second HIP stream?  Mistral-7B, random weights: times decode-alone, prefill-alone
and both concurrently, plus library GEMM times at mid-size M (decode + piggybacked prefill)."""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from copilot_for_consensus_amd.models.decoder import DecoderModel, DecoderWeights, get_config  # noqa: E402
from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402
from copilot_for_consensus_amd.runtime.engine import LLMEngine  # noqa: E402
from copilot_for_consensus_amd.runtime.kv_cache import PagedKVCache, blocks_needed  # noqa: E402


def gemm_scan(out):
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    for M in (128, 256, 384, 512, 768, 1024, 2048, 4096, 16384):
        tot = 0.0
        for name, (N, Kd) in shapes.items():
            x = torch.randn(M, Kd, device="cuda").bfloat16()
            w = torch.randn(N, Kd, device="cuda").bfloat16()
            for _ in range(3):
                F.linear(x, w)
            torch.cuda.synchronize()
            it = 20
            t = time.perf_counter()
            for _ in range(it):
                F.linear(x, w)
            torch.cuda.synchronize()
            tot += (time.perf_counter() - t) / it
        flops = 2 * M * sum(n * k for n, k in shapes.values())
        out[f"layer_gemms_M{M}"] = {"us": round(tot * 1e6, 1), "PFs": round(flops / tot / 1e15, 3),
                                    "us_per_token": round(tot * 1e6 / M, 3)}
        print(f"M={M:6d} layer GEMMs {tot*1e6:8.1f} us  {flops/tot/1e15:.3f} PF/s  {tot*1e6/M:.3f} us/token", flush=True)


def main():
    res = {}
    gemm_scan(res)
    cfg = get_config("mistral-7b")
    w = DecoderWeights.random(cfg, "cuda", seed=1)
    model = DecoderModel(w)
    B, L, new = 128, 2600, 64
    nblk = 2 * B * blocks_needed(L + 600) + 64
    kv = PagedKVCache(cfg.layers, nblk, cfg.kv_heads, cfg.head_dim, "cuda")
    eng = LLMEngine(model, kv, prefix_cache=False)
    g = torch.Generator().manual_seed(0)
    prompts = [torch.randint(3, 32000, (L,), generator=g).tolist() for _ in range(B)]
    side = [torch.randint(3, 32000, (2048,), generator=g).tolist() for _ in range(8)]   # 16k-token chunk

    def run_decode():
        return eng.generate(prompts, new, ignore_eos=True)

    # the side prefill's blocks are taken up front: the block pool is not shared across threads
    side_tables = [kv.pool.alloc(blocks_needed(len(p))) for p in side]

    def run_prefill(stream):
        with torch.cuda.stream(stream):
            eng._prefill(side, side_tables, 0.0, 0, None)
            stream.synchronize()

    s2 = torch.cuda.Stream()
    run_decode()
    run_prefill(s2)
    torch.cuda.synchronize()
    r = run_decode()
    res["decode_alone_s"] = r.decode_s
    res["prefill_b128_alone_s"] = r.prefill_s
    t = time.perf_counter()
    run_prefill(s2)
    torch.cuda.synchronize()
    res["side_prefill_16k_alone_s"] = time.perf_counter() - t
    # concurrent: batch prefill+decode on the main stream, the 16k-token prefill on s2 from a thread
    th = threading.Thread(target=run_prefill, args=(s2,))
    t = time.perf_counter()
    th.start()
    r2 = run_decode()
    th.join()
    torch.cuda.synchronize()
    res["concurrent_total_s"] = time.perf_counter() - t
    res["concurrent_main_decode_s"] = r2.decode_s
    res["concurrent_main_prefill_s"] = r2.prefill_s
    print(json.dumps(res, indent=1), flush=True)
    with open("gpurun_out/overlap.json", "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
