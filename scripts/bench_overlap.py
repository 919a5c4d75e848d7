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


def kernel_overlap(out):
    """Decode-like stream (paged attention B=128 ctx 2900 + the 4 projection GEMMs at M=128, per
    layer) vs prefill-like stream (the 4 projection GEMMs at M=4096) alone and on two streams."""
    import math
    B, L, Hq, Hkv, D = 128, 2900, 32, 8, 128
    nb_per = math.ceil(L / 32) + 1
    kc = torch.randn(B * nb_per, Hkv, 32, D, device="cuda").bfloat16()
    vc = torch.randn(B * nb_per, Hkv, D, 32, device="cuda").bfloat16()
    bt = torch.randperm(B * nb_per, device="cuda").int().view(B, nb_per)
    ctx = torch.full((B,), L, device="cuda", dtype=torch.int32)
    q = torch.randn(B, Hq, D, device="cuda").bfloat16()
    ao = torch.empty_like(q)
    ws = torch.empty(B * Hq * 4 * (D + 2), device="cuda")
    shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
    Ws = [torch.randn(n, k, device="cuda").bfloat16() for n, k in shapes]
    xd = [torch.randn(128, k, device="cuda").bfloat16() for _, k in shapes]
    xp = [torch.randn(4096, k, device="cuda").bfloat16() for _, k in shapes]

    def dec(layers=32):
        for _ in range(layers):
            for x, w in zip(xd, Ws):
                F.linear(x, w)
            K.paged_decode_attention(q, kc, vc, bt, ctx, 1 / math.sqrt(D), out=ao, part_blocks=26, workspace=ws)

    def pre(layers=8):
        for _ in range(layers):
            for x, w in zip(xp, Ws):
                F.linear(x, w)

    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for fn in (dec, pre):
        fn()
    torch.cuda.synchronize()

    def timed(fn):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t

    def both():
        with torch.cuda.stream(s1):
            dec()
        with torch.cuda.stream(s2):
            pre()

    a, b = timed(dec), timed(pre)
    c = timed(both)
    out["overlap_decode_alone_ms"] = round(a * 1e3, 2)
    out["overlap_prefill_alone_ms"] = round(b * 1e3, 2)
    out["overlap_both_ms"] = round(c * 1e3, 2)
    out["overlap_saved_frac_of_prefill"] = round((a + b - c) / b, 3)
    print(f"decode-like {a*1e3:.2f} ms, prefill-like {b*1e3:.2f} ms, both on 2 streams {c*1e3:.2f} ms", flush=True)


def main():
    res = {}
    kernel_overlap(res)
    if os.environ.get("OVERLAP_ONLY"):
        print(json.dumps(res, indent=1))
        return
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
