#!/usr/bin/env python3
"""Memory-bound decoder elementwise kernels at prefill-chunk (T = 18432) and decode (T = 128)
sizes on Mistral-7B shapes: RoPE + paged KV write, SwiGLU, residual + RMSNorm.  Prints us and the
bytes-moved rate."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402
from copilot_for_consensus_amd.ops import reference as R  # noqa: E402

Hq, Hkv, D, H, FF = 32, 8, 128, 4096, 14336


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def graph_us(fn, iters=200):
    """Per-call time inside one replayed hipGraph (launch overhead excluded, as in decode)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def decode_sizes():
    """The per-layer elementwise kernels of one B=128 decode step, graph-replayed."""
    B = 128
    cs = R.rope_cos_sin(32768, D, 1e6, device="cuda")
    kc = torch.zeros(B * 100, Hkv, 32, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.zeros(B * 100, Hkv, D, 32, device="cuda", dtype=torch.bfloat16)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
    pos = (torch.arange(B, device="cuda", dtype=torch.int32) * 37 + 2000) % 4000
    slots = torch.arange(B, device="cuda", dtype=torch.int32) * 3200 + 2900
    print(f"[graph] rope_kv B={B}: {graph_us(lambda: K.rope_kv_write(qkv, pos, slots, cs, kc, vc, Hq, Hkv, D)):.2f} us")
    gu = torch.randn(B, 2 * FF, device="cuda").bfloat16()
    print(f"[graph] silu_mul B={B}: {graph_us(lambda: K.silu_mul(gu)):.2f} us")
    for K_, split in ((Hq * D, 4), (FF, 8)):
        a = torch.randn(B, K_, device="cuda").bfloat16()
        w = torch.randn(H, K_, device="cuda").bfloat16()
        res = torch.randn(B, H, device="cuda").bfloat16()
        nw = torch.randn(H, device="cuda").bfloat16()
        part = torch.randn(split, B, H, device="cuda")
        out = torch.empty(B, H, device="cuda").bfloat16()
        f = lambda: K.kernels().cfc_splitk_residual_rmsnorm(part.data_ptr(), split, B, H, res.data_ptr(),  # noqa: E731
                                                             nw.data_ptr(), 1e-5, out.data_ptr(), K._stream(a))
        print(f"[graph] splitk_residual_rmsnorm split={split}: {graph_us(f):.2f} us")
        g = lambda: K.lib_splitk_linear_residual_rmsnorm(a, w, split, res, nw, 1e-5)  # noqa: E731
        print(f"[graph] lib split-K GEMM + reduce K={K_} split={split}: {graph_us(g, 50):.2f} us")
    x = torch.randn(B, H, device="cuda").bfloat16()
    res = torch.randn(B, H, device="cuda").bfloat16()
    nw = torch.randn(H, device="cuda").bfloat16()
    print(f"[graph] add+rmsnorm B={B}: {graph_us(lambda: K.rmsnorm(x, nw, 1e-5, residual=res)):.2f} us")


def main():
    cs = R.rope_cos_sin(32768, D, 1e6, device="cuda")
    for T in (18432, 128):
        nblk = T // 32 + 64
        kc = torch.zeros(nblk, Hkv, 32, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.zeros(nblk, Hkv, D, 32, device="cuda", dtype=torch.bfloat16)
        qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
        pos = torch.arange(T, device="cuda", dtype=torch.int32) % 4096
        slots = torch.arange(T, device="cuda", dtype=torch.int32) + 32 * 7
        us = timeit(lambda: K.rope_kv_write(qkv, pos, slots, cs, kc, vc, Hq, Hkv, D))
        byts = qkv.numel() * 2 + T * Hq * D * 2 + 2 * T * Hkv * D * 2
        print(f"rope_kv T={T}: {us:.1f} us  {byts / us / 1e6:.2f} TB/s", flush=True)
        runs = torch.from_numpy(K.v_runs(slots.cpu().numpy())).cuda()
        us = timeit(lambda: K.rope_kv_write(qkv, pos, slots, cs, kc, vc, Hq, Hkv, D, runs=runs))
        print(f"rope_kv+v_runs T={T}: {us:.1f} us  {byts / us / 1e6:.2f} TB/s", flush=True)
        gu = torch.randn(T, 2 * FF, device="cuda").bfloat16()
        us = timeit(lambda: K.silu_mul(gu))
        print(f"silu_mul T={T}: {us:.1f} us  {gu.numel() * 3 / us / 1e6:.2f} TB/s", flush=True)
        x = torch.randn(T, H, device="cuda").bfloat16()
        res = torch.randn(T, H, device="cuda").bfloat16()
        w = torch.randn(H, device="cuda").bfloat16()
        us = timeit(lambda: K.rmsnorm(x, w, 1e-5, residual=res))
        print(f"add+rmsnorm T={T}: {us:.1f} us  {x.numel() * 2 * 4 / us / 1e6:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
    decode_sizes()
