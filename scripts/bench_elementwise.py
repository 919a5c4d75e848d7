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
