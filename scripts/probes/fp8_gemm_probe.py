#!/usr/bin/env python3
"""Is hipBLASLt FP8 (OCP e4m3fn, gfx950) reachable through torch._scaled_mm, and how fast is it at
the decoder's prefill (M=16k) and decode (M=128) shapes against bf16?"""
import json
import time

import torch


def bench(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it


def main():
    out = {"torch": torch.__version__, "arch": torch.cuda.get_device_properties(0).gcnArchName}
    f8 = torch.float8_e4m3fn
    for M, N, K in ((16384, 28672, 4096), (16384, 6144, 4096), (16384, 4096, 14336), (128, 28672, 4096),
                    (128, 6144, 4096), (128, 4096, 14336)):
        a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        ref = a.float() @ w.float().T
        sa = (a.abs().amax() / 448.0).float().reshape(1)
        sw = (w.abs().amax() / 448.0).float().reshape(1)
        a8 = (a / sa).to(f8)
        w8 = (w / sw).to(f8)
        rec = {}
        try:
            y = torch._scaled_mm(a8, w8.t(), scale_a=sa, scale_b=sw, out_dtype=torch.bfloat16)
            rec["fp8_rel_err"] = float((y.float() - ref).norm() / ref.norm())
            rec["fp8_us"] = round(1e6 * bench(lambda: torch._scaled_mm(a8, w8.t(), scale_a=sa, scale_b=sw,
                                                                        out_dtype=torch.bfloat16)), 1)
        except Exception as e:  # noqa: BLE001
            rec["fp8_error"] = f"{type(e).__name__}: {str(e)[:200]}"
        try:   # rowwise: per-token activation scales x per-output-channel weight scales
            ra = (a.abs().amax(1, keepdim=True) / 448.0).float()
            rw = (w.abs().amax(1, keepdim=True) / 448.0).float()
            a8r, w8r = (a / ra).to(f8), (w / rw).to(f8)
            y = torch._scaled_mm(a8r, w8r.t(), scale_a=ra, scale_b=rw.t(), out_dtype=torch.bfloat16)
            rec["fp8_rowwise_rel_err"] = float((y.float() - ref).norm() / ref.norm())
            rec["fp8_rowwise_us"] = round(1e6 * bench(lambda: torch._scaled_mm(
                a8r, w8r.t(), scale_a=ra, scale_b=rw.t(), out_dtype=torch.bfloat16)), 1)
        except Exception as e:  # noqa: BLE001
            rec["fp8_rowwise_error"] = f"{type(e).__name__}: {str(e)[:200]}"
        rec["bf16_us"] = round(1e6 * bench(lambda: torch.nn.functional.linear(a, w)), 1)
        flops = 2 * M * N * K
        if "fp8_us" in rec:
            rec["fp8_PFs"] = round(flops / rec["fp8_us"] / 1e9, 3)
        rec["bf16_PFs"] = round(flops / rec["bf16_us"] / 1e9, 3)
        out[f"{M}x{N}x{K}"] = rec
        print(f"{M}x{N}x{K}: {rec}", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
