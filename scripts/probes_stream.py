#!/usr/bin/env python3
"""Weight-stream access-shape probe (csrc/probes/stream_probe.hip): TB/s per (rows per load
instruction, steps in flight, K rotation) over rotated > 1 GB copies of a [N, 4096] bf16 matrix."""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "build", "probes", "stream_probe.so"))
lib.stream_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_void_p, ctypes.c_void_p]


def main():
    out = torch.zeros(4, device="cuda")
    res = []
    for N in (28672, 32768, 6144):
        K = 4096
        w = torch.randn(N, K, device="cuda").bfloat16()
        n = max(2, (1 << 30) // (N * K * 2) + 1)
        ws = [w] + [w.clone() for _ in range(n - 1)]
        calls = [ws[i % n] for i in range(max(48, n))]
        for rpi, d, rot in [(1, 2, 0), (1, 2, 1), (2, 2, 1), (2, 4, 1), (4, 4, 1), (4, 8, 1), (8, 8, 1), (8, 16, 1),
                            (16, 16, 0), (16, 16, 1), (16, 32, 1), (16, 8, 1)]:
            def run(ww):
                rc = lib.stream_probe(ww.data_ptr(), N, K, rpi, d, rot, out.data_ptr(),
                                      torch.cuda.current_stream().cuda_stream)
                assert rc == 0, rc
            run(calls[0])
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for ww in calls:
                    run(ww)
            g.replay()
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                t = time.perf_counter()
                g.replay()
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t) / len(calls))
            us = sorted(ts)[1] * 1e6
            r = {"N": N, "rpi": rpi, "d": d, "rot": rot, "us": round(us, 1), "TBs": round(N * K * 2 / us / 1e6, 2)}
            print(json.dumps(r), flush=True)
            res.append(r)
        del ws, calls, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
