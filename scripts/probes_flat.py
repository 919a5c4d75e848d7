#!/usr/bin/env python3
"""HBM read roofline vs grid / waves / pieces in flight (csrc/probes/stream_probe.hip flat_kernel),
235 MB (Mistral gate_up) rotated over > 1 GB of copies."""
import ctypes
import json
import os
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "build", "probes", "stream_probe.so"))
lib.flat_probe.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_void_p, ctypes.c_void_p]


def main():
    out = torch.zeros(4, device="cuda")
    nbytes = 28672 * 4096 * 2
    w = torch.empty(nbytes // 2, dtype=torch.bfloat16, device="cuda").normal_()
    ws = [w] + [w.clone() for _ in range(4)]
    calls = [ws[i % 5] for i in range(40)]
    for grid in (224, 256, 512, 1024, 2048, 4096):
        for nwv in (4, 8):
            for f in (4, 8, 16):
                def run(ww):
                    assert lib.flat_probe(ww.data_ptr(), nbytes, grid, nwv, f, out.data_ptr(),
                                          torch.cuda.current_stream().cuda_stream) == 0
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
                print(json.dumps({"grid": grid, "waves": nwv, "inflight_KB_per_wave": f, "us": round(us, 1),
                                  "TBs": round(nbytes / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
