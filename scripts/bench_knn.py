#!/usr/bin/env python3
"""BASELINE config 5 (retrieval half): a 100M x 384 bf16 cosine index resident in one MI355X's HBM
(77 GB of 288 GB), exact top-k by the fused MFMA scan + radix-select kernels.

The vectors are generated on the GPU (random, L2-normalised) straight into the index storage;
queries are batches of <= 16 (the scan kernel's query tile).  Reports scan bandwidth, query
latency and queries/s for top-k = 10 and 150 (the reporting service's limit*3, main.py:205)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from copilot_for_consensus_amd.vectorstore import HipFlatIndex  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
    dim = 384
    idx = HipFlatIndex(dim, device="cuda", capacity=n)
    chunk = 1 << 22
    g = torch.Generator(device="cuda").manual_seed(0)
    t = time.perf_counter()
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        v = torch.randn(e - s, dim, device="cuda", generator=g)
        idx._X[s:e] = torch.nn.functional.normalize(v, dim=1).bfloat16()
        del v
    idx._norm2[:n] = 1.0
    idx._alive[:n] = True
    idx._n = n
    idx._ids = [None] * 0          # device-side search() only; ids are not materialised at this scale
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t
    res = {"vectors": n, "dim": dim, "index_bytes": n * dim * 2, "fill_s": round(build_s, 2)}
    for nq, k in ((1, 10), (16, 10), (16, 150)):
        Q = torch.nn.functional.normalize(torch.randn(nq, dim, device="cuda", generator=g), dim=1)
        for _ in range(2):
            idx.search(Q, k)
        torch.cuda.synchronize()
        it = 5
        t = time.perf_counter()
        for _ in range(it):
            v, i = idx.search(Q, k)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / it
        res[f"nq{nq}_k{k}"] = {"ms": round(dt * 1e3, 2), "qps": round(nq / dt, 1),
                               "scan_TBs": round(n * dim * 2 / dt / 1e12, 2)}
        print(f"nq={nq} k={k}: {dt*1e3:.2f} ms/batch, {nq/dt:.1f} qps, {n*dim*2/dt/1e12:.2f} TB/s", flush=True)
    # exactness spot check on a slice against a plain fp32 matmul
    Q = torch.nn.functional.normalize(torch.randn(4, dim, device="cuda", generator=g), dim=1)
    m = min(n, 1 << 22)
    v, i = idx.search(Q, 10, rows=(0, m))
    ref = torch.topk(Q @ idx._X[:m].float().T, 10, dim=1)
    res["exact_top10_overlap"] = float((i.cpu().sort(1).values == ref.indices.cpu().sort(1).values).float().mean())
    print(json.dumps(res), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/bench_knn.json", "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
