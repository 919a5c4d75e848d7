#!/usr/bin/env python3
"""BASELINE config 5 (retrieval half): a 100M x 384 bf16 cosine index resident in one MI355X's HBM
(77 GB of 288 GB), exact top-k by the fused MFMA scan + radix-select kernel (knn_topk_kernel: the
[nq, N] scores never reach HBM).  ``--ivf NLIST NPROBE``: the same index as IVF-flat over
clustered data (a Gaussian mixture, so lists mean something), k-means on a bf16 sample, one
fused launch per query batch; reports build time, ms per batch and recall@10 against the flat
scan.

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
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("n", nargs="?", type=float, default=100_000_000)
    ap.add_argument("--ivf", type=int, nargs=2, metavar=("NLIST", "NPROBE"), default=None)
    ap.add_argument("--clusters", type=int, default=20000)
    args = ap.parse_args()
    n = int(args.n)
    dim = 384
    if args.ivf:
        from copilot_for_consensus_amd.vectorstore import HipIVFIndex
        idx = HipIVFIndex(dim, "cosine", nlist=args.ivf[0], nprobe=args.ivf[1], device="cuda", capacity=n)
    else:
        idx = HipFlatIndex(dim, device="cuda", capacity=n)
    chunk = 1 << 22
    g = torch.Generator(device="cuda").manual_seed(0)
    centers = torch.nn.functional.normalize(torch.randn(args.clusters, dim, device="cuda", generator=g), dim=1) \
        if args.ivf else None
    t = time.perf_counter()
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        v = torch.randn(e - s, dim, device="cuda", generator=g)
        if centers is not None:   # Gaussian mixture: a center + noise of ~0.35 of its norm
            v = centers[torch.randint(0, args.clusters, (e - s,), device="cuda", generator=g)] + 0.02 * v
        idx._X[s:e] = torch.nn.functional.normalize(v, dim=1).bfloat16()
        del v
    idx._norm2[:n] = 1.0
    idx._alive[:n] = True
    idx._n = n
    idx._ids = [None] * 0          # device-side search() only; ids are not materialised at this scale
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t
    res = {"vectors": n, "dim": dim, "index_bytes": n * dim * 2, "fill_s": round(build_s, 2)}
    if args.ivf:
        idx._ids = [None] * n          # regroup permutes ids: placeholders at this scale
        idx._meta = [None] * n
        t = time.perf_counter()
        idx.train(iters=8)
        torch.cuda.synchronize()
        res.update(ivf_nlist=idx.nlist, ivf_nprobe=idx.nprobe, ivf_train_s=round(time.perf_counter() - t, 2),
                   ivf_max_chunks=idx._maxc)
        print(f"ivf: nlist={idx.nlist} trained+regrouped in {res['ivf_train_s']} s", flush=True)

    def queries(nq):
        if centers is None:
            return torch.nn.functional.normalize(torch.randn(nq, dim, device="cuda", generator=g), dim=1)
        c = centers[torch.randint(0, args.clusters, (nq,), device="cuda", generator=g)]
        return torch.nn.functional.normalize(c + 0.02 * torch.randn(nq, dim, device="cuda", generator=g), dim=1)
    for nq, k in ((1, 10), (1, 150), (16, 10), (16, 150)):
        Q = queries(nq)
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
    if args.ivf:   # recall@10 of the IVF search against the exact flat scan of the same rows
        Q = queries(64)
        hits = 0
        for s in range(0, 64, 16):
            _, i_ivf = idx.search(Q[s:s + 16], 10)
            _, i_flat = HipFlatIndex.search(idx, Q[s:s + 16], 10, rows=(0, n))
            hits += sum(len(set(a) & set(b)) for a, b in zip(i_ivf.cpu().tolist(), i_flat.cpu().tolist()))
        res["ivf_recall_at_10"] = round(hits / 640, 4)
        print(f"ivf recall@10 vs flat: {res['ivf_recall_at_10']}", flush=True)
        out = "gpurun_out/bench_ivf.json"
    else:
        out = "gpurun_out/bench_knn.json"
    # exactness spot check on a slice against a plain fp32 matmul
    Q = torch.nn.functional.normalize(torch.randn(4, dim, device="cuda", generator=g), dim=1)
    m = min(n, 1 << 22)
    v, i = HipFlatIndex.search(idx, Q, 10, rows=(0, m))
    ref = torch.topk(Q @ idx._X[:m].float().T, 10, dim=1)
    res["exact_top10_overlap"] = float((i.cpu().sort(1).values == ref.indices.cpu().sort(1).values).float().mean())
    print(json.dumps(res), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
