#!/usr/bin/env python3
"""IVF-flat quality and speed on honest data (BASELINE config 5's retrieval half; the reference's
FAISS IndexIVFFlat, faiss_store.py:105-111, and its id maps, :303-345).

Datasets (--data):
  * uniform  -- uniformly random unit vectors: no cluster structure at all, IVF's worst case;
  * minilm   -- MiniLM-L6 encoder outputs (the HIP encoder, random-init weights: no checkpoint can be
                downloaded here) of the synthetic mailing-list chunks, tiled to N rows with a small
                per-copy perturbation (--noise) so no two rows are identical.
Every row carries a real id string and its metadata through the build (RowTable: add_bulk, the
k-means regroup permutation, the search results).  For nprobe in --nprobe: recall@10 against the
exact flat scan of the same rows, ms per 16-query batch, and the bytes the probed lists really hold
(scan_TBs = those bytes / time; each (query, list) work item reads its list once).
Writes one JSON line per nprobe to --out."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from copilot_for_consensus_amd.vectorstore import HipFlatIndex, HipIVFIndex  # noqa: E402


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def minilm_vectors(n_unique: int, device) -> torch.Tensor:
    from copilot_for_consensus_amd.chunking import create_chunker
    from copilot_for_consensus_amd.embedding import HipEncoderProvider
    from copilot_for_consensus_amd.utils.synthetic import SyntheticArchive
    arc = SyntheticArchive(seed=3)
    texts = []
    while len(texts) < n_unique:
        for t in arc.thread(8):
            body = t.split(b"\n\n", 1)[1].decode("utf-8", "replace")
            words = body.split()
            for s in range(0, max(1, len(words)), 300):   # ~300-word chunks (chunker-sized)
                texts.append(" ".join(words[s:s + 384]))
    texts = texts[:n_unique]
    enc = HipEncoderProvider("all-MiniLM-L6-v2", device=str(device))
    out = []
    for s in range(0, len(texts), 4096):
        out.append(enc.embed_tensor(texts[s:s + 4096]).to(torch.bfloat16))
    return torch.nn.functional.normalize(torch.cat(out).float(), dim=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=10_000_000)
    ap.add_argument("--data", choices=["uniform", "minilm"], default="uniform")
    ap.add_argument("--nlist", type=int, default=0, help="0 = sqrt(N)")
    ap.add_argument("--nprobe", type=int, nargs="*", default=[8, 32, 128])
    ap.add_argument("--unique", type=int, default=200_000, help="minilm: distinct encoder outputs before tiling")
    ap.add_argument("--queries", type=int, default=256)
    ap.add_argument("--noise", type=float, default=0.01,
                    help="minilm: per-dimension gaussian perturbation of each tiled copy (0.01 ~ norm 0.2)")
    ap.add_argument("--out", default="gpurun_out/bench_ivf.jsonl")
    ap.add_argument("--device", default="cuda", help="cpu: a functional dry run at small --n")
    args = ap.parse_args()
    n, dim, dev = int(args.n), 384, torch.device(args.device)
    g = torch.Generator(device=dev).manual_seed(0)
    t0 = time.perf_counter()
    base = minilm_vectors(args.unique, dev) if args.data == "minilm" else None
    enc_s = time.perf_counter() - t0

    def rows(s, e):
        if base is None:
            return torch.nn.functional.normalize(torch.randn(e - s, dim, device=dev, generator=g), dim=1)
        src = base[torch.arange(s, e, device=dev) % base.shape[0]]
        return torch.nn.functional.normalize(src + args.noise * torch.randn(e - s, dim, device=dev, generator=g), dim=1)

    idx = HipIVFIndex(dim, "cosine", nlist=args.nlist, nprobe=8, device=str(dev), capacity=n)
    t0 = time.perf_counter()
    chunk = 1 << 22
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        ids = [f"{i:016x}" for i in range(s, e)]
        metas = [{"thread_id": f"t{i // 32:012x}"} for i in range(s, e)] if n <= 20_000_000 else None
        idx.add_bulk(ids, rows(s, e).to(torch.bfloat16), metas)
    _sync(dev)
    fill_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    idx.train(iters=8)
    _sync(dev)
    train_s = time.perf_counter() - t0
    host_bytes = sum(a.nbytes for a in idx._tab._cols.values()) + idx._tab._ids.n + idx._tab._meta.n
    # queries: fresh rows from the same distribution (minilm: perturbed encoder outputs)
    qsrc = rows(0, args.queries) if base is None else torch.nn.functional.normalize(
        base[torch.randint(0, base.shape[0], (args.queries,), device=dev, generator=g)]
        + args.noise * torch.randn(args.queries, dim, device=dev, generator=g), dim=1)
    Q = qsrc.to(torch.bfloat16)
    exact = []
    t0 = time.perf_counter()
    for s in range(0, args.queries, 16):
        exact.append(HipFlatIndex.search(idx, Q[s:s + 16], 10, rows=(0, n))[1].cpu())
    _sync(dev)
    flat_ms = (time.perf_counter() - t0) * 1e3 / (args.queries // 16)
    exact = torch.cat(exact)
    sizes = (idx._list_off_t[1:] - idx._list_off_t[:-1])
    # ids survive the regroup: a returned row's id names the vector stored there
    v, i = idx.search(Q[:1], 1)
    r0 = int(i[0, 0])
    id_ok = idx._tab.id_at(r0) is not None and idx.get(idx._tab.id_at(r0)).vector is not None
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    for npb in args.nprobe:
        idx.nprobe = npb
        got, scanned = [], 0
        for s in range(0, args.queries, 16):
            got.append(idx.search(Q[s:s + 16], 10)[1].cpu())
            probe = idx.probe_lists(torch.nn.functional.normalize(Q[s:s + 16].float(), dim=1).to(torch.bfloat16))
            scanned += int(sizes[probe.long()].sum())
        got = torch.cat(got)
        recall = sum(len(set(a) & set(b)) for a, b in zip(got.tolist(), exact.tolist())) / (10 * args.queries)
        Qb = Q[:16]
        for _ in range(2):
            idx.search(Qb, 10)
        _sync(dev)
        it = 10
        t0 = time.perf_counter()
        for _ in range(it):
            idx.search(Qb, 10)
        _sync(dev)
        dt = (time.perf_counter() - t0) / it
        per_batch_rows = scanned / (args.queries / 16)
        row = {"data": args.data, "n": n, "nlist": idx.nlist, "nprobe": npb, "recall_at_10": round(recall, 4),
               "ms_per_16q": round(dt * 1e3, 3), "flat_ms_per_16q": round(flat_ms, 2),
               "rows_scanned_per_16q": int(per_batch_rows),
               "scan_TBs": round(per_batch_rows * dim * 2 / dt / 1e12, 3),
               "fill_s": round(fill_s, 1), "train_regroup_s": round(train_s, 1), "encoder_s": round(enc_s, 1),
               "host_rowtable_bytes_per_row": round(host_bytes / n, 1), "ids_materialised": bool(id_ok),
               "largest_list": int(sizes.max()), "empty_lists": int((sizes == 0).sum())}
        print(json.dumps(row), flush=True)
        with open(args.out, "a") as fh:
            fh.write(json.dumps(row) + "\n")


if __name__ == "__main__":
    main()
