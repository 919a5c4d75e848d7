"""Vector stores: interface, HBM-resident HIP flat / IVF indexes, in-memory reference, factory.

Interface = adapters/copilot_vectorstore/copilot_vectorstore/interface.py:12-114 of the reference
(add_embedding / add_embeddings [upsert] / query(vector, top_k) -> [SearchResult] / delete / clear /
count / get).  Replaces Qdrant / FAISS / Azure AI Search on the hot path:

* :class:`HipFlatIndex` -- the whole index lives in one bf16 [capacity, dim] HBM tensor (a
  288 GB MI355X holds 100M x 384 bf16 = 77 GB with room to spare); cosine = dot product of
  L2-normalised rows (normalised on insert by a HIP kernel), or squared-L2 with stored norms
  (FAISS IndexFlatL2 parity, score 1/(1+d), faiss_store.py:224).  Queries: <=16 at a time run the
  fused MFMA scan kernel, larger batches a hipBLASLt GEMM; exact top-k by the radix-select kernel.
  Vectors produced on the GPU (the encoder) are inserted without a host round trip.
  Upserts overwrite in place; deletes tombstone + periodic compaction.
* :class:`HipIVFIndex` -- IVF-flat: k-means coarse quantiser trained on the GPU, rows stored
  list-contiguous, ``nprobe`` lists scanned per query.
* :class:`InMemoryVectorStore` -- numpy reference (fixes the reference's duplicate-id error,
  inmemory.py:46, which violates the upsert contract).
"""
from __future__ import annotations

import dataclasses
import json
import math
import threading
from abc import ABC, abstractmethod
from pathlib import Path
from typing import Any, Sequence

import numpy as np
import torch

from .rowtable import RowTable


@dataclasses.dataclass
class SearchResult:
    id: str
    score: float
    vector: list[float]
    metadata: dict[str, Any]


class VectorStore(ABC):
    def add_embedding(self, id: str, vector, metadata: dict[str, Any] | None = None) -> None:
        self.add_embeddings([id], [vector], [metadata or {}])

    @abstractmethod
    def add_embeddings(self, ids: Sequence[str], vectors, metadatas: Sequence[dict] | None = None) -> None: ...

    @abstractmethod
    def query(self, query_vector, top_k: int = 10) -> list[SearchResult]: ...

    @abstractmethod
    def delete(self, id: str) -> None: ...

    @abstractmethod
    def clear(self) -> None: ...

    @abstractmethod
    def count(self) -> int: ...

    @abstractmethod
    def get(self, id: str) -> SearchResult: ...

    def __len__(self) -> int:
        return self.count()

    def query_batch(self, query_vectors, top_k: int = 10) -> list[list[SearchResult]]:
        return [self.query(q, top_k) for q in query_vectors]

    def centroid_scores(self, ids: Sequence[str]) -> dict[str, float]:
        """Cosine similarity of each stored vector of ``ids`` to their normalised mean -- the
        orchestrator's relevance of a thread's chunks to the thread (a search restricted to the
        thread's own rows: every chunk scored on one scale, none dropped by a global top-k).
        Ids not in the store are left out.  Generic path: one get() per id."""
        have, vecs = [], []
        for i in ids:
            try:
                vecs.append(np.asarray(self.get(i).vector, dtype=np.float32))
            except KeyError:
                continue
            have.append(i)
        if not vecs:
            return {}
        X = np.stack(vecs)
        X = X / np.maximum(np.linalg.norm(X, axis=1, keepdims=True), 1e-12)
        c = X.mean(0)
        c = c / max(float(np.linalg.norm(c)), 1e-12)
        return dict(zip(have, (X @ c).astype(float).tolist()))


    def centroid_scores_many(self, groups: Sequence[Sequence[str]]) -> list[dict[str, float]]:
        """centroid_scores of many id groups (one per thread); stores with a device path score them
        all in one pass."""
        return [self.centroid_scores(g) for g in groups]


def _as_matrix(vectors, dim: int | None, device=None, dtype=torch.float32) -> torch.Tensor:
    if isinstance(vectors, torch.Tensor):
        t = vectors
    elif isinstance(vectors, (list, tuple)) and vectors and all(isinstance(v, torch.Tensor) for v in vectors):
        t = torch.stack([v.reshape(-1) for v in vectors])
    else:
        t = torch.as_tensor(np.asarray(vectors, dtype=np.float32))
    if t.dim() == 1:
        t = t[None]
    if t.dim() != 2 or t.shape[1] == 0:
        raise ValueError(f"expected non-empty vectors, got shape {tuple(t.shape)}")
    if dim is not None and t.shape[1] != dim:
        raise ValueError(f"vector dimension {t.shape[1]} != index dimension {dim}")
    return t.to(device=device, dtype=dtype) if device is not None else t.to(dtype)


class InMemoryVectorStore(VectorStore):
    """numpy cosine store (reference semantics, but upsert-correct)."""

    def __init__(self, dimension: int | None = None, **_):
        if dimension is not None and int(dimension) <= 0:
            raise ValueError(f"dimension must be positive, got {dimension}")
        self.dim = dimension
        self._ids: list[str] = []
        self._row: dict[str, int] = {}
        self._vecs: list[np.ndarray] = []
        self._meta: list[dict] = []
        self._lock = threading.Lock()

    def add_embeddings(self, ids, vectors, metadatas=None):
        mats = _as_matrix(vectors, self.dim).cpu().numpy()
        if len(ids) != len(mats):
            raise ValueError("ids and vectors length mismatch")
        metadatas = metadatas or [{} for _ in ids]
        with self._lock:
            if self.dim is None:
                self.dim = mats.shape[1]
            for i, v, m in zip(ids, mats, metadatas):
                if i in self._row:
                    r = self._row[i]
                    self._vecs[r], self._meta[r] = v.copy(), dict(m)
                else:
                    self._row[i] = len(self._ids)
                    self._ids.append(i)
                    self._vecs.append(v.copy())
                    self._meta.append(dict(m))

    def query(self, query_vector, top_k=10):
        if not self._ids:
            return []
        q = _as_matrix(query_vector, self.dim).cpu().numpy()[0]
        X = np.stack(self._vecs)
        sims = X @ q / np.maximum(np.linalg.norm(X, axis=1) * max(np.linalg.norm(q), 1e-12), 1e-12)
        order = np.argsort(-sims, kind="stable")[:top_k]
        return [SearchResult(self._ids[r], float(sims[r]), self._vecs[r].tolist(), dict(self._meta[r])) for r in order]

    def delete(self, id):
        with self._lock:
            r = self._row.pop(id)
            last = len(self._ids) - 1
            if r != last:
                self._ids[r], self._vecs[r], self._meta[r] = self._ids[last], self._vecs[last], self._meta[last]
                self._row[self._ids[r]] = r
            self._ids.pop()
            self._vecs.pop()
            self._meta.pop()

    def clear(self):
        with self._lock:
            self._ids, self._row, self._vecs, self._meta = [], {}, [], []

    def count(self):
        return len(self._ids)

    def get(self, id):
        r = self._row[id]
        return SearchResult(id, 1.0, self._vecs[r].tolist(), dict(self._meta[r]))


class HipFlatIndex(VectorStore):
    """Exact flat index resident in HBM (see module docstring)."""

    def __init__(self, dimension: int = 384, distance: str = "cosine", capacity: int = 1 << 16, device="cuda",
                 faiss_scores: bool = False, **_):
        if distance not in ("cosine", "dot", "l2", "euclid"):
            raise ValueError(f"unknown distance {distance!r}")
        if int(dimension) <= 0:
            raise ValueError(f"dimension must be positive, got {dimension}")
        self.dim = int(dimension)
        self.metric = "l2" if distance in ("l2", "euclid") else distance
        self.faiss_scores = faiss_scores
        self.device = torch.device(device if (device != "cuda" or torch.cuda.is_available()) else "cpu")
        self._cap = 0
        self._n = 0                       # rows in use (incl. tombstones)
        self._X = torch.empty(0, self.dim, dtype=torch.bfloat16, device=self.device)
        self._norm2 = torch.empty(0, dtype=torch.float32, device=self.device)
        self._alive = torch.empty(0, dtype=torch.bool, device=self.device)
        # ids + metadata: numpy columns and byte heaps, no Python object per row (rowtable.py)
        self._tab = RowTable(max(1024, int(capacity)))
        self._dead = 0
        self._lock = threading.RLock()
        self._reserve(capacity)

    # ------------------------------------------------------------------ storage
    def _reserve(self, n: int) -> None:
        if n <= self._cap:
            return
        cap = max(n, 2 * self._cap, 1024)
        X = torch.zeros(cap, self.dim, dtype=torch.bfloat16, device=self.device)
        n2 = torch.zeros(cap, dtype=torch.float32, device=self.device)
        al = torch.zeros(cap, dtype=torch.bool, device=self.device)
        # rows already written (add_embeddings counts new rows in _n before it reserves them)
        k = min(self._n, self._cap)
        if k:
            X[:k] = self._X[:k]
            n2[:k] = self._norm2[:k]
            al[:k] = self._alive[:k]
        self._X, self._norm2, self._alive, self._cap = X, n2, al, cap

    def _prepare(self, vecs: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        from ..ops import kernels as K
        v = vecs.to(device=self.device, dtype=torch.bfloat16).contiguous()
        n2 = torch.empty(v.shape[0], dtype=torch.float32, device=self.device)
        if self.metric == "cosine":
            v = K.l2_normalize(v, norms2=n2)
            n2.fill_(1.0)
        else:
            n2 = v.float().pow(2).sum(1)
        return v, n2

    def add_embeddings(self, ids, vectors, metadatas=None):
        vecs = _as_matrix(vectors, self.dim)
        if len(ids) != vecs.shape[0]:
            raise ValueError("ids and vectors length mismatch")
        metadatas = list(metadatas) if metadatas is not None else [{} for _ in ids]
        v, n2 = self._prepare(vecs)
        with self._lock:
            rows = self._tab.upsert(ids, metadatas)
            self._n = self._tab.n
            self._reserve(self._n)
            idx = torch.from_numpy(rows).to(self.device)
            self._X.index_copy_(0, idx, v)
            self._norm2.index_copy_(0, idx, n2)
            self._alive[idx] = True

    def add_bulk(self, ids, vectors, metadatas=None) -> None:
        """Bulk build of NEW ids (no upsert check): vectors straight into HBM, ids / metadata into
        the row table in one vectorised append -- the path for 10M-100M-row indexes."""
        vecs = _as_matrix(vectors, self.dim, device=self.device, dtype=torch.bfloat16) \
            if not isinstance(vectors, torch.Tensor) else vectors
        if len(ids) != vecs.shape[0]:
            raise ValueError("ids and vectors length mismatch")
        with self._lock:
            n0 = self._n
            self._tab.append_bulk(ids, metadatas)
            self._n = self._tab.n
            self._reserve(self._n)
            for s in range(0, vecs.shape[0], 1 << 22):
                v, n2 = self._prepare(vecs[s:s + (1 << 22)])
                self._X[n0 + s:n0 + s + v.shape[0]] = v
                self._norm2[n0 + s:n0 + s + v.shape[0]] = n2
            self._alive[n0:self._n] = True

    def has(self, id) -> bool:
        return self._tab.find(id) >= 0

    def delete(self, id):
        with self._lock:
            r = self._tab.find(id)
            if r < 0:
                raise KeyError(id)   # reference contract
            self._tab.kill(r)
            self._alive[r] = False
            self._dead += 1
            if self._dead > 1024 and self._dead > self._n // 4:
                self.compact()

    def compact(self) -> None:
        with self._lock:
            if self._dead == 0:
                return
            keep = np.nonzero(self._tab.live)[0]
            idx = torch.from_numpy(keep).to(self.device)
            n = int(keep.size)
            self._X[:n] = self._X.index_select(0, idx) if n else self._X[:0]
            self._norm2[:n] = self._norm2.index_select(0, idx) if n else self._norm2[:0]
            self._alive[:n] = True
            self._alive[n:] = False
            self._tab.permute(keep)
            self._n, self._dead = n, 0

    def clear(self):
        with self._lock:
            self._n, self._dead = 0, 0
            self._tab.clear()
            self._alive.zero_()

    def count(self):
        return self._n - self._dead

    def get(self, id):
        r = self._tab.find(id)
        if r < 0:
            raise KeyError(id)
        return SearchResult(id, 1.0, self._X[r].float().cpu().tolist(), self._tab.meta_at(r))

    # ------------------------------------------------------------------ search
    def centroid_scores(self, ids):
        """Device path of VectorStore.centroid_scores: one gather of the rows, one GEMV, one copy out."""
        with self._lock:
            rows = self._tab.find_many(list(ids))
            have = [i for i, r in zip(ids, rows) if r >= 0]
            if not have:
                return {}
            idx = torch.from_numpy(rows[rows >= 0]).to(self.device)
            s = self.span_centroid_scores(self._X.index_select(0, idx), [(0, len(have))])
            return dict(zip(have, s.cpu().tolist()))

    def centroid_scores_many(self, groups):
        """All groups in one gather + one segment reduction (span_centroid_scores over the gathered
        rows, one span per group) and one copy out."""
        with self._lock:
            have, rows_all, spans = [], [], []
            for g in groups:
                g = list(g)
                rows = self._tab.find_many(g) if g else np.zeros(0, np.int64)
                h = [i for i, r in zip(g, rows) if r >= 0]
                a = sum(len(x) for x in have)
                have.append(h)
                rows_all.append(rows[rows >= 0])
                spans.append((a, a + len(h)))
            n = sum(len(h) for h in have)
            if n == 0:
                return [{} for _ in groups]
            idx = torch.from_numpy(np.concatenate(rows_all)).to(self.device)
            live = [(a, b) for a, b in spans if b > a]
            s = self.span_centroid_scores(self._X.index_select(0, idx), live).cpu().tolist()
        return [dict(zip(h, s[a:b])) for h, (a, b) in zip(have, spans)]

    @staticmethod
    def span_centroid_scores(X: torch.Tensor, spans) -> torch.Tensor:
        """Rows of X grouped in consecutive spans (one per thread): cosine of every row to its own
        span's normalised mean, fp32 [rows] on X's device (segment sums, no per-span launches)."""
        Xf = torch.nn.functional.normalize(X.float(), dim=1)
        lens = torch.tensor([b - a for a, b in spans], device=X.device)
        seg = torch.repeat_interleave(torch.arange(len(spans), device=X.device), lens)
        base = spans[0][0]
        rows = Xf[base:base + int(lens.sum())]
        cent = torch.zeros(len(spans), X.shape[1], device=X.device).index_add_(0, seg, rows)
        cent = torch.nn.functional.normalize(cent, dim=1)
        return (rows * cent[seg]).sum(1)

    def search(self, Q: torch.Tensor, k: int, rows: tuple[int, int] | None = None) -> tuple[torch.Tensor, torch.Tensor]:
        """Device-side exact search: (scores [nq, k], row indices [nq, k]) for queries Q."""
        from ..ops import kernels as K
        lo, hi = rows if rows is not None else (0, self._n)
        Q = _as_matrix(Q, self.dim, device=self.device, dtype=torch.bfloat16)
        nq = Q.shape[0]
        if hi <= lo:
            return (torch.empty(nq, 0, device=self.device), torch.empty(nq, 0, dtype=torch.long, device=self.device))
        X = self._X[lo:hi]
        if self.metric == "cosine":
            Qn = K.l2_normalize(Q.contiguous())
            qn2 = None
        else:
            Qn = Q.contiguous()
            qn2 = Qn.float().pow(2).sum(1)
        if Q.is_cuda and nq <= 16 and k <= 256:
            # fused scan + top-k: only k candidates per 1024-row chunk leave the CUs
            return K.knn_topk(self._X, Qn, k, self._norm2 if self.metric == "l2" else None, qn2,
                              self._alive if self._dead else None, row_lo=lo, N=hi)
        xn2 = self._norm2[lo:hi] if self.metric == "l2" else None
        if Q.is_cuda and nq <= 16:
            scores = K.knn_scores(X, Qn, xn2, qn2)
        else:
            scores = Qn.float() @ X.float().T if not Q.is_cuda else (Qn @ X.T).float()
            if self.metric == "l2":
                scores = -(xn2[None, :] + qn2[:, None] - 2 * scores)
        if self._dead:
            scores = scores.masked_fill(~self._alive[lo:hi][None, :], float("-inf"))
        v, i = K.topk(scores.contiguous(), k)
        return v, i + lo

    def _to_results(self, v: torch.Tensor, i: torch.Tensor, with_vectors: bool = True) -> list[list[SearchResult]]:
        v, i = v.cpu(), i.cpu()
        out = []
        for qv, qi in zip(v.tolist(), i.tolist()):
            res = []
            for s, r in zip(qv, qi):
                rid = self._tab.id_at(r) if r >= 0 and s != float("-inf") else None
                if rid is None:
                    continue
                if self.metric == "l2":
                    s = 1.0 / (1.0 + max(0.0, -s)) if self.faiss_scores else -s
                vec = self._X[r].float().cpu().tolist() if with_vectors else []
                res.append(SearchResult(rid, float(s), vec, self._tab.meta_at(r)))
            out.append(res)
        return out

    def query(self, query_vector, top_k=10):
        return self.query_batch(_as_matrix(query_vector, self.dim), top_k)[0]

    def query_batch(self, query_vectors, top_k=10, with_vectors: bool = False):
        with self._lock:
            if self.count() == 0:
                return [[] for _ in range(len(query_vectors))]
            Q = _as_matrix(query_vectors, self.dim)
            outs = []
            for s in range(0, Q.shape[0], 16):
                v, i = self.search(Q[s:s + 16], min(top_k, self.count()))
                outs.extend(self._to_results(v, i, with_vectors))
            return outs

    # ------------------------------------------------------------------ persistence
    def save(self, path) -> None:
        """Index shard = safetensors blob (vectors, norms) + the row table's .npy columns and heaps
        (ids, metadata) + a small JSON header.  Nothing pickled."""
        from safetensors.torch import save_file
        p = Path(path)
        p.mkdir(parents=True, exist_ok=True)
        with self._lock:
            self.compact()
            save_file({"vectors": self._X[:self._n].contiguous().cpu(), "norm2": self._norm2[:self._n].cpu()},
                      str(p / "vectors.safetensors"))
            self._tab.save(p)
            hdr = {"dim": self.dim, "metric": self.metric, "rows": self._n, "format": "rowtable-1"}
            hdr.update(self._extra_header())
            (p / "index.json").write_text(json.dumps(hdr))
            extra = self._extra_tensors()
            if extra:
                save_file(extra, str(p / "ivf.safetensors"))

    def _extra_header(self) -> dict:
        return {}

    def _extra_tensors(self) -> dict:
        return {}

    def _restore_extra(self, meta: dict, path: Path) -> None:
        pass

    @classmethod
    def load(cls, path, device="cuda") -> "HipFlatIndex":
        from safetensors.torch import load_file
        p = Path(path)
        meta = json.loads((p / "index.json").read_text())
        t = load_file(str(p / "vectors.safetensors"))
        n = int(meta["rows"]) if "rows" in meta else len(meta["ids"])
        idx = cls(meta["dim"], "l2" if meta["metric"] == "l2" else meta["metric"], capacity=n + 1024, device=device)
        idx._X[:n] = t["vectors"].to(idx.device)
        idx._norm2[:n] = t["norm2"].to(idx.device)
        idx._alive[:n] = True
        if meta.get("format") == "rowtable-1":
            idx._tab = RowTable.load(p)
        else:                                  # round-3 JSON sidecar (ids / metadata lists)
            idx._tab = RowTable(n + 1024)
            idx._tab.append_bulk(meta["ids"], meta["metadata"])
        idx._n = n
        idx._restore_extra(meta, p)
        return idx


class HipIVFIndex(HipFlatIndex):
    """IVF-flat (FAISS IndexIVFFlat semantics, faiss_store.py:105-111): rows regrouped so every
    inverted list is one contiguous row range of the HBM index; a search probes the ``nprobe``
    nearest centroids and scans all (query, list, 1024-row chunk) work items in ONE fused
    scan + top-k launch (knn.hip cfc_ivf_topk, list-offset table on the device), then merges
    the candidates on the device -- no per-list launches, no host syncs before the results.
    Rows added after training form an unsorted tail scanned by the fused flat kernel until the
    next regroup.  k-means runs on a bf16 row sample (fp32 only for the sample and centroids:
    a 100M x 384 index never gets an fp32 copy); assignment of all rows is chunked bf16 GEMMs.

    Cosine / dot indexes are clustered CENTERED: the sample mean mu is removed before k-means
    (FAISS's centering pre-transform), and rows / queries are assigned by argmax (x - mu).c =
    x.c - mu.c -- mu only enters as a per-list bias, the stored rows stay untouched.  Encoder
    embeddings share a dominant common direction (random-init MiniLM rows are ~0.98 cosine to each
    other); uncentered, their scores against every centroid differ below bf16 resolution and one list
    took 74 % of a 10M-row index (profiles/r04_bench_ivf_10M.jsonl)."""

    SAMPLE_PER_LIST = 256
    ASSIGN_CHUNK = 1 << 20

    def __init__(self, dimension=384, distance="cosine", nlist: int = 0, nprobe: int = 8, **kw):
        super().__init__(dimension, distance, **kw)
        self.nlist, self.nprobe = int(nlist), int(nprobe)
        self.centroids: torch.Tensor | None = None
        self._list_off: list[int] = []
        self._list_off_t: torch.Tensor | None = None
        self._maxc = 1
        self._trained_n = 0
        self.center: torch.Tensor | None = None     # fp32 [dim] (cosine / dot), see the class note

    def train(self, sample: torch.Tensor | None = None, iters: int = 10, seed: int = 0) -> None:
        """k-means on the GPU over a sample of <= SAMPLE_PER_LIST rows per list, then regroup."""
        with self._lock:
            self.compact()
            n = self._n
            if n == 0:
                return
            nlist = self.nlist or max(1, int(math.sqrt(n)))
            g = torch.Generator(device="cpu").manual_seed(seed)
            if sample is None:
                m = min(n, max(nlist, self.SAMPLE_PER_LIST * nlist))
                idx = torch.randperm(n, generator=g)[:m].to(self.device)
                sample = self._X.index_select(0, idx)         # bf16 rows, no full-index copy
            X = sample.to(self.device).float()
            if self.metric != "l2":
                self.center = X.mean(0)
                X = X - self.center
            Xb = X.to(torch.bfloat16).contiguous()
            C = X[torch.randperm(X.shape[0], generator=g)[:nlist].to(self.device)].clone()
            if self.metric == "cosine":
                C = torch.nn.functional.normalize(C, dim=1)
            for _ in range(iters):
                a = self._nearest(Xb, C)
                sums = torch.zeros_like(C).index_add_(0, a, X)
                cnt = torch.bincount(a, minlength=C.shape[0])
                C = torch.where(cnt[:, None] > 0, sums / cnt.clamp_min(1).float()[:, None], C)   # keep empty lists' seeds
                if self.metric == "cosine":
                    C = torch.nn.functional.normalize(C, dim=1)
            self.centroids = C.to(torch.bfloat16)
            self.nlist = C.shape[0]
            self._regroup()

    def _center_bias(self, C: torch.Tensor) -> torch.Tensor | None:
        """-mu.c per list (None before a centered training)."""
        return None if self.center is None else -(C.float() @ self.center)

    def _nearest(self, X: torch.Tensor, C: torch.Tensor, extra_bias: torch.Tensor | None = None) -> torch.Tensor:
        """Nearest centroid of every row of bf16 X: argmax of x.c (cosine / dot) or of
        2 x.c - |c|^2 (L2), in ASSIGN_CHUNK-row pieces.  On the GPU the scores come from the
        hand-written MFMA GEMM (pgemm.hip) with the -|c|^2 term in its bias epilogue (the L2 form
        uses W = 2C) and the padding centroids' bias at -3e4; the argmax runs over bf16 scores."""
        from ..ops import kernels as K
        Cf = C.float()
        bias = -Cf.pow(2).sum(1) if self.metric == "l2" else torch.zeros(C.shape[0], device=C.device)
        if extra_bias is not None:
            bias = bias + extra_bias
        Wf = 2 * Cf if self.metric == "l2" else Cf
        use_hip = X.is_cuda and X.shape[1] % 64 == 0 and X.shape[0] >= 256
        if use_hip:
            npad = -(-C.shape[0] // 64) * 64
            Wb = torch.zeros(npad, X.shape[1], dtype=torch.bfloat16, device=X.device)
            Wb[:C.shape[0]] = Wf.to(torch.bfloat16)
            bb = torch.full((npad,), -3e4, dtype=torch.float32, device=X.device)
            bb[:C.shape[0]] = bias
            bb = bb.to(torch.bfloat16)
        out = []
        for s in range(0, X.shape[0], self.ASSIGN_CHUNK):
            xc = X[s:s + self.ASSIGN_CHUNK]
            if use_hip and xc.shape[0] >= 256:
                out.append(torch.argmax(K.pgemm(xc.contiguous(), Wb, "bias", bias=bb), 1))
            else:
                out.append(torch.argmax(xc.float() @ Wf.T + bias[None, :], 1))
        return torch.cat(out)

    def _assign(self, X: torch.Tensor) -> torch.Tensor:
        return self._nearest(X, self.centroids, self._center_bias(self.centroids))

    def _regroup(self):
        n = self._n
        a = self._assign(self._X[:n])
        order = torch.argsort(a, stable=True)
        self._X[:n] = self._X[:n].index_select(0, order)
        self._norm2[:n] = self._norm2[:n].index_select(0, order)
        self._alive[:n] = self._alive[:n].index_select(0, order)
        self._tab.permute(order.cpu().numpy())
        counts = torch.bincount(a, minlength=self.nlist)
        off = torch.zeros(self.nlist + 1, dtype=torch.int64, device=self.device)
        off[1:] = torch.cumsum(counts, 0)
        self._list_off_t = off
        self._list_off = off.cpu().tolist()
        R = 1024
        self._maxc = max(1, -(-int(counts.max()) // R)) if n else 1
        self._trained_n = n

    def compact(self) -> None:
        """Drop deleted rows; the survivors keep their order, so every list stays one contiguous
        range: its new offsets are the live-row prefix counts at the old ones."""
        with self._lock:
            if self._dead == 0 or self.centroids is None:
                return super().compact()
            pre = np.concatenate([[0], np.cumsum(self._tab.live.astype(np.int64))])
            old = np.asarray(self._list_off, dtype=np.int64)
            tn = int(pre[self._trained_n])
            super().compact()
            off = pre[old]
            self._list_off = off.tolist()
            self._list_off_t = torch.from_numpy(off).to(self.device)
            self._maxc = max(1, -(-int(np.diff(off).max()) // 1024)) if off.size > 1 else 1
            self._trained_n = tn

    def _extra_header(self) -> dict:
        if self.centroids is None:
            return {"ivf": None}
        return {"ivf": {"nlist": self.nlist, "nprobe": self.nprobe, "trained_rows": self._trained_n,
                        "list_off": self._list_off}}

    def _extra_tensors(self) -> dict:
        if self.centroids is None:
            return {}
        t = {"centroids": self.centroids.float().cpu()}
        if self.center is not None:
            t["center"] = self.center.float().cpu()
        return t

    def _restore_extra(self, meta: dict, path: Path) -> None:
        ivf = meta.get("ivf")
        if not ivf:
            return
        from safetensors.torch import load_file
        t = load_file(str(path / "ivf.safetensors"))
        self.centroids = t["centroids"].to(self.device).to(torch.bfloat16)
        self.center = t["center"].to(self.device) if "center" in t else None
        self.nlist, self.nprobe = int(ivf["nlist"]), int(ivf["nprobe"])
        self._trained_n = int(ivf["trained_rows"])
        self._list_off = [int(v) for v in ivf["list_off"]]
        self._list_off_t = torch.tensor(self._list_off, dtype=torch.int64, device=self.device)
        self._maxc = max(1, -(-max(b - a for a, b in zip(self._list_off, self._list_off[1:])) // 1024)) \
            if len(self._list_off) > 1 else 1

    def add_embeddings(self, ids, vectors, metadatas=None):
        super().add_embeddings(ids, vectors, metadatas)
        # rows appended after training form an unsorted tail scanned exhaustively until re-train
        if self.centroids is not None and self._n > 2 * max(self._trained_n, 1):
            self._regroup()

    def probe_lists(self, Q: torch.Tensor) -> torch.Tensor:
        """[nq, nprobe] int32 ids of each query's nearest lists (on the device)."""
        sc = Q.float() @ self.centroids.float().T
        if self.metric == "l2":
            sc = 2 * sc - self.centroids.float().pow(2).sum(1)[None, :]
        elif self.center is not None:
            sc = sc + self._center_bias(self.centroids)[None, :]
        return torch.topk(sc, min(self.nprobe, self.nlist), dim=1).indices.to(torch.int32).contiguous()

    def search(self, Q, k, rows=None):
        if self.centroids is None or rows is not None:
            return super().search(Q, k, rows)
        from ..ops import kernels as K
        Q = _as_matrix(Q, self.dim, device=self.device, dtype=torch.bfloat16)
        if self.metric == "cosine":
            Qn, qn2 = K.l2_normalize(Q.contiguous()), None
        else:
            Qn = Q.contiguous()
            qn2 = Qn.float().pow(2).sum(1)
        probe = self.probe_lists(Qn)
        xn2 = self._norm2 if self.metric == "l2" else None
        alive = self._alive if self._dead else None
        if not Q.is_cuda or k > 256:
            return self._search_ref(Qn, qn2, probe, k)
        cv, ci = K.ivf_topk(self._X, Qn, probe, self._list_off_t, self._maxc, k, xn2, qn2, alive)
        if self._n > self._trained_n:       # the unsorted tail, for every query
            tv, ti = [], []
            for s in range(0, Qn.shape[0], 16):
                v, i = K.knn_topk(self._X, Qn[s:s + 16], k, xn2, None if qn2 is None else qn2[s:s + 16], alive,
                                  row_lo=self._trained_n, N=self._n)
                tv.append(v)
                ti.append(i)
            cv, ci = torch.cat([cv, torch.cat(tv)], 1), torch.cat([ci, torch.cat(ti)], 1)
        return K.topk(cv, min(k, self.count()), ci)

    def _search_ref(self, Qn, qn2, probe, k):
        """CPU / large-k path: the probed lists' rows, exact scores, top-k (same results)."""
        rows = []
        for qi in range(Qn.shape[0]):
            rr = [torch.arange(self._list_off[c], self._list_off[c + 1]) for c in probe[qi].tolist()]
            rr.append(torch.arange(self._trained_n, self._n))
            rows.append(torch.cat(rr))
        vs, is_ = [], []
        for qi, r in enumerate(rows):
            r = r.to(self.device)
            X = self._X.index_select(0, r).float()
            sc = X @ Qn[qi].float()
            if self.metric == "l2":
                sc = -(self._norm2.index_select(0, r) + qn2[qi] - 2 * sc)
            sc = sc.masked_fill(~self._alive.index_select(0, r), float("-inf"))
            kk = min(k, sc.numel())
            v, i = torch.topk(sc, kk)
            pad = k - kk
            vs.append(torch.cat([v, v.new_full((pad,), float("-inf"))]))
            is_.append(torch.cat([r[i], r.new_full((pad,), -1)]))
        return torch.stack(vs), torch.stack(is_)


def create_vector_store(cfg=None, **overrides) -> VectorStore:
    name = str(getattr(cfg, "driver_name", cfg) or "hip").strip().lower()
    kw = {k: v for k, v in dict(getattr(cfg, "driver_config", {}) or {}).items() if v is not None}
    kw.update(overrides)
    if kw.get("index_type", "flat") not in ("flat", "ivf"):
        raise ValueError(f"unknown index_type {kw['index_type']!r} (flat or ivf)")
    if name == "hip":
        if kw.get("index_type", "flat") == "ivf":
            return HipIVFIndex(**kw)
        return HipFlatIndex(**kw)
    if name == "faiss":
        # FAISS parity (IndexFlatL2 semantics, score = 1/(1+d)) on the HIP index
        kw.setdefault("distance", "l2")
        return HipFlatIndex(faiss_scores=True, **kw) if kw.get("index_type", "flat") == "flat" else \
            HipIVFIndex(faiss_scores=True, **kw)
    if name == "inmemory":
        return InMemoryVectorStore(**kw)
    if name == "qdrant":
        from .remote import QdrantVectorStore
        return QdrantVectorStore(**kw)
    if name in ("azure_ai_search", "aisearch"):
        from .remote import AzureAISearchVectorStore
        return AzureAISearchVectorStore(**kw)
    raise ValueError(f"unknown vector_store driver {name!r}")
