"""Vector index sharded over ranks (one HBM-resident :class:`HipFlatIndex` shard per GPU).

A 288 GB MI355X holds ~350M x 384 bf16 vectors, so sharding is about aggregate scan bandwidth
(8 x 8 TB/s) more than capacity.  Query = every rank scans its shard with the fused MFMA kernel
and keeps its exact local top-k; the k candidates (score, owner rank, row) are all-gathered as one
small fp32 tensor over RCCL and merged with a top-k over world*k -- exact global top-k, traffic
O(world * nq * k) independent of the index size.  Ids/metadata of the winners are resolved with
one all_gather_object of the local candidates.

Insert modes:
  * ``add_embeddings`` -- replicated input (every rank sees the same batch); each rank stores only
    the ids it owns (sha1(id) % world), so upserts of an id always land on the same shard;
  * ``add_local`` -- rank-local input (each rank embedded its own chunks); owner = producer;
  * ``add_thread_rows`` -- rank-local input stored on the shard that owns each row's THREAD
    (sha1(thread_id) % world), with the orchestrator's thread-restricted relevance computed by the
    owner and returned: the DP orchestrator's data plane (every rank embeds its own batch, the
    vectors of a thread live on one GPU, two all_to_all exchanges over RCCL per batch).
All query methods are collectives: every rank of the group must call them with the same nq / k.

Reference query path: reporting topic search query(top_k=limit*3) (reporting/app/service.py:828),
FAISS IndexFlat search (faiss_store.py:214).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..vectorstore import HipFlatIndex, SearchResult, VectorStore, _as_matrix
from .dp import owner_of


class ShardedVectorIndex(VectorStore):
    def __init__(self, local: HipFlatIndex, group=None):
        self.local = local
        self.group = group
        self.dist = dist.is_initialized()
        self.rank = dist.get_rank(group) if self.dist else 0
        self.world = dist.get_world_size(group) if self.dist else 1
        self.dim = local.dim

    # ---------------------------------------------------------------- writes
    def add_embeddings(self, ids, vectors, metadatas=None):
        vecs = _as_matrix(vectors, self.dim)
        metadatas = list(metadatas) if metadatas is not None else [{} for _ in ids]
        mine = [j for j, i in enumerate(ids) if owner_of(i, self.world) == self.rank]
        if mine:
            self.local.add_embeddings([ids[j] for j in mine], vecs[mine], [metadatas[j] for j in mine])

    def add_local(self, ids, vectors, metadatas=None):
        self.local.add_embeddings(ids, vectors, metadatas)

    def delete(self, id):
        if self.local.has(id):
            self.local.delete(id)

    def clear(self):
        self.local.clear()

    def count(self) -> int:
        """Global count (collective)."""
        t = torch.tensor([self.local.count()], dtype=torch.int64, device=self._comm_device())
        if self.world > 1:
            dist.all_reduce(t, group=self.group)
        return int(t.item())

    def get(self, id):
        """Collective: the owner returns the vector, every rank receives it."""
        res = self.local.get(id) if self.local.has(id) else None
        if self.world == 1:
            if res is None:
                raise KeyError(id)
            return res
        out = [None] * self.world
        dist.all_gather_object(out, res, group=self.group)
        for r in out:
            if r is not None:
                return r
        raise KeyError(id)

    def add_thread_rows(self, thread_ids, ids, vectors, metadatas=None) -> torch.Tensor:
        """Collective.  Rows (each thread's rows consecutive) go to the shard owning their thread;
        the owner appends them (one thread's rows contiguous) and scores every row by cosine to its
        thread's centroid (HipFlatIndex.span_centroid_scores, the OrchestratorService relevance);
        the scores come back in input order, fp32 on the local device.  Stored metadata: the row's
        ``thread_id`` plus ``source_rank`` (only tensors cross the wire: vectors, fixed-width id
        bytes, thread lengths, scores -- RCCL all_to_all on GPUs, gloo on CPU)."""
        vecs = _as_matrix(vectors, self.dim, device=self.local.device, dtype=torch.bfloat16)
        n = len(ids)
        # thread spans of the input (consecutive rows) and their owners
        spans, start = [], 0
        for i in range(1, n + 1):
            if i == n or thread_ids[i] != thread_ids[start]:
                spans.append((thread_ids[start], start, i))
                start = i
        if len({t for t, _, _ in spans}) != len(spans):
            raise ValueError("add_thread_rows: each thread's rows must be consecutive")
        if self.world == 1:
            row0 = self.local._n
            self.local.add_embeddings(list(ids), vecs, [{"thread_id": t, "source_rank": 0} for t in thread_ids])
            return HipFlatIndex.span_centroid_scores(
                self.local._X, [(row0 + a, row0 + b) for _, a, b in spans]) if spans else vecs.new_zeros(0).float()
        W = self.world
        owner = [owner_of(t, W) for t, _, _ in spans]
        order = sorted(range(len(spans)), key=lambda j: owner[j])       # stable: input order per owner
        perm = [r for j in order for r in range(spans[j][1], spans[j][2])]
        send_rows = [0] * W
        send_thr = [0] * W
        for j in order:
            send_rows[owner[j]] += spans[j][2] - spans[j][1]
            send_thr[owner[j]] += 1
        dev = self._comm_device()
        cnt = torch.tensor(send_rows + send_thr, dtype=torch.int64).view(2, W).t().contiguous().view(-1).to(dev)
        rcnt = torch.empty_like(cnt)
        dist.all_to_all_single(rcnt, cnt, group=self.group)             # 2 numbers from every rank
        rc = rcnt.view(W, 2).cpu()
        recv_rows, recv_thr = rc[:, 0].tolist(), rc[:, 1].tolist()
        # ids and thread ids as fixed-width bytes (width agreed by a MAX all-reduce)
        keys = [f"{ids[r]}\x00{thread_ids[r]}".encode("utf-8") for r in perm]
        wid = torch.tensor([max((len(k) for k in keys), default=1)], dtype=torch.int64, device=dev)
        dist.all_reduce(wid, op=dist.ReduceOp.MAX, group=self.group)
        wid = -(-int(wid.item()) // 4) * 4           # int32 words on the wire (gloo has no 8/16-bit types)
        kb = torch.zeros(n, wid, dtype=torch.uint8)
        for i, k in enumerate(keys):
            kb[i, :len(k)] = torch.frombuffer(bytearray(k), dtype=torch.uint8)
        pidx = torch.tensor(perm, dtype=torch.long, device=vecs.device)
        if self.dim % 2:
            raise ValueError("add_thread_rows: odd dimension")
        xs = vecs.index_select(0, pidx).contiguous().view(torch.int32).to(dev)     # bf16 pairs as int32
        xr = torch.empty(sum(recv_rows), self.dim // 2, dtype=torch.int32, device=dev)
        dist.all_to_all_single(xr, xs, recv_rows, send_rows, group=self.group)
        kr = torch.empty(sum(recv_rows), wid // 4, dtype=torch.int32, device=dev)
        dist.all_to_all_single(kr, kb.view(torch.int32).to(dev), recv_rows, send_rows, group=self.group)
        kr = kr.cpu().view(torch.uint8)
        tl = torch.tensor([spans[j][2] - spans[j][1] for j in order], dtype=torch.int64, device=dev)
        tr = torch.empty(sum(recv_thr), dtype=torch.int64, device=dev)
        dist.all_to_all_single(tr, tl, recv_thr, send_thr, group=self.group)
        # owner side: append the received rows (threads contiguous), score them per thread
        m = sum(recv_rows)
        scores = torch.zeros(m, dtype=torch.float32, device=self.local.device)
        if m:
            recv = [bytes(r).rstrip(b"\x00").decode("utf-8").split("\x00", 1) for r in kr.numpy()]
            src = [r for r, c in enumerate(recv_rows) for _ in range(c)]
            row0 = self.local._n
            self.local.add_embeddings([k[0] for k in recv], xr.to(self.local.device).view(torch.bfloat16),
                                      [{"thread_id": k[1], "source_rank": s} for k, s in zip(recv, src)])
            lens = tr.cpu().tolist()
            sp, a = [], row0
            for L in lens:
                sp.append((a, a + L))
                a += L
            scores = HipFlatIndex.span_centroid_scores(self.local._X, sp)
        back = torch.empty(n, dtype=torch.float32, device=dev)
        dist.all_to_all_single(back, scores.to(dev).contiguous(), send_rows, recv_rows, group=self.group)
        out = torch.empty(n, dtype=torch.float32, device=self.local.device)
        out[pidx] = back.to(self.local.device)
        return out

    # ---------------------------------------------------------------- search
    def _comm_device(self):
        backend = dist.get_backend(self.group) if self.dist else None
        return self.local.device if backend == "nccl" else torch.device("cpu")

    def search(self, Q, k: int):
        """Global exact top-k: (scores [nq,k], owner rank [nq,k], local row [nq,k]); collective."""
        Q = _as_matrix(Q, self.dim)
        nq = Q.shape[0]
        kk = min(k, self.local.count())
        if kk > 0:
            v, i = self.local.search(Q, kk)
        else:
            v = torch.empty(nq, 0, device=self.local.device)
            i = torch.empty(nq, 0, dtype=torch.long, device=self.local.device)
        cand = torch.full((nq, k, 2), float("-inf"), dtype=torch.float32, device=self.local.device)
        cand[:, :v.shape[1], 0] = v.float()
        cand[:, :v.shape[1], 1] = i.float()  # rows < 2^24 per shard are exact in fp32
        cand[:, v.shape[1]:, 1] = -1
        dev = self._comm_device()
        cand = cand.to(dev)
        if self.world > 1:
            allc = [torch.empty_like(cand) for _ in range(self.world)]
            dist.all_gather(allc, cand, group=self.group)
            allc = torch.stack(allc, 0)              # [world, nq, k, 2]
        else:
            allc = cand[None]
        scores = allc[..., 0].permute(1, 0, 2).reshape(nq, self.world * k)
        rows = allc[..., 1].permute(1, 0, 2).reshape(nq, self.world * k)
        top = min(k, scores.shape[1])
        sv, si = torch.topk(scores, top, dim=1)
        owner = torch.div(si, k, rounding_mode="floor")
        row = torch.gather(rows, 1, si).long()
        return sv, owner, row

    def query_batch(self, query_vectors, top_k: int = 10, with_vectors: bool = False) -> list[list[SearchResult]]:
        sv, owner, row = self.search(query_vectors, top_k)
        sv, owner, row = sv.cpu(), owner.cpu(), row.cpu()
        # resolve winners owned here, then share the resolved records
        local: dict[int, tuple] = {}
        for r in row[owner == self.rank].tolist():
            if r >= 0 and r not in local and self.local._tab.id_at(r) is not None:
                vec = self.local._X[r].float().cpu().tolist() if with_vectors else []
                local[r] = (self.local._tab.id_at(r), vec, self.local._tab.meta_at(r))
        tables = [local]
        if self.world > 1:
            tables = [None] * self.world
            dist.all_gather_object(tables, local, group=self.group)
        out = []
        for q in range(sv.shape[0]):
            res = []
            for s, o, r in zip(sv[q].tolist(), owner[q].tolist(), row[q].tolist()):
                if s == float("-inf") or r < 0:
                    continue
                rec = tables[o].get(r)
                if rec is None:
                    continue
                if self.local.metric == "l2":
                    s = 1.0 / (1.0 + max(0.0, -s)) if self.local.faiss_scores else -s
                res.append(SearchResult(rec[0], float(s), rec[1], rec[2]))
            out.append(res)
        return out

    def query(self, query_vector, top_k: int = 10):
        return self.query_batch(_as_matrix(query_vector, self.dim), top_k)[0]
