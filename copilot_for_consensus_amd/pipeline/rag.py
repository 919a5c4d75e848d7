"""In-process, batched RAG pipeline: ingest -> parse -> chunk -> embed -> index -> select -> prompt
(-> summarize, done by the caller's LLM engine) -> summaries / reports.

This is the reference's six-service event flow collapsed into one process per GPU
with the same documents, ids, events and schemas, minus the per-item hops the survey lists as hot
loops: documents are inserted in batches, every chunk of a step is embedded in a few packed
encoder forwards, vectors go from the encoder to the HBM index without leaving the GPU, and the
orchestrator scores candidates for 16 threads per fused HIP kNN scan.

Stage events (ArchiveIngested, JSONParsed, ChunksPrepared, EmbeddingsGenerated,
SummarizationRequested, SummaryComplete, ReportPublished) are built and schema-validated exactly
as the services publish them; they go to ``publisher`` (a recording NoopPublisher by default).

Reference: orchestrator context selection (orchestrator/app/context_selectors.py:17,95-107;
context_sources.py:21,57-64) and the summarization request path
(summarization/app/service.py:289).
"""
from __future__ import annotations

import dataclasses
import hashlib
import time
from datetime import datetime, timezone

import torch

from ..archive import InMemoryArchiveStore
from ..bus import NoopPublisher, ValidatingEventPublisher
from ..chunking import Thread as ChunkThread
from ..chunking import TokenWindowChunker
from ..contracts import ids as cids
from ..contracts.events import EXCHANGE, Event, utc_now_iso
from ..orchestration import (TopKRelevanceSelector, build_context, format_citations, prompt_template,
                             substitute_prompt)
from ..parsing import MessageParser, ThreadBuilder
from ..storage.document_store import DocumentAlreadyExistsError, InMemoryDocumentStore
from ..utils.synthetic import SyntheticArchive


@dataclasses.dataclass
class PreparedBatch:
    threads: list[dict]
    prompts: list[list[int]]
    prompt_texts: list[str]
    selections: list
    contexts: list[dict]
    stage_s: dict[str, float]
    archive_id: str


class RagPipeline:
    def __init__(self, encoder: str = "minilm-l6", device="cuda", decoder_vocab: int = 32000, bos_id: int = 1,
                 seed: int = 0, top_k: int = 5, context_window_tokens: int = 2048, index_prefill: int = 1_000_000,
                 publisher=None, validate_events: bool = True, llm_model: str = "mistral-7b",
                 max_prompt_tokens: int | None = None, index_group=None):
        from ..embedding import HipEncoderProvider
        from ..runtime.tokenizer import synthetic_bpe
        from ..vectorstore import HipFlatIndex
        self.device = torch.device(device)
        self.embedder = HipEncoderProvider(model_name=encoder, device=str(self.device), seed=seed)
        self.bpe = synthetic_bpe(decoder_vocab)
        self.bos_id = bos_id
        self.docs = InMemoryDocumentStore()
        self.archives = InMemoryArchiveStore()
        self.local_index = HipFlatIndex(dimension=self.embedder.dimension, distance="cosine",
                                        capacity=index_prefill + (1 << 18), device=str(self.device))
        # DP ranks (index_group): one logical index sharded over the GPUs -- each rank's shard holds
        # its 1M prefill rows and the chunk vectors of the threads it owns (parallel/knn.py
        # add_thread_rows: vectors out and relevance scores back over RCCL every batch)
        self.sharded = None
        if index_group is not None:
            from ..parallel.knn import ShardedVectorIndex
            self.sharded = ShardedVectorIndex(self.local_index, group=index_group)
        self.index = self.local_index
        if index_prefill:
            g = torch.Generator(device=self.device).manual_seed(seed + 99)
            noise = torch.randn(index_prefill, self.embedder.dimension, device=self.device, generator=g)
            self.index.add_embeddings([f"prefill-{i}" for i in range(index_prefill)], noise,
                                      [{} for _ in range(index_prefill)])
        self.parser = MessageParser()
        self.threads = ThreadBuilder()
        self.chunker = TokenWindowChunker()
        self.selector = TopKRelevanceSelector()
        self.top_k, self.budget = top_k, context_window_tokens
        self.template = prompt_template()
        self.pub = publisher or NoopPublisher()
        if validate_events:
            self.pub = ValidatingEventPublisher(self.pub)
        self.generator = SyntheticArchive(seed=seed)
        self.sources: dict[int, bytes] = {}
        self.llm_model = llm_model
        self.max_prompt_tokens = max_prompt_tokens

    # ------------------------------------------------------------------ data source
    def prepare_sources(self, n_threads: int, steps: list[int]) -> None:
        """Pre-generate the step archives (the remote mailing list; not part of the timed work)."""
        for s in steps:
            if s not in self.sources:
                self.sources[s] = self.generator.mbox(n_threads)

    def _publish(self, event_type: str, **data) -> None:
        ev = Event.create(event_type, **data)
        self.pub.publish(EXCHANGE, ev.routing_key, ev.to_dict())

    # ------------------------------------------------------------------ stages
    def prepare(self, n_threads: int, step: int) -> PreparedBatch:
        st: dict[str, float] = {}
        t = time.perf_counter()
        raw = self.sources.pop(step, None) or self.generator.mbox(n_threads)
        started = utc_now_iso()
        aid = self.archives.store_archive("bench", f"step{step}.mbox", raw)
        sha = hashlib.sha256(raw).hexdigest()
        try:
            self.docs.insert_document("archives", {"_id": aid, "file_hash": sha, "file_size_bytes": len(raw),
                                                   "source": "bench", "ingestion_date": started, "status": "pending"})
        except DocumentAlreadyExistsError:
            pass    # the same synthetic archive again (content-addressed id): nothing new to record
        self._publish("ArchiveIngested", archive_id=aid, source_name="bench", source_type="local",
                      source_url=f"file:///bench/step{step}.mbox", file_size_bytes=len(raw), file_hash_sha256=sha,
                      ingestion_started_at=started, ingestion_completed_at=utc_now_iso())
        st["ingest"] = time.perf_counter() - t

        t = time.perf_counter()
        msgs, _errs = self.parser.parse_mbox_bytes(raw, aid)
        threads = self.threads.build_threads(msgs)
        self.docs.insert_many("messages", msgs)
        self.docs.insert_many("threads", threads)
        self.docs.update_document("archives", aid, {"status": "completed", "message_count": len(msgs)})
        self._publish("JSONParsed", archive_id=aid, message_count=len(msgs), message_doc_ids=[m["_id"] for m in msgs],
                      thread_count=len(threads), thread_ids=[x["_id"] for x in threads],
                      parsing_duration_seconds=round(time.perf_counter() - t, 6))
        st["parse"] = time.perf_counter() - t

        t = time.perf_counter()
        now = utc_now_iso()
        chunk_docs = []
        by_thread: dict[str, list[dict]] = {}
        for m in msgs:
            if not m["body_normalized"].strip():
                continue
            meta = {"sender": (m.get("from") or {}).get("email", ""), "subject": m.get("subject", ""),
                    "date": m.get("date")}
            for c in self.chunker.chunk(ChunkThread(m["thread_id"], m["body_normalized"], meta, m["_id"],
                                                    m["message_id"])):
                d = {"_id": c.chunk_id, "message_doc_id": c.message_doc_id, "message_id": m["message_id"],
                     "thread_id": c.thread_id, "archive_id": aid, "chunk_index": c.chunk_index, "text": c.text,
                     "token_count": c.token_count, "metadata": c.metadata, "created_at": now,
                     "embedding_generated": False}
                chunk_docs.append(d)
                by_thread.setdefault(c.thread_id, []).append(d)
        self.docs.insert_many("chunks", chunk_docs)
        self._publish("ChunksPrepared", message_doc_ids=[m["_id"] for m in msgs], chunk_count=len(chunk_docs),
                      chunk_ids=[c["_id"] for c in chunk_docs], chunks_ready=True,
                      chunking_strategy=self.chunker.strategy,
                      avg_chunk_size_tokens=int(sum(c["token_count"] for c in chunk_docs) / max(1, len(chunk_docs))))
        st["chunk"] = time.perf_counter() - t

        # embed (packed varlen encoder on the GPU) -> HBM index, rows grouped per thread
        t = time.perf_counter()
        order = [c for tid in by_thread for c in by_thread[tid]]
        vecs = self.embedder.embed_tensor([c["text"] for c in order])
        row0 = self.index._n
        sharded_scores = None
        if self.sharded is not None:
            # insert on the owning shards + the owners' thread-restricted relevance (collective)
            sharded_scores = self.sharded.add_thread_rows([c["thread_id"] for c in order], [c["_id"] for c in order],
                                                          vecs)
        else:
            self.index.add_embeddings([c["_id"] for c in order], vecs,
                                      [{"thread_id": c["thread_id"], "message_id": c["message_id"]} for c in order])
        self.docs.update_many("chunks", {"_id": {"$in": [c["_id"] for c in order]}}, {"embedding_generated": True})
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dt = time.perf_counter() - t
        self._publish("EmbeddingsGenerated", chunk_ids=[c["_id"] for c in order], embedding_count=len(order),
                      embedding_model=self.embedder.model_name, embedding_backend="hip",
                      embedding_dimension=self.embedder.dimension, vector_store_collection="embeddings",
                      vector_store_updated=True, avg_generation_time_ms=1000 * dt / max(1, len(order)))
        st["embed"] = dt

        # orchestrate: the service's relevance (OrchestratorService.candidates): every chunk scored by
        # cosine to its thread's centroid, a search restricted to the thread's own rows of the HBM
        # index -- here all threads of the batch in one segment pass over their (consecutive) rows
        t = time.perf_counter()
        tids = list(by_thread)
        spans, r = [], row0
        for tid in tids:
            spans.append((r, r + len(by_thread[tid])))
            r += len(by_thread[tid])
        sc = (sharded_scores if sharded_scores is not None
              else self.index.span_centroid_scores(self.index._X, spans)).cpu().tolist()
        cand_scores = {c["_id"]: s for c, s in zip(order, sc)}
        prepared_threads, prompts, texts, sels, ctxs = [], [], [], [], []
        msg_by_id = {m["_id"]: m for m in msgs}
        thread_docs = {x["_id"]: x for x in threads}
        for tid in tids:
            cands = []
            for c in by_thread[tid]:
                cc = dict(c)
                cc["similarity_score"] = cand_scores[c["_id"]]
                cc["source_type"] = "vector_store"
                cands.append(cc)
            sel = self.selector.select(tid, cands, self.top_k, self.budget)
            chosen = {s_.chunk_id for s_ in sel.selected_chunks}
            ordered = [c for s_ in sel.selected_chunks for c in by_thread[tid] if c["_id"] == s_.chunk_id]
            ctx = build_context(ordered, msg_by_id)
            prompt = substitute_prompt(self.template, tid, ctx)
            self._publish("SummarizationRequested", thread_ids=[tid], top_k=self.top_k, prompt_template=self.template,
                          selected_chunks=[s_.to_dict() for s_ in sel.selected_chunks],
                          context_selection=sel.metadata())
            del chosen
            prepared_threads.append(thread_docs[tid])
            texts.append(prompt)
            sels.append(sel)
            ctxs.append(ctx)
        st["select"] = time.perf_counter() - t

        t = time.perf_counter()
        prompts = [self._clip(ids) for ids in self.bpe.encode_batch(texts)]
        st["tokenize"] = time.perf_counter() - t
        return PreparedBatch(prepared_threads, prompts, texts, sels, ctxs, st, aid)

    def _clip(self, ids: list[int]) -> list[int]:
        """Keep the instructions (head) and the latest excerpts (tail) if a prompt exceeds the context."""
        L = self.max_prompt_tokens
        if L is None or len(ids) <= L:
            return ids
        half = L // 2
        return ids[:half] + ids[-(L - half):]

    def finish(self, batch: PreparedBatch, gen) -> list[dict]:
        """Detokenise, build citations + ids, persist summaries, update threads, emit events."""
        reports = []
        now = datetime.now(timezone.utc).isoformat().replace("+00:00", "Z")
        for th, ctx, toks, p in zip(batch.threads, batch.contexts, gen.tokens, batch.prompts):
            text = self.bpe.decode(toks).strip() or "(empty summary)"
            cites = format_citations(ctx["chunks"])
            sid = cids.summary_id(th["_id"], [c["chunk_id"] for c in cites])
            self._publish("SummaryComplete", summary_id=sid, thread_id=th["_id"], summary_markdown=text,
                          citations=cites, llm_backend="hip", llm_model=self.llm_model, tokens_prompt=len(p),
                          tokens_completion=len(toks), latency_ms=int(1000 * gen.total_s))
            rid = cids.report_id(sid)
            doc = {"_id": rid, "thread_id": th["_id"], "summary_type": "thread", "title": th.get("subject", ""),
                   "content_markdown": text, "citations": cites, "generated_by": self.llm_model, "generated_at": now,
                   "first_message_date": th.get("first_message_date"), "last_message_date": th.get("last_message_date"),
                   "metadata": {"summary_id": sid, "tokens_prompt": len(p), "tokens_completion": len(toks)}}
            try:
                self.docs.insert_document("summaries", doc)
            except DocumentAlreadyExistsError:
                self.docs.update_document("summaries", rid, doc)    # regenerated: the newest summary wins
            self.docs.update_document("threads", th["_id"], {"summary_id": rid})
            self._publish("ReportPublished", thread_id=th["_id"], report_id=rid, format="markdown", notified=False,
                          delivery_channels=["api"], summary_url=f"/api/reports/{rid}")
            reports.append(doc)
        return reports
