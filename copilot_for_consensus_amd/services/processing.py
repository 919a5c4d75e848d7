"""The five bus-driven processing services: parsing, chunking, embedding, orchestrator, summarization.

Each mirrors its reference service's event contract and forward-progress behaviour (SURVEY §3.3,
§3.5): consume the upstream event with the retry policy, read documents (eventual-consistency
misses raise DocumentNotFoundError -> jittered retry), write documents idempotently (deterministic
ids, duplicate inserts tolerated), publish the downstream event or the stage's *Failed event,
requeue incomplete work at startup, and delete a source's documents on SourceDeletionRequested
(reporting a SourceCleanupProgress).

MI355X differences: embedding embeds a whole ChunksPrepared batch in packed encoder forwards and
keeps vectors in HBM; summarization micro-batches SummarizationRequested events (up to
``max_batch_threads`` threads or ``batch_wait_ms``) into one engine.generate call.
"""
from __future__ import annotations

import threading
import time
from datetime import datetime, timezone

from ..chunking import Thread as ChunkThread
from ..chunking import ThreadChunker, TokenWindowChunker
from ..contracts import ids as cids
from ..contracts.events import utc_now_iso
from ..orchestration import (TopKRelevanceSelector, build_context, create_context_selector, format_citations,
                             prompt_template, substitute_prompt)
from ..parsing import MessageParser, ThreadBuilder
from ..retry import DocumentNotFoundError, RetryExhaustedError, retry_with_backoff
from ..storage.document_store import DocumentAlreadyExistsError
from ..summarization import Summarizer
from ..summarization import Thread as SumThread
from .base import BaseService


def _now() -> str:
    return datetime.now(timezone.utc).isoformat().replace("+00:00", "Z")


class _CleanupMixin:
    """SourceDeletionRequested -> delete this service's documents of the source's archives."""

    cleanup_collections: tuple[str, ...] = ()

    def _handle_source_deletion(self, event: dict) -> None:
        d = event["data"]
        archive_ids = d.get("archive_ids") or [a["_id"] for a in self.store.query_documents(
            "archives", {"source": d["source_name"]}, limit=1 << 30)]
        counts = {}
        for coll in self.cleanup_collections:
            counts[coll] = self.store.delete_many(coll, {"archive_id": {"$in": archive_ids}})
        self.publish("SourceCleanupProgress", source_name=d["source_name"], correlation_id=d["correlation_id"],
                     service_name=self.name, status="completed", deletion_counts=counts, completed_at=utc_now_iso())


class ParsingService(_CleanupMixin, BaseService):
    name = "parsing"
    cleanup_collections = ("messages", "threads")

    def __init__(self, publisher, subscriber, document_store, archive_store, parser: MessageParser | None = None,
                 **kw):
        super().__init__(publisher, subscriber, document_store, **kw)
        self.archives = archive_store
        self.parser = parser or MessageParser()
        self.threads = ThreadBuilder()
        self._parsed: dict[str, int] = {}    # archive_id -> messages parsed by the current attempt

    def _set_archive_status(self, archive_id: str, fields: dict) -> None:
        """Archive status is bookkeeping: a store outage must not fail the parse, but is logged and
        counted (a lost update leaves the archive 'processing' until requeue_incomplete)."""
        try:
            self.store.update_document("archives", archive_id, fields)
        except Exception as e:  # noqa: BLE001 -- logged + counted, the parse result stands
            self.log.warning("archive status update failed", archive_id=archive_id, status=fields.get("status"),
                             error=repr(e))
            self.metrics.increment("parsing_archive_status_update_failures_total",
                                   tags={"status": str(fields.get("status"))})

    def subscriptions(self):
        return {"ArchiveIngested": self._on_archive, "SourceDeletionRequested": self._handle_source_deletion}

    def _on_archive(self, event: dict) -> None:
        self.process_archive(event["data"]["archive_id"])

    def process_archive(self, archive_id: str) -> dict | None:
        raw = self.archives.get_archive(archive_id)
        if raw is None:
            raise DocumentNotFoundError(f"archive {archive_id} not in archive store yet")
        t = time.perf_counter()
        self._set_archive_status(archive_id, {"status": "processing", "lastAttemptTime": _now()})
        msgs, errs = self.parser.parse_mbox_bytes(raw, archive_id)
        self._parsed[archive_id] = len(msgs)
        threads = self.threads.build_threads(msgs)
        self.store.insert_many("messages", msgs)
        self.store.insert_many("threads", threads)
        self._set_archive_status(archive_id, {"status": "completed", "message_count": len(msgs),
                                              "lastUpdated": _now()})
        self._parsed.pop(archive_id, None)
        self.metrics.increment("parsing_messages_parsed_total", len(msgs))
        self.metrics.observe("parsing_duration_seconds", time.perf_counter() - t)
        # one JSONParsed per message (reference parsing/app/service.py:681-740): downstream
        # chunking fans out per message; the payload lists stay schema-valid
        for m in msgs:
            self.publish("JSONParsed", archive_id=archive_id, message_count=1, message_doc_ids=[m["_id"]],
                         thread_count=1, thread_ids=[m["thread_id"]],
                         parsing_duration_seconds=round(time.perf_counter() - t, 6))
        return {"messages": len(msgs), "threads": len(threads), "errors": errs,
                "message_doc_ids": [m["_id"] for m in msgs], "thread_ids": [x["_id"] for x in threads]}

    def on_failure(self, event_type, event, error):
        if event_type == "ArchiveIngested":
            aid = event["data"]["archive_id"]
            self._set_archive_status(aid, {"status": "failed", "lastUpdated": _now()})
            ctx = getattr(error, "context", None)       # RetryExhaustedError carries the retry context
            retries = max(0, int(getattr(ctx, "attempt_number", 1)) - 1) if ctx is not None else 0
            cause = error.__cause__ if isinstance(error, RetryExhaustedError) and error.__cause__ else error
            self.publish("ParsingFailed", archive_id=aid, error_message=str(cause) or type(cause).__name__,
                         error_type=type(cause).__name__,
                         messages_parsed_before_failure=self._parsed.pop(aid, 0), retry_count=retries,
                         failed_at=utc_now_iso())

    def requeue_incomplete(self):
        n = 0
        for a in self.store.query_documents("archives", {"status": {"$in": ["pending", "processing"]}}, limit=10000):
            self.publish("ArchiveIngested", archive_id=a["_id"], source_name=a.get("source", "unknown"),
                         source_type=a.get("source_type") or "local", source_url=a.get("source_url") or a.get("file_path") or "requeue",
                         file_size_bytes=int(a.get("file_size_bytes", 0)), file_hash_sha256=a.get("file_hash", "-"),
                         ingestion_started_at=a.get("ingestion_date") or utc_now_iso(),
                         ingestion_completed_at=utc_now_iso())
            n += 1
        return n


class ChunkingService(_CleanupMixin, BaseService):
    name = "chunking"
    cleanup_collections = ("chunks",)

    def __init__(self, publisher, subscriber, document_store, chunker: ThreadChunker | None = None, **kw):
        super().__init__(publisher, subscriber, document_store, **kw)
        self.chunker = chunker or TokenWindowChunker()

    def subscriptions(self):
        return {"JSONParsed": self._on_parsed, "SourceDeletionRequested": self._handle_source_deletion}

    def _on_parsed(self, event):
        self.process_messages(event["data"]["message_doc_ids"])

    def process_messages(self, message_doc_ids: list[str]) -> list[str]:
        msgs = self.store.query_documents("messages", {"_id": {"$in": list(message_doc_ids)}},
                                          limit=len(message_doc_ids))
        if len(msgs) < len(set(message_doc_ids)):
            raise DocumentNotFoundError(f"{len(set(message_doc_ids)) - len(msgs)} messages not visible yet")
        now = _now()
        docs = []
        for m in msgs:
            if not (m.get("body_normalized") or "").strip():
                continue
            meta = {"sender": (m.get("from") or {}).get("email", ""), "subject": m.get("subject", ""),
                    "date": m.get("date")}
            for c in self.chunker.chunk(ChunkThread(m["thread_id"], m["body_normalized"], meta, m["_id"],
                                                    m["message_id"])):
                docs.append({"_id": c.chunk_id, "message_doc_id": c.message_doc_id, "message_id": m["message_id"],
                             "thread_id": c.thread_id, "archive_id": m.get("archive_id"),
                             "chunk_index": c.chunk_index, "text": c.text, "token_count": c.token_count,
                             "metadata": c.metadata, "created_at": now, "embedding_generated": False})
        if not docs:  # only empty bodies: nothing to embed (and ChunksPrepared needs >= 1 chunk id)
            self.metrics.increment("chunking_empty_messages_total", len(msgs))
            return []
        self.store.insert_many("chunks", docs)  # duplicate ids tolerated (idempotent)
        self.metrics.increment("chunking_chunks_created_total", len(docs))
        self.publish("ChunksPrepared", message_doc_ids=list(message_doc_ids), chunk_count=len(docs),
                     chunk_ids=[d["_id"] for d in docs], chunks_ready=True,
                     chunking_strategy=getattr(self.chunker, "strategy", "token_window"),
                     avg_chunk_size_tokens=int(sum(d["token_count"] for d in docs) / max(1, len(docs))))
        return [d["_id"] for d in docs]

    def on_failure(self, event_type, event, error):
        if event_type == "JSONParsed":
            self.publish("ChunkingFailed", message_doc_ids=event["data"]["message_doc_ids"],
                         error_message=str(error) or type(error).__name__, error_type=type(error).__name__,
                         retry_count=0, failed_at=utc_now_iso())

    def requeue_incomplete(self):
        # messages without chunks: republish JSONParsed for them in groups of 100
        chunked = {c["message_doc_id"] for c in self.store.query_documents("chunks", {}, limit=1 << 30)}
        pending = [m for m in self.store.query_documents("messages", {}, limit=1 << 30) if m["_id"] not in chunked]
        for s in range(0, len(pending), 100):
            grp = pending[s:s + 100]
            self.publish("JSONParsed", archive_id=grp[0]["archive_id"], message_count=len(grp),
                         message_doc_ids=[m["_id"] for m in grp], thread_count=len({m["thread_id"] for m in grp}),
                         thread_ids=sorted({m["thread_id"] for m in grp}), parsing_duration_seconds=0.0)
        return len(pending)


class EmbeddingService(BaseService):
    name = "embedding"

    def __init__(self, publisher, subscriber, document_store, embedding_provider, vector_store,
                 max_retries: int = 3, retry_backoff_seconds: float = 5.0, max_batch_chunks: int = 4096,
                 batch_wait_ms: int = 20, **kw):
        super().__init__(publisher, subscriber, document_store, **kw)
        self.embedder, self.vectors = embedding_provider, vector_store
        self.max_retries, self.backoff = max_retries, retry_backoff_seconds
        # micro-batching (start_async): ChunksPrepared events of many messages -> one encoder batch
        self.max_batch_chunks, self.batch_wait = int(max_batch_chunks), batch_wait_ms / 1000.0
        self._queue: list[dict] = []
        self._qlock = threading.Condition()
        self._worker: threading.Thread | None = None
        self._stop = False

    def subscriptions(self):
        return {"ChunksPrepared": self._on_chunks, "SourceDeletionRequested": self._on_delete}

    def _on_chunks(self, event):
        if self._worker is not None:
            with self._qlock:
                self._queue.append(event)
                self._qlock.notify()
            return
        self.process_chunks(event["data"]["chunk_ids"])

    def start_async(self) -> None:
        """Batch ChunksPrepared events (<= max_batch_chunks chunks or batch_wait_ms) into one
        encoder call on this service's own GPU stream; a failing batch is retried event by event
        so one bad message fails alone."""
        from .base import own_gpu_stream

        def loop():
            own_gpu_stream()
            while True:
                with self._qlock:
                    if not self._queue:
                        if self._stop:
                            break          # stopped and drained: no acked ChunksPrepared is dropped
                        self._qlock.wait(0.1)
                        continue
                    deadline = time.time() + (0.0 if self._stop else self.batch_wait)
                    while (sum(len(e["data"]["chunk_ids"]) for e in self._queue) < self.max_batch_chunks
                           and time.time() < deadline):
                        self._qlock.wait(max(0.0, deadline - time.time()))
                    batch, n = [], 0
                    while self._queue and (not batch or n + len(self._queue[0]["data"]["chunk_ids"])
                                           <= self.max_batch_chunks):
                        ev = self._queue.pop(0)
                        batch.append(ev)
                        n += len(ev["data"]["chunk_ids"])
                try:
                    self.process_chunks([c for ev in batch for c in ev["data"]["chunk_ids"]])
                except Exception:  # noqa: BLE001 -- isolate: each event on its own, with the retry policy
                    for ev in batch:
                        try:
                            self._wrap("ChunksPrepared", lambda e: self.process_chunks(e["data"]["chunk_ids"]))(ev)
                        except Exception as e:  # noqa: BLE001 -- already reported by the wrapper
                            self.log.error("embedding event failed", error=repr(e))
        self._worker = threading.Thread(target=loop, name="embedding-batcher", daemon=True)
        self._worker.start()

    def stop_async(self, timeout: float = 120.0) -> None:
        """Stop the batcher after it embedded every queued event (their bus messages were acked
        when queued, so dropping them would lose the chunks until a restart's requeue)."""
        with self._qlock:
            self._stop = True
            self._qlock.notify_all()
        if self._worker is not None:
            self._worker.join(timeout=timeout)
            if not self._worker.is_alive():
                self._worker = None

    def process_chunks(self, chunk_ids: list[str]) -> int:
        if not chunk_ids:
            return 0
        chunks = self.store.query_documents("chunks", {"_id": {"$in": list(chunk_ids)}, "embedding_generated": False},
                                            limit=len(chunk_ids))
        if not chunks:
            done = self.store.count_documents("chunks", {"_id": {"$in": list(chunk_ids)}})
            if done < len(set(chunk_ids)):
                raise DocumentNotFoundError("chunks not visible yet")
            return 0  # already embedded (idempotent replay)
        # each thread's chunks consecutive (first-appearance order): a thread-sharded index takes a
        # thread's rows as one span, and the HBM index keeps them adjacent for the centroid pass
        first: dict[str, int] = {}
        for c in chunks:
            first.setdefault(c["thread_id"], len(first))
        chunks.sort(key=lambda c: first[c["thread_id"]])
        t = time.perf_counter()
        metas = [{"thread_id": c["thread_id"], "message_id": c["message_id"], "message_doc_id": c["message_doc_id"],
                  "chunk_index": c["chunk_index"]} for c in chunks]
        model, backend, dim = self.embedder.model_name, self.embedder.backend, int(self.embedder.dimension)
        if hasattr(self.vectors, "embed_and_store"):
            # data-parallel node (parallel/dp_node.py): each thread's chunks are embedded on, and
            # stay in the HBM index shard of, the GPU that owns the thread
            info = retry_with_backoff(lambda: self.vectors.embed_and_store(
                [{"id": c["_id"], "thread_id": c["thread_id"], "text": c["text"], "meta": m}
                 for c, m in zip(chunks, metas)]), self.max_retries, self.backoff)
            model, backend, dim = info["model"], info["backend"], int(info["dimension"])
            dt = time.perf_counter() - t
        else:
            vecs = retry_with_backoff(lambda: self.embedder.embed_tensor([c["text"] for c in chunks]),
                                      self.max_retries, self.backoff)
            dt = time.perf_counter() - t
            self.vectors.add_embeddings([c["_id"] for c in chunks], vecs, metas)
            if getattr(vecs, "is_cuda", False):
                # the index rows are written on this thread's stream; readers (the orchestrator) use
                # their own: the rows must be in HBM before the event that announces them
                import torch
                torch.cuda.current_stream(vecs.device).synchronize()
        self.store.update_many("chunks", {"_id": {"$in": [c["_id"] for c in chunks]}},
                               {"embedding_generated": True, "lastUpdated": _now()})
        self.metrics.increment("embedding_chunks_processed_total", len(chunks))
        self.metrics.observe("embedding_generation_duration_seconds", dt)
        self.publish("EmbeddingsGenerated", chunk_ids=[c["_id"] for c in chunks], embedding_count=len(chunks),
                     embedding_model=model, embedding_backend=backend,
                     embedding_dimension=dim, vector_store_collection="embeddings",
                     vector_store_updated=True, avg_generation_time_ms=1000 * dt / len(chunks))
        return len(chunks)

    def _on_delete(self, event):
        d = event["data"]
        archive_ids = d.get("archive_ids") or []
        n = 0
        for c in self.store.query_documents("chunks", {"archive_id": {"$in": archive_ids}}, limit=1 << 30):
            try:
                self.vectors.delete(c["_id"])
                n += 1
            except KeyError:
                pass
        self.publish("SourceCleanupProgress", source_name=d["source_name"], correlation_id=d["correlation_id"],
                     service_name=self.name, status="completed", deletion_counts={"vectors": n},
                     completed_at=utc_now_iso())

    def on_failure(self, event_type, event, error):
        if event_type == "ChunksPrepared":
            self.publish("EmbeddingGenerationFailed", chunk_ids=event["data"]["chunk_ids"] or ["none"],
                         error_message=str(error) or type(error).__name__, error_type=type(error).__name__,
                         embedding_backend=getattr(self.embedder, "backend", "unknown"), retry_count=self.max_retries,
                         failed_at=utc_now_iso())

    def requeue_incomplete(self):
        pending = self.store.query_documents("chunks", {"embedding_generated": False}, limit=1 << 30)
        for s in range(0, len(pending), 512):
            grp = pending[s:s + 512]
            self.publish("ChunksPrepared", message_doc_ids=sorted({c["message_doc_id"] for c in grp}),
                         chunk_count=len(grp), chunk_ids=[c["_id"] for c in grp], chunks_ready=True,
                         chunking_strategy="requeue", avg_chunk_size_tokens=0)
        return len(pending)


class OrchestratorService(BaseService):
    name = "orchestrator"

    def __init__(self, publisher, subscriber, document_store, vector_store=None, top_k: int = 5,
                 context_window_tokens: int = 2048, chunk_selection_strategy: str = "top_k_relevance",
                 system_prompt_path: str | None = None, user_prompt_path: str | None = None,
                 consensus_detector=None, **kw):
        super().__init__(publisher, subscriber, document_store, **kw)
        self.vectors = vector_store
        # optional: annotate threads with has_consensus / consensus_type (the threads schema carries
        # these fields; the reference ships the detector but never calls it)
        self.consensus = consensus_detector
        self.top_k, self.budget = top_k, context_window_tokens
        self.selector = create_context_selector(chunk_selection_strategy)
        self.template = prompt_template(system_prompt_path, user_prompt_path)

    def subscriptions(self):
        return {"EmbeddingsGenerated": self._on_embeddings}

    def _on_embeddings(self, event):
        self.process_embeddings(event["data"]["chunk_ids"])

    def _resolve_threads(self, chunk_ids):
        chunks = self.store.query_documents("chunks", {"_id": {"$in": list(chunk_ids)}}, limit=len(chunk_ids))
        if not chunks and chunk_ids:
            raise DocumentNotFoundError("chunks not visible yet")
        return sorted({c["thread_id"] for c in chunks})

    @staticmethod
    def _scored(chunks: list[dict], scores: dict[str, float]) -> list[dict]:
        missing = 0.0 if scores else 0.5        # neutral score (context_sources.py:21) only when none scored
        out = []
        for c in chunks:
            cc = dict(c)
            cc["similarity_score"] = scores.get(c["_id"], missing)
            cc["source_type"] = "vector_store" if c["_id"] in scores else "thread_chunks"
            out.append(cc)
        return out

    def candidates_many(self, thread_ids: list[str]) -> dict[str, list[dict]]:
        """candidates() of many threads with ONE vector-store pass (centroid_scores_many: a single
        gather + segment reduction on the HBM index instead of one search per thread)."""
        chunks = {tid: self.store.query_documents("chunks", {"thread_id": tid}, limit=1 << 20) for tid in thread_ids}
        scores: list[dict] = [{} for _ in thread_ids]
        many = getattr(self.vectors, "centroid_scores_many", None)
        if self.vectors is not None and many is not None and not getattr(self.vectors, "thread_sharded", False):
            try:
                scores = many([[c["_id"] for c in chunks[t] if c.get("embedding_generated")] for t in thread_ids])
            except (RuntimeError, ValueError, OSError) as e:
                self.log.warning("vector scoring failed; neutral scores", threads=len(thread_ids), error=repr(e))
                scores = [{} for _ in thread_ids]
        elif self.vectors is not None:
            return {t: self.candidates(t) for t in thread_ids}
        return {t: self._scored(chunks[t], sc) for t, sc in zip(thread_ids, scores)}

    def candidates(self, thread_id: str) -> list[dict]:
        """The thread's chunks scored by cosine to the thread's centroid, in ONE search restricted to
        the thread's own rows (HipFlatIndex: a device gather + GEMV; reference context_sources.py
        queries the whole collection, keeps the global top-k and filters it to the thread, which
        can drop the thread's own chunks).  Every chunk is on one scale: without a vector store
        (or none of the thread's vectors stored) all get the reference's neutral 0.5; a chunk whose
        vector is missing while others have one ranks last (0.0)."""
        chunks = self.store.query_documents("chunks", {"thread_id": thread_id}, limit=1 << 20)
        scores: dict[str, float] = {}
        if self.vectors is not None and chunks:
            try:
                ids = [c["_id"] for c in chunks if c.get("embedding_generated")]
                # a thread-sharded (DP) store answers from the shard that owns the thread
                scores = (self.vectors.centroid_scores(ids, thread_id=thread_id)
                          if getattr(self.vectors, "thread_sharded", False) else self.vectors.centroid_scores(ids))
            except (RuntimeError, ValueError, OSError) as e:
                self.log.warning("vector scoring failed; neutral scores", thread_id=thread_id, error=repr(e))
                scores = {}
        return self._scored(chunks, scores)

    def orchestrate_threads(self, thread_ids: list[str]) -> list[dict | None]:
        """orchestrate_thread over many threads, their candidates scored in one vector-store pass
        (the in-process batch driver, pipeline/rag.py, calls this once per batch)."""
        cands = self.candidates_many(list(thread_ids))
        return [self._request(t, cands[t]) for t in thread_ids]

    def orchestrate_thread(self, thread_id: str) -> dict | None:
        return self._request(thread_id, self.candidates(thread_id))

    def _request(self, thread_id: str, cands: list[dict]) -> dict | None:
        if not cands or not all(c.get("embedding_generated") for c in cands):
            return None  # wait until every chunk of the thread is embedded
        sel = self.selector.select(thread_id, cands, self.top_k, self.budget)
        sid = cids.summary_id(thread_id, [s.chunk_id for s in sel.selected_chunks])
        rid = cids.report_id(sid)
        if self.store.get_document("summaries", rid) is not None:
            thread = self.store.get_document("threads", thread_id)
            if thread and not thread.get("summary_id"):
                self.store.update_document("threads", thread_id, {"summary_id": rid})  # backfill
            self.metrics.increment("orchestrator_summary_skipped_total")
            return None
        self.metrics.increment("orchestrator_summary_triggered_total")
        if self.consensus is not None:
            self._annotate_consensus(thread_id)
        return self.publish("SummarizationRequested", thread_ids=[thread_id], top_k=self.top_k,
                            prompt_template=self.template,
                            selected_chunks=[s.to_dict() for s in sel.selected_chunks],
                            context_selection=sel.metadata())

    def _annotate_consensus(self, thread_id: str) -> None:
        from ..consensus import ConsensusLevel, Thread
        thread = self.store.get_document("threads", thread_id)
        if thread is None:
            return
        msgs = self.store.query_documents("messages", {"thread_id": thread_id}, limit=1 << 20)
        sig = self.consensus.detect(Thread.from_documents(thread, msgs))
        agreed = sig.level in (ConsensusLevel.STRONG_CONSENSUS, ConsensusLevel.CONSENSUS)
        self.store.update_document("threads", thread_id, {"has_consensus": agreed, "consensus_type": sig.level.value})
        self.metrics.increment("orchestrator_consensus_total", tags={"level": sig.level.value})

    def process_embeddings(self, chunk_ids: list[str]) -> int:
        return sum(ev is not None for ev in self.orchestrate_threads(self._resolve_threads(chunk_ids)))

    def on_failure(self, event_type, event, error):
        if event_type == "EmbeddingsGenerated":
            try:
                tids = self._resolve_threads(event["data"]["chunk_ids"])
            except Exception as e:  # noqa: BLE001 -- the store failing too: logged below, nothing to name
                self.log.warning("could not resolve the failed event's threads", error=repr(e))
                tids = []
            if not tids:  # chunks never became visible: nothing to name (the event needs >= 1 thread)
                self.log.error("orchestration failed before threads resolved", error=repr(error))
                return
            ctx = getattr(error, "context", None)
            self.publish("OrchestrationFailed", thread_ids=tids, error_type=type(error).__name__,
                         error_message=str(error) or type(error).__name__,
                         retry_count=max(0, int(getattr(ctx, "attempt_number", 1)) - 1) if ctx is not None else 0)

    def requeue_incomplete(self):
        n = 0
        for t in self.store.query_documents("threads", {"summary_id": None}, limit=1 << 30):
            if self.orchestrate_thread(t["_id"]) is not None:
                n += 1
        return n


class SummarizationService(BaseService):
    name = "summarization"

    def __init__(self, publisher, subscriber, document_store, summarizer: Summarizer, citation_count: int = 12,
                 context_window_tokens: int = 4096, max_batch_threads: int = 128, batch_wait_ms: int = 50,
                 max_retries: int = 3, retry_delay_seconds: float = 5.0, continuous: bool = True,
                 min_admit: int = 1, admit_wait_ms: int = 50, **kw):
        super().__init__(publisher, subscriber, document_store, **kw)
        self.summarizer = summarizer
        # continuous batching (a summarizer with start_continuous, e.g. the HIP engine): requests go
        # straight into the running decode batch; otherwise micro-batches of <= max_batch_threads
        self.continuous = continuous
        self.min_admit, self.admit_wait = int(min_admit), admit_wait_ms / 1000.0
        self._streaming = False
        self.citation_count, self.ctx_tokens = citation_count, context_window_tokens
        self.max_batch, self.batch_wait = max_batch_threads, batch_wait_ms / 1000.0
        self.max_retries, self.retry_delay = max_retries, retry_delay_seconds
        self._queue: list[dict] = []
        self._qlock = threading.Condition()
        self._worker: threading.Thread | None = None
        self._stop = False
        # requests in the engine, by (thread, selected chunks): the orchestrator can request one
        # thread twice when its chunks arrive in two EmbeddingsGenerated events that both find every
        # chunk embedded; the copy is dropped instead of decoded a second time
        self._inflight: set = set()
        self._flight_lock = threading.Lock()

    def subscriptions(self):
        return {"SummarizationRequested": self._on_request}

    @staticmethod
    def _request_key(event: dict) -> tuple:
        d = event["data"]
        return (d["thread_ids"][0], tuple(s.get("chunk_id") for s in d.get("selected_chunks") or []))

    def _claim(self, event: dict) -> bool:
        """True when this request is not already in flight (and marks it so)."""
        key = self._request_key(event)
        with self._flight_lock:
            if key in self._inflight:
                self.metrics.increment("summarization_duplicate_skipped_total")
                self.log.info("duplicate summarization request skipped", thread_id=key[0])
                return False
            self._inflight.add(key)
            return True

    def _release(self, event: dict) -> None:
        with self._flight_lock:
            self._inflight.discard(self._request_key(event))

    def _context(self, thread_id: str, selected: list[dict]) -> dict:
        ids = [s["chunk_id"] for s in selected]
        chunks = self.store.query_documents("chunks", {"_id": {"$in": ids}}, limit=len(ids))
        if not chunks:
            raise DocumentNotFoundError(f"selected chunks of {thread_id} not visible")
        by = {c["_id"]: c for c in chunks}
        ordered = [by[i] for i in ids if i in by]
        msgs = {m["_id"]: m for m in self.store.query_documents(
            "messages", {"_id": {"$in": sorted({c["message_doc_id"] for c in ordered})}}, limit=len(ordered))}
        return build_context(ordered, msgs)

    def prepare(self, event: dict) -> tuple[str, dict, str]:
        d = event["data"]
        tid = d["thread_ids"][0]
        selected = d.get("selected_chunks") or [{"chunk_id": c["_id"]} for c in self.store.query_documents(
            "chunks", {"thread_id": tid}, limit=d.get("top_k", 12))]
        ctx = self._context(tid, selected)
        return tid, ctx, substitute_prompt(d["prompt_template"], tid, ctx)

    def summarize_events(self, events: list[dict]) -> list[dict]:
        """Batch path: one engine call for all requested threads (in-flight duplicates dropped)."""
        events = [ev for ev in events if self._claim(ev)]
        try:
            return self._summarize_claimed(events)
        finally:
            for ev in events:
                self._release(ev)

    def _summarize_claimed(self, events: list[dict]) -> list[dict]:
        prepared = []
        for ev in events:
            try:
                prepared.append(self.prepare(ev))
            except Exception as e:  # per-thread failure isolation
                self.publish("SummarizationFailed", thread_id=ev["data"]["thread_ids"][0],
                             error_type=type(e).__name__, error_message=str(e) or type(e).__name__, retry_count=0)
        if not prepared:
            return []
        threads = [SumThread(tid, ctx["messages"], len(ctx["chunks"]), self.ctx_tokens, prompt)
                   for tid, ctx, prompt in prepared]
        t0 = time.perf_counter()
        summaries = retry_with_backoff(lambda: self.summarizer.summarize_batch(threads), self.max_retries,
                                       self.retry_delay)
        self.metrics.observe("summarization_latency_seconds", time.perf_counter() - t0)
        for k, v in (getattr(self.summarizer, "last_stats", None) or {}).items():
            self.metrics.gauge(f"summarization_gpu_{k}", float(v))
        return [self._publish_summary(tid, ctx, s) for (tid, ctx, _), s in zip(prepared, summaries)]

    def publish_summary(self, tid: str, ctx: dict, s) -> dict:
        """SummaryComplete for one summarized thread (citations from its context); returns the event."""
        return self._publish_summary(tid, ctx, s)

    def _publish_summary(self, tid: str, ctx: dict, s) -> dict:
        cites = format_citations(ctx["chunks"], self.citation_count)
        sid = cids.summary_id(tid, [c["chunk_id"] for c in cites])
        self.metrics.increment("summarization_tokens_total", s.tokens_prompt, tags={"type": "prompt"})
        self.metrics.increment("summarization_tokens_total", s.tokens_completion, tags={"type": "completion"})
        return self.publish("SummaryComplete", summary_id=sid, thread_id=tid,
                            summary_markdown=s.summary_markdown or "(empty summary)", citations=cites,
                            llm_backend=s.llm_backend, llm_model=s.llm_model, tokens_prompt=s.tokens_prompt,
                            tokens_completion=s.tokens_completion, latency_ms=int(s.latency_ms))

    # continuous batching (start_async with a streaming summarizer): each request is prepared and
    # submitted at once; the engine thread publishes its summary when its sequence finishes.
    # micro-batching otherwise: requests accumulate for up to batch_wait_ms (or max_batch) before
    # one engine call
    def _on_request(self, event):
        if self._streaming:
            if not self._claim(event):
                return
            try:
                tid, ctx, prompt = self.prepare(event)     # store not ready -> raises -> the retry policy
            except BaseException:
                self._release(event)
                raise
            t0 = time.perf_counter()

            def done(s, err, tid=tid, ctx=ctx, event=event):
                try:
                    if err is not None:
                        self.log.error("summarization failed", thread_id=tid, error=repr(err))
                        self.on_failure("SummarizationRequested", event, err)
                        return
                    self.metrics.observe("summarization_latency_seconds", time.perf_counter() - t0)
                    self._publish_summary(tid, ctx, s)
                finally:
                    self._release(event)    # after the SummaryComplete is out
            try:
                self.summarizer.submit(SumThread(tid, ctx["messages"], len(ctx["chunks"]), self.ctx_tokens, prompt),
                                       done)
            except BaseException:
                self._release(event)
                raise
            return
        if self._worker is None:
            self.summarize_events([event])
            return
        with self._qlock:
            self._queue.append(event)
            self._qlock.notify()

    def start_batching(self) -> None:
        def loop():
            while not self._stop:
                with self._qlock:
                    if not self._queue:
                        self._qlock.wait(0.1)
                        continue
                    deadline = time.time() + self.batch_wait
                    while len(self._queue) < self.max_batch and time.time() < deadline:
                        self._qlock.wait(max(0.0, deadline - time.time()))
                    batch, self._queue = self._queue[:self.max_batch], self._queue[self.max_batch:]
                try:
                    self.summarize_events(batch)
                except Exception as e:  # engine failure after retries: every thread of the batch fails
                    self.log.error("summarization batch failed", error=repr(e))
                    for ev in batch:
                        self.on_failure("SummarizationRequested", ev, e)
        self._worker = threading.Thread(target=loop, name="summarization-batcher", daemon=True)
        self._worker.start()

    def stop_batching(self) -> None:
        self._stop = True

    def start_async(self) -> None:
        """Background engine for a consuming service: continuous batching when the summarizer
        streams, else the micro-batcher (when batches are allowed)."""
        start = getattr(self.summarizer, "start_continuous", None)
        if self.continuous and callable(start):
            start(min_admit=self.min_admit, max_wait_s=self.admit_wait)
            self._streaming = True
        elif self.max_batch > 1:
            self.start_batching()

    def stop_async(self) -> None:
        if self._streaming:
            self.summarizer.stop_continuous()
            self._streaming = False
        self.stop_batching()

    def on_failure(self, event_type, event, error):
        if event_type == "SummarizationRequested":
            self.publish("SummarizationFailed", thread_id=event["data"]["thread_ids"][0],
                         error_type=type(error).__name__, error_message=str(error) or type(error).__name__,
                         retry_count=self.max_retries)


__all__ = ["ParsingService", "ChunkingService", "EmbeddingService", "OrchestratorService", "SummarizationService",
           "TopKRelevanceSelector", "DocumentAlreadyExistsError"]
