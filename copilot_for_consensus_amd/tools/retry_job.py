"""Periodic job that re-drives documents stuck in the pipeline.

Parity target: scripts/retry_stuck_documents.py of the reference (RetryStuckDocumentsJob :143,
COLLECTION_CONFIGS :147-172, exponential backoff base*2^(n-1) capped, stuck threshold,
``failed_max_retries`` marking, Prometheus gauges/counters pushed per run, loop interval 900 s in
compose).  Differences:
  * works against any DocumentStore / EventPublisher (in-proc node, Mongo + RabbitMQ);
  * the republished events are schema-valid and batched (the reference emits e.g. ``JSONParsed``
    with a ``parsed_message_ids`` field its own schema rejects, one event per document);
  * "stuck" is defined per collection on this framework's document model: archives by status,
    messages without chunks, chunks not embedded, threads with embedded chunks but no summary.

Reference: scripts/retry_stuck_documents.py:143 (COLLECTION_CONFIGS :147-172, failed_max_retries
terminal state :355).
"""
from __future__ import annotations

import argparse
import dataclasses
import sys
import time
from datetime import datetime, timedelta, timezone
from typing import Any, Callable

from ..contracts.events import Event, utc_now_iso

EXCHANGE = "copilot.events"


def _parse_ts(v) -> datetime | None:
    if v is None or v == "":
        return None
    if isinstance(v, datetime):
        return v if v.tzinfo else v.replace(tzinfo=timezone.utc)
    try:
        t = datetime.fromisoformat(str(v).replace("Z", "+00:00"))
        return t if t.tzinfo else t.replace(tzinfo=timezone.utc)
    except ValueError:
        return None


@dataclasses.dataclass
class CollectionPolicy:
    max_attempts: int
    event_type: str
    batch: int
    find: Callable[[Any], list[dict]]                 # store -> candidate documents
    build: Callable[[Any, list[dict]], dict]          # (store, docs) -> event data


def _archives(store):
    return store.query_documents("archives", {"status": {"$in": ["pending", "processing"]}}, limit=1 << 30)


def _archive_event(store, docs):
    a = docs[0]
    return dict(archive_id=a["_id"], source_name=a.get("source") or "unknown", source_type=a.get("source_type") or "local",
                source_url=a.get("source_url") or a.get("file_path") or "retry",
                file_size_bytes=int(a.get("file_size_bytes", 0)), file_hash_sha256=a.get("file_hash") or "-",
                ingestion_started_at=a.get("ingestion_date") or utc_now_iso(), ingestion_completed_at=utc_now_iso())


def _unchunked_messages(store):
    chunked = {c["message_doc_id"] for c in store.query_documents("chunks", {}, limit=1 << 30)}
    return [m for m in store.query_documents("messages", {}, limit=1 << 30) if m["_id"] not in chunked]


def _parsed_event(store, docs):
    return dict(archive_id=docs[0].get("archive_id", "retry"), message_count=len(docs),
                message_doc_ids=[m["_id"] for m in docs], thread_count=len({m.get("thread_id") for m in docs}),
                thread_ids=sorted({m["thread_id"] for m in docs if m.get("thread_id")}), parsing_duration_seconds=0.0)


def _unembedded_chunks(store):
    return store.query_documents("chunks", {"embedding_generated": False}, limit=1 << 30)


def _chunks_event(store, docs):
    return dict(message_doc_ids=sorted({c["message_doc_id"] for c in docs}), chunk_count=len(docs),
                chunk_ids=[c["_id"] for c in docs], chunks_ready=True, chunking_strategy="retry",
                avg_chunk_size_tokens=0)


def _unsummarized_threads(store):
    out = []
    for t in store.query_documents("threads", {}, limit=1 << 30):
        if t.get("summary_id"):
            continue
        chunks = store.query_documents("chunks", {"thread_id": t["_id"]}, limit=1 << 20)
        if chunks and all(c.get("embedding_generated") for c in chunks):
            t = dict(t)
            t["_chunk_ids"] = [c["_id"] for c in chunks]
            out.append(t)
    return out


def _embedded_event(store, docs):
    ids = [cid for t in docs for cid in t.get("_chunk_ids", [])]
    return dict(chunk_ids=ids, embedding_count=len(ids), embedding_model="retry", embedding_backend="retry",
                embedding_dimension=1, vector_store_collection="retry", vector_store_updated=True,
                avg_generation_time_ms=0.0)


COLLECTION_POLICIES: dict[str, CollectionPolicy] = {
    "archives": CollectionPolicy(3, "ArchiveIngested", 1, _archives, _archive_event),
    "messages": CollectionPolicy(3, "JSONParsed", 100, _unchunked_messages, _parsed_event),
    "chunks": CollectionPolicy(5, "ChunksPrepared", 512, _unembedded_chunks, _chunks_event),
    "threads": CollectionPolicy(5, "EmbeddingsGenerated", 64, _unsummarized_threads, _embedded_event),
}


class RetryStuckDocumentsJob:
    def __init__(self, store, publisher, metrics=None, base_delay_seconds: int = 300, max_delay_seconds: int = 3600,
                 stuck_threshold_hours: float = 24, policies: dict[str, CollectionPolicy] | None = None,
                 clock: Callable[[], datetime] | None = None):
        self.store, self.publisher, self.metrics = store, publisher, metrics
        self.base_delay, self.max_delay = base_delay_seconds, max_delay_seconds
        self.stuck_threshold = timedelta(hours=stuck_threshold_hours)
        self.policies = policies or COLLECTION_POLICIES
        self.now = clock or (lambda: datetime.now(timezone.utc))

    def backoff_seconds(self, attempts: int) -> float:
        return 0 if attempts <= 0 else min(self.base_delay * 2 ** (attempts - 1), self.max_delay)

    def eligible(self, doc: dict) -> bool:
        last = _parse_ts(doc.get("lastAttemptTime"))
        if last is None:
            return True
        now = self.now()
        return now - last >= self.stuck_threshold or now >= last + timedelta(seconds=self.backoff_seconds(
            int(doc.get("attemptCount", 0))))

    def _metric(self, kind, name, value, **tags):
        if self.metrics is not None:
            getattr(self.metrics, kind)(name, value, tags=tags)

    def process_collection(self, name: str, pol: CollectionPolicy) -> dict:
        docs = pol.find(self.store)
        stats = {"stuck": len(docs), "requeued": 0, "skipped_backoff": 0, "max_retries_exceeded": 0, "errors": 0}
        ready = []
        for d in docs:
            n = int(d.get("attemptCount", 0))
            if n >= pol.max_attempts:
                if d.get("status") != "failed_max_retries":
                    self.store.update_document(name, d["_id"], {"status": "failed_max_retries",
                                                                "lastAttemptTime": self.now().isoformat()})
                    stats["max_retries_exceeded"] += 1
                continue
            if not self.eligible(d):
                stats["skipped_backoff"] += 1
                continue
            ready.append(d)
        for s in range(0, len(ready), pol.batch):
            grp = ready[s:s + pol.batch]
            try:
                ev = Event.create(pol.event_type, **pol.build(self.store, grp))
                self.publisher.publish(EXCHANGE, ev.routing_key, ev.to_dict())
            except Exception:
                stats["errors"] += 1
                continue
            ts = self.now().isoformat()
            for d in grp:
                self.store.update_document(name, d["_id"], {"$inc": {"attemptCount": 1},
                                                            "$set": {"lastAttemptTime": ts}})
            stats["requeued"] += len(grp)
        self._metric("gauge", "retry_job_stuck_documents", stats["stuck"], collection=name)
        self._metric("increment", "retry_job_documents_requeued_total", stats["requeued"], collection=name)
        self._metric("increment", "retry_job_documents_skipped_backoff_total", stats["skipped_backoff"],
                     collection=name)
        self._metric("increment", "retry_job_documents_max_retries_exceeded_total", stats["max_retries_exceeded"],
                     collection=name)
        failed = self.store.count_documents(name, {"status": "failed_max_retries"})
        self._metric("gauge", "retry_job_failed_documents", failed, collection=name)
        return stats

    def run_once(self) -> dict[str, dict]:
        t = time.perf_counter()
        out = {name: self.process_collection(name, pol) for name, pol in self.policies.items()}
        self._metric("observe", "retry_job_duration_seconds", time.perf_counter() - t)
        if self.metrics is not None and hasattr(self.metrics, "safe_push"):
            self.metrics.safe_push()
        return out


def main(argv=None) -> int:
    from ..bus import create_publisher
    from ..config.loader import load_adapter_config
    from ..observability import create_metrics_collector
    from ..storage.document_store import create_document_store
    ap = argparse.ArgumentParser(description="Re-drive stuck documents (see module docstring)")
    ap.add_argument("--once", action="store_true")
    ap.add_argument("--interval", type=int, default=900)
    ap.add_argument("--base-delay", type=int, default=300)
    ap.add_argument("--max-delay", type=int, default=3600)
    ap.add_argument("--stuck-hours", type=float, default=24)
    a = ap.parse_args(argv)
    store = create_document_store(load_adapter_config("document_store"))
    job = RetryStuckDocumentsJob(store, create_publisher(load_adapter_config("message_bus")),
                                 create_metrics_collector(load_adapter_config("metrics")), a.base_delay, a.max_delay,
                                 a.stuck_hours)
    while True:
        res = job.run_once()
        print(res, file=sys.stderr, flush=True)
        if a.once:
            return 0
        time.sleep(a.interval)


if __name__ == "__main__":
    sys.exit(main())
