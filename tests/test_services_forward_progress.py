"""Per-service behaviour with in-memory adapters and a recording publisher -- the reference's
{svc}/tests/test_service.py, test_forward_progress.py and test_integration.py: failure events,
retry on not-yet-visible documents, idempotent replays, startup requeue, summary skip/backfill,
webhook delivery, and that every event a service emits is schema-valid."""
from __future__ import annotations

import http.server
import os
import threading

import pytest

from copilot_for_consensus_amd.archive import InMemoryArchiveStore
from copilot_for_consensus_amd.bus import NoopPublisher, NoopSubscriber, ValidatingEventPublisher
from copilot_for_consensus_amd.chunking import TokenWindowChunker
from copilot_for_consensus_amd.contracts import ids
from copilot_for_consensus_amd.contracts.events import Event
from copilot_for_consensus_amd.embedding import MockEmbeddingProvider
from copilot_for_consensus_amd.parsing import MessageParser, ThreadBuilder
from copilot_for_consensus_amd.retry import RetryConfig
from copilot_for_consensus_amd.services.processing import (ChunkingService, EmbeddingService, OrchestratorService,
                                                           ParsingService, SummarizationService)
from copilot_for_consensus_amd.services.reporting import ReportingService
from copilot_for_consensus_amd.storage.document_store import InMemoryDocumentStore
from copilot_for_consensus_amd.summarization import MockSummarizer
from copilot_for_consensus_amd.vectorstore import InMemoryVectorStore

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "sample.mbox")
FAST = RetryConfig(max_attempts=3, base_delay_ms=0, use_jitter=False)


def _pub():
    # validating decorator over a recorder: a schema-invalid event fails the test where it is emitted
    rec = NoopPublisher()
    return ValidatingEventPublisher(rec), rec


def _wire(svc):
    sub = NoopSubscriber()
    svc.subscriber = sub
    svc.start()
    return sub


def _archive(store, archives, data=None):
    data = data or open(FIX, "rb").read()
    aid = archives.store_archive("wg", "list.mbox", data)
    store.insert_document("archives", {"_id": aid, "file_hash": ids.sha256_16(aid) * 4, "file_size_bytes": len(data),
                                       "source": "wg", "ingestion_date": "2025-01-01T00:00:00Z", "status": "pending"})
    return aid


def _archive_event(aid):
    return Event("ArchiveIngested", {"archive_id": aid, "source_name": "wg", "source_type": "local",
                                     "source_url": "/x", "file_size_bytes": 1, "file_hash_sha256": "h",
                                     "ingestion_started_at": "2025-01-01T00:00:00Z",
                                     "ingestion_completed_at": "2025-01-01T00:00:00Z"}).to_dict()


# ------------------------------------------------------------------ parsing
def test_parsing_happy_path_and_per_message_events():
    store, archives = InMemoryDocumentStore(), InMemoryArchiveStore()
    pub, rec = _pub()
    svc = ParsingService(pub, None, store, archives, retry_config=FAST)
    sub = _wire(svc)
    aid = _archive(store, archives)
    sub.inject_event(_archive_event(aid))
    assert store.get_document("archives", aid)["status"] == "completed"
    assert store.count_documents("messages") == 10 and store.count_documents("threads") == 2
    parsed = rec.get_events("JSONParsed")
    assert len(parsed) == 10 and all(len(e["data"]["message_doc_ids"]) == 1 for e in parsed)
    # replay: idempotent (duplicate inserts tolerated, same ids)
    sub.inject_event(_archive_event(aid))
    assert store.count_documents("messages") == 10


def test_parsing_missing_archive_retries_then_fails():
    store, archives = InMemoryDocumentStore(), InMemoryArchiveStore()
    pub, rec = _pub()
    svc = ParsingService(pub, None, store, archives, retry_config=FAST)
    sub = _wire(svc)
    store.insert_document("archives", {"_id": "0123456789abcdef", "status": "pending", "source": "wg"})
    sub.inject_event(_archive_event("0123456789abcdef"))
    failed = rec.get_events("ParsingFailed")
    # the event names the root cause and how many retries ran (not the wrapper / zero)
    assert len(failed) == 1 and failed[0]["data"]["error_type"] == "DocumentNotFoundError"
    assert failed[0]["data"]["retry_count"] == FAST.max_attempts - 1
    assert failed[0]["data"]["messages_parsed_before_failure"] == 0
    assert store.get_document("archives", "0123456789abcdef")["status"] == "failed"
    assert svc.get_stats()["events_failed"] == 1


def test_parsing_failure_after_parse_reports_progress_and_logs_status_errors():
    """A store that fails inserting messages: ParsingFailed carries the messages parsed before the
    failure; a failing archive-status update is logged and counted, not silently dropped."""
    from copilot_for_consensus_amd.observability import PrometheusMetricsCollector

    class FlakyStore(InMemoryDocumentStore):
        def insert_many(self, coll, docs):
            raise ConnectionError("store down")

        def update_document(self, coll, doc_id, fields):
            if coll == "archives":
                raise ConnectionError("store down")
            return super().update_document(coll, doc_id, fields)

    store, archives = FlakyStore(), InMemoryArchiveStore()
    aid = _archive(store, archives)
    pub, rec = _pub()
    metrics = PrometheusMetricsCollector()
    svc = ParsingService(pub, None, store, archives, retry_config=FAST, metrics=metrics)
    sub = _wire(svc)
    with pytest.raises(ConnectionError):      # not a transient error class: fails at once, re-raised
        sub.inject_event(_archive_event(aid))
    failed = rec.get_events("ParsingFailed")
    assert len(failed) == 1 and failed[0]["data"]["error_type"] == "ConnectionError"
    assert failed[0]["data"]["messages_parsed_before_failure"] > 0
    assert metrics.get_counter("parsing_archive_status_update_failures_total", {"status": "processing"}) >= 1


def test_parsing_startup_requeue_of_pending_archives():
    store, archives = InMemoryDocumentStore(), InMemoryArchiveStore()
    aid = _archive(store, archives)
    pub, rec = _pub()
    svc = ParsingService(pub, None, store, archives)
    svc.start()
    ev = rec.get_events("ArchiveIngested")
    assert [e["data"]["archive_id"] for e in ev] == [aid] and svc.is_ready()


# ------------------------------------------------------------------ chunking
def _parsed(store):
    msgs, _ = MessageParser().parse_mbox_bytes(open(FIX, "rb").read(), "0123456789abcdef")
    threads = ThreadBuilder().build_threads(msgs)
    store.insert_many("messages", msgs)
    store.insert_many("threads", threads)
    return msgs, threads


def test_chunking_idempotent_and_waits_for_messages():
    store = InMemoryDocumentStore()
    pub, rec = _pub()
    svc = ChunkingService(pub, None, store, TokenWindowChunker(chunk_size=64, overlap=8, min_chunk_size=8),
                          retry_config=FAST)
    msgs, _ = _parsed(store)
    first = svc.process_messages([msgs[0]["_id"]])
    again = svc.process_messages([msgs[0]["_id"]])
    assert first == again and store.count_documents("chunks", {"message_doc_id": msgs[0]["_id"]}) == len(first)
    assert [c["chunk_index"] for c in store.query_documents("chunks", {"message_doc_id": msgs[0]["_id"]},
                                                           sort_by="chunk_index", sort_order="asc")] == \
        list(range(len(first)))
    sub = _wire(svc)
    sub.inject_event(Event("JSONParsed", {"archive_id": "0123456789abcdef", "message_count": 1,
                                          "message_doc_ids": ["feedfacefeedface"], "thread_count": 0,
                                          "thread_ids": [], "parsing_duration_seconds": 0.0}).to_dict())
    assert rec.get_events("ChunkingFailed")[0]["data"]["message_doc_ids"] == ["feedfacefeedface"]


def test_chunking_empty_body_emits_no_invalid_event():
    store = InMemoryDocumentStore()
    pub, rec = _pub()
    svc = ChunkingService(pub, None, store)
    store.insert_document("messages", {"_id": "aaaaaaaaaaaaaaaa", "message_id": "m", "thread_id": "aaaaaaaaaaaaaaaa",
                                       "archive_id": "0123456789abcdef", "body_normalized": "   "})
    assert svc.process_messages(["aaaaaaaaaaaaaaaa"]) == []
    assert rec.get_events("ChunksPrepared") == []


def test_chunking_requeue_messages_without_chunks():
    store = InMemoryDocumentStore()
    msgs, _ = _parsed(store)
    pub, rec = _pub()
    svc = ChunkingService(pub, None, store)
    assert svc.requeue_incomplete() == 10
    assert sum(len(e["data"]["message_doc_ids"]) for e in rec.get_events("JSONParsed")) == 10


# ------------------------------------------------------------------ embedding
def _chunked(store):
    msgs, threads = _parsed(store)
    ChunkingService(NoopPublisher(), None, store).process_messages([m["_id"] for m in msgs])
    return msgs, threads


def test_embedding_marks_chunks_and_is_idempotent():
    store = InMemoryDocumentStore()
    _chunked(store)
    vs = InMemoryVectorStore()
    pub, rec = _pub()
    svc = EmbeddingService(pub, None, store, MockEmbeddingProvider(dimension=16), vs, retry_backoff_seconds=0)
    cids = [c["_id"] for c in store.query_documents("chunks", {}, limit=None)]
    assert svc.process_chunks(cids) == len(cids)
    assert store.count_documents("chunks", {"embedding_generated": False}) == 0
    assert len(vs) == len(cids)
    assert svc.process_chunks(cids) == 0  # replay: nothing to do
    ev = rec.get_events("EmbeddingsGenerated")
    assert len(ev) == 1 and ev[0]["data"]["embedding_dimension"] == 16


def test_embedding_failure_event_after_provider_errors():
    store = InMemoryDocumentStore()
    _chunked(store)

    class Broken(MockEmbeddingProvider):
        def embed_tensor(self, texts):
            raise RuntimeError("device lost")

    pub, rec = _pub()
    svc = EmbeddingService(pub, None, store, Broken(dimension=16), InMemoryVectorStore(), max_retries=2,
                           retry_backoff_seconds=0, retry_config=FAST)
    sub = _wire(svc)
    cid = store.query_documents("chunks", {}, limit=1)[0]["_id"]
    with pytest.raises(RuntimeError):
        sub.inject_event(Event("ChunksPrepared", {"message_doc_ids": ["0123456789abcdef"], "chunk_count": 1,
                                                  "chunk_ids": [cid], "chunks_ready": True,
                                                  "chunking_strategy": "token_window",
                                                  "avg_chunk_size_tokens": 1}).to_dict())
    f = rec.get_events("EmbeddingGenerationFailed")
    assert f and f[0]["data"]["error_type"] == "RuntimeError" and f[0]["data"]["chunk_ids"] == [cid]


# ------------------------------------------------------------------ orchestrator + summarization + reporting
def _embedded(store):
    msgs, threads = _chunked(store)
    vs = InMemoryVectorStore()
    EmbeddingService(NoopPublisher(), None, store, MockEmbeddingProvider(dimension=16), vs).process_chunks(
        [c["_id"] for c in store.query_documents("chunks", {}, limit=None)])
    return msgs, threads, vs


def test_orchestrator_requests_once_then_skips_and_backfills():
    store = InMemoryDocumentStore()
    _, threads, vs = _embedded(store)
    pub, rec = _pub()
    orch = OrchestratorService(pub, None, store, vs, top_k=3, context_window_tokens=100000)
    tid = threads[0]["_id"]
    req = orch.orchestrate_thread(tid)
    sel = req["data"]["selected_chunks"]
    assert len(sel) == 3 and [s["rank"] for s in sel] == [0, 1, 2]
    # run the rest of the pipeline for that thread
    spub, srec = _pub()
    summ = SummarizationService(spub, None, store, MockSummarizer(mock_latency_ms=0))
    done = summ.summarize_events([req])[0]
    cites = done["data"]["citations"]
    assert done["data"]["summary_id"] == ids.summary_id(tid, [c["chunk_id"] for c in cites])
    rpub, rrec = _pub()
    ReportingService(rpub, None, store).process_summary(done["data"], done)
    rid = ids.report_id(done["data"]["summary_id"])
    assert store.get_document("threads", tid)["summary_id"] == rid
    # a summary whose id matches the selection already exists -> skipped; a lost backfill is repaired
    store.update_document("threads", tid, {"summary_id": None})
    assert orch.orchestrate_thread(tid) is None
    assert store.get_document("threads", tid)["summary_id"] == rid
    # startup requeue only picks threads without a summary
    n = orch.requeue_incomplete()
    assert n == len(threads) - 1


def test_orchestrator_waits_for_all_chunks_embedded():
    store = InMemoryDocumentStore()
    _, threads, vs = _embedded(store)
    tid = threads[0]["_id"]
    one = store.query_documents("chunks", {"thread_id": tid}, limit=1)[0]
    store.update_document("chunks", one["_id"], {"embedding_generated": False})
    pub, rec = _pub()
    assert OrchestratorService(pub, None, store, vs).orchestrate_thread(tid) is None
    assert rec.get_events() == []


def test_summarizer_failure_is_reported_per_thread():
    store = InMemoryDocumentStore()
    _, threads, vs = _embedded(store)
    opub, orec = _pub()
    orch = OrchestratorService(opub, None, store, vs)
    reqs = [orch.orchestrate_thread(t["_id"]) for t in threads]

    class Down(MockSummarizer):
        def summarize_batch(self, threads):
            raise ConnectionError("engine down")

    pub, rec = _pub()
    svc = SummarizationService(pub, None, store, Down(mock_latency_ms=0), max_retries=1, retry_delay_seconds=0)
    svc.start_batching()
    try:
        for r in reqs:
            svc._on_request(r)
        import time
        deadline = time.time() + 10
        while time.time() < deadline and len(rec.get_events("SummarizationFailed")) < len(reqs):
            time.sleep(0.02)
    finally:
        svc.stop_batching()
    failed = rec.get_events("SummarizationFailed")
    assert sorted(e["data"]["thread_id"] for e in failed) == sorted(t["_id"] for t in threads)


def test_reporting_idempotent_and_webhook():
    store = InMemoryDocumentStore()
    _, threads, vs = _embedded(store)
    req = OrchestratorService(NoopPublisher(), None, store, vs).orchestrate_thread(threads[0]["_id"])
    done = SummarizationService(NoopPublisher(), None, store, MockSummarizer(mock_latency_ms=0)).summarize_events(
        [req])[0]
    got = []

    class H(http.server.BaseHTTPRequestHandler):
        def do_POST(self):
            import json
            got.append(json.loads(self.rfile.read(int(self.headers["Content-Length"]))))
            self.send_response(200)
            self.end_headers()

        def log_message(self, *a):
            pass

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        pub, rec = _pub()
        rep = ReportingService(pub, None, store, notify_enabled=True,
                               notify_webhook_url=f"http://127.0.0.1:{srv.server_port}/hook",
                               webhook_summary_max_length=20)
        rid1 = rep.process_summary(done["data"], done)
        rid2 = rep.process_summary(done["data"], done)
    finally:
        srv.shutdown()
    assert rid1 == rid2 and store.count_documents("summaries") == 1
    assert got[0]["report_id"] == rid1 and len(got[0]["summary"]) <= 20
    pubd = rec.get_events("ReportPublished")
    assert pubd[0]["data"]["notified"] is True and pubd[0]["data"]["delivery_channels"] == ["webhook"]
    # unreachable webhook: ReportDeliveryFailed, report still published
    pub2, rec2 = _pub()
    ReportingService(pub2, None, store, notify_enabled=True, notify_webhook_url="http://127.0.0.1:9/x").process_summary(
        done["data"], done)
    assert rec2.get_events("ReportDeliveryFailed") and rec2.get_events("ReportPublished")


def test_reporting_waits_for_thread():
    pub, rec = _pub()
    svc = ReportingService(pub, None, InMemoryDocumentStore(), retry_config=FAST)
    sub = _wire(svc)
    ev = Event("SummaryComplete", {"summary_id": "ab" * 32, "thread_id": "0123456789abcdef", "summary_markdown": "x",
                                   "citations": [], "llm_backend": "mock", "llm_model": "m", "tokens_prompt": 1,
                                   "tokens_completion": 1, "latency_ms": 1}).to_dict()
    sub.inject_event(ev)  # thread never appears: retries exhausted, no report
    assert svc.get_stats()["events_failed"] == 1 and rec.get_events("ReportPublished") == []


def test_summarization_continuous_engine_publishes_each_thread():
    """start_async with the HIP summarizer (tiny decoder, CPU path): requests are submitted into a
    ContinuousEngine as they arrive and every thread's SummaryComplete is published from the
    engine thread; the texts equal the batch path's (greedy)."""
    import time

    from copilot_for_consensus_amd.summarization import HipLLMSummarizer, Thread
    store = InMemoryDocumentStore()
    _, threads, vs = _embedded(store)
    opub, _ = _pub()
    orch = OrchestratorService(opub, None, store, vs)
    reqs = [orch.orchestrate_thread(t["_id"]) for t in threads]
    llm = HipLLMSummarizer(model="tiny", device="cpu", max_new_tokens=12, kv_cache_tokens=16384, max_batch=4,
                           temperature=0.0)
    pub, rec = _pub()
    svc = SummarizationService(pub, None, store, llm, max_retries=1, retry_delay_seconds=0)
    svc.start_async()
    assert svc._streaming
    try:
        for r in reqs:
            svc._on_request(r)
        deadline = time.time() + 120
        while time.time() < deadline and len(rec.get_events("SummaryComplete")) < len(reqs):
            time.sleep(0.05)
    finally:
        svc.stop_async()
    done = rec.get_events("SummaryComplete")
    assert sorted(e["data"]["thread_id"] for e in done) == sorted(t["_id"] for t in threads)
    # same text as the one-shot batch path for the same prompts
    batch = SummarizationService(pub, None, store, llm)
    prepared = [batch.prepare(r) for r in reqs]
    want = llm.summarize_batch([Thread(tid, ctx["messages"], len(ctx["chunks"]), 4096, p) for tid, ctx, p in prepared])
    got = {e["data"]["thread_id"]: e["data"]["summary_markdown"] for e in done}
    assert [got[s.thread_id] for s in want] == [s.summary_markdown for s in want]


def test_duplicate_in_flight_summarization_request_is_dropped():
    """The orchestrator can request one thread twice (its chunks embedded in two events that both
    find every chunk done): while the first request is in the engine the copy is dropped; once it
    has completed, the same request is served again (the orchestrator's own "report exists" check
    is what stops re-requests after that)."""
    import threading as th

    store = InMemoryDocumentStore()
    _, threads, vs = _embedded(store)
    opub, _ = _pub()
    req = OrchestratorService(opub, None, store, vs).orchestrate_thread(threads[0]["_id"])
    gate = th.Event()
    submitted = []

    class Streaming(MockSummarizer):
        def start_continuous(self, **kw):
            pass

        def stop_continuous(self):
            pass

        def submit(self, thread, done):
            submitted.append(thread.thread_id)

            def run():
                gate.wait(10)
                done(self.summarize(thread), None)
            th.Thread(target=run, daemon=True).start()

    pub, rec = _pub()
    svc = SummarizationService(pub, None, store, Streaming(mock_latency_ms=0))
    svc.start_async()
    svc._on_request(req)
    svc._on_request(req)                   # in flight: dropped
    assert submitted == [threads[0]["_id"]]
    gate.set()
    import time
    deadline = time.time() + 10
    while time.time() < deadline and not rec.get_events("SummaryComplete"):
        time.sleep(0.01)
    while time.time() < deadline and svc._inflight:
        time.sleep(0.01)
    assert len(rec.get_events("SummaryComplete")) == 1
    svc._on_request(req)                   # completed: a new request is served
    assert len(submitted) == 2
    # batch path: copies inside one batch are summarised once
    batch = SummarizationService(pub, None, store, MockSummarizer(mock_latency_ms=0))
    assert len(batch.summarize_events([req, req])) == 1
