"""Reporting read/write semantics checked against the reference's documented behaviour
(reporting/app/service.py:192-451 write path, :532-755 get_reports, :970-1113 get_threads;
reporting/main.py:73-474 routes).  The fixtures are synthetic threads with hand-picked dates,
participant and message counts so every filter boundary is exercised."""
from __future__ import annotations

import threading

import pytest
from fastapi.testclient import TestClient

from copilot_for_consensus_amd.bus import NoopPublisher
from copilot_for_consensus_amd.retry import DocumentNotFoundError
from copilot_for_consensus_amd.services.base import create_app
from copilot_for_consensus_amd.services.reporting import ReportingService, reporting_routes
from copilot_for_consensus_amd.storage.document_store import InMemoryDocumentStore

THREADS = [  # id, first, last, participants, messages, archive
    ("t1", "2025-01-01T00:00:00Z", "2025-01-10T00:00:00Z", 2, 3, "a1"),
    ("t2", "2025-02-01T00:00:00Z", "2025-02-05T00:00:00Z", 5, 12, "a2"),
    ("t3", "2025-03-01T00:00:00Z", "2025-03-02T00:00:00Z", 1, 1, "a1"),
    ("t4", None, None, 3, 4, "a2"),                       # no dates
    ("t5", "2025-01-15T00:00:00Z", "2025-04-01T00:00:00Z", 4, 7, "gone"),   # archive missing
]


@pytest.fixture
def svc():
    store = InMemoryDocumentStore()
    store.insert_document("archives", {"_id": "a1", "source": "ietf-quic", "source_url": "rsync://x/quic"})
    store.insert_document("archives", {"_id": "a2", "source": "ietf-tls", "source_url": "rsync://x/tls"})
    for i, (tid, first, last, np_, nm, arch) in enumerate(THREADS):
        store.insert_document("threads", {"_id": tid, "thread_id": tid, "archive_id": arch, "subject": f"s{tid}",
                                          "participants": [f"p{j}@x" for j in range(np_)], "message_count": nm,
                                          "first_message_date": first, "last_message_date": last,
                                          "summary_id": None})
        store.insert_document("summaries", {"_id": f"r{tid}", "thread_id": tid, "content_markdown": f"# {tid}",
                                            "generated_at": f"2025-06-0{i + 1}T00:00:00Z"})
    pub = NoopPublisher()
    return ReportingService(pub, None, store), pub


def ids(docs):
    return [d["thread_id"] for d in docs]


def test_date_overlap_filters(svc):
    s, _ = svc
    # inclusive overlap with [Jan 5, Feb 1]: t1 (ends Jan 10), t2 (starts Feb 1, boundary), t5 (spans)
    got = s.get_reports(limit=100, message_start_date="2025-01-05T00:00:00Z", message_end_date="2025-02-01T00:00:00Z")
    assert sorted(ids(got)) == ["t1", "t2", "t5"]
    assert s.get_reports(limit=100, message_start_date="2026-01-01", message_end_date="2026-02-01") == []
    # start only / end only; t4 (no dates) is never returned once a date filter is present
    assert sorted(ids(s.get_reports(limit=100, message_start_date="2025-03-01T00:00:00Z"))) == ["t3", "t5"]
    assert sorted(ids(s.get_reports(limit=100, message_end_date="2025-01-31T00:00:00Z"))) == ["t1", "t5"]
    assert "t4" in ids(s.get_reports(limit=100))
    assert sorted(t["_id"] for t in s.get_threads(limit=100, message_end_date="2025-01-31T00:00:00Z")) == ["t1", "t5"]


def test_count_and_source_filters(svc):
    s, _ = svc
    assert sorted(ids(s.get_reports(limit=100, min_participants=3, max_participants=4))) == ["t4", "t5"]
    assert sorted(ids(s.get_reports(limit=100, min_messages=4, max_messages=12))) == ["t2", "t4", "t5"]
    assert sorted(ids(s.get_reports(limit=100, source="ietf-quic"))) == ["t1", "t3"]
    assert ids(s.get_reports(limit=100, source="ietf-quic", min_messages=2)) == ["t1"]
    assert s.get_reports(limit=100, source="nobody") == []
    assert s.get_sources() == ["ietf-quic", "ietf-tls"]


def test_reports_are_enriched_and_sorted(svc):
    s, _ = svc
    r = {d["thread_id"]: d for d in s.get_reports(limit=100)}
    assert r["t2"]["thread_metadata"] == {"subject": "st2", "participants": [f"p{j}@x" for j in range(5)],
                                          "participant_count": 5, "message_count": 12,
                                          "first_message_date": "2025-02-01T00:00:00Z",
                                          "last_message_date": "2025-02-05T00:00:00Z"}
    assert r["t2"]["archive_metadata"]["source"] == "ietf-tls"
    assert "archive_metadata" not in r["t5"]                   # archive gone: enrichment skipped gracefully
    # thread_start_date: missing dates last in BOTH directions
    asc = ids(s.get_reports(limit=100, sort_by="thread_start_date", sort_order="asc"))
    desc = ids(s.get_reports(limit=100, sort_by="thread_start_date", sort_order="desc"))
    assert asc == ["t1", "t5", "t2", "t3", "t4"] and desc == ["t3", "t2", "t5", "t1", "t4"]
    assert ids(s.get_reports(limit=100, sort_by="generated_at", sort_order="asc")) == ["t1", "t2", "t3", "t4", "t5"]
    # pagination after filtering + sorting
    assert ids(s.get_reports(limit=2, skip=1, sort_by="generated_at", sort_order="asc")) == ["t2", "t3"]
    assert s.get_reports(limit=10, skip=50) == []
    # a report whose thread no longer exists is not listed
    s.store.delete_document("threads", "t3")
    assert "t3" not in ids(s.get_reports(limit=100))


def test_threads_enriched_sorted_paged(svc):
    s, _ = svc
    th = {t["_id"]: t for t in s.get_threads(limit=100)}
    assert th["t1"]["archive_source"] == "ietf-quic" and th["t5"]["archive_source"] is None
    assert [t["_id"] for t in s.get_threads(limit=100, sort_by="last_message_date", sort_order="desc")] == \
        ["t5", "t3", "t2", "t1", "t4"]
    assert [t["_id"] for t in s.get_threads(limit=100, archive_id="a2")] == ["t2", "t4"]
    assert s.get_threads(limit=5, skip=10) == []


def test_write_path_events_and_failures(svc):
    s, pub = svc
    data = {"summary_id": "ab" * 32, "thread_id": "t1", "summary_markdown": "# ok", "citations": [
        {"chunk_id": "c1", "message_id": "<m@x>", "text": "quote"}], "llm_backend": "hip", "llm_model": "m",
        "tokens_prompt": 10, "tokens_completion": 5, "latency_ms": 7}
    rid = s.process_summary(data)
    doc = s.store.get_document("summaries", rid)
    assert doc["citations"][0]["quote"] == "quote" and doc["first_message_date"] == "2025-01-01T00:00:00Z"
    assert s.store.get_document("threads", "t1")["summary_id"] == rid
    assert s.process_summary(data) == rid                      # idempotent: same id, no duplicate
    assert [e["event_type"] for e in pub.get_events()] == ["ReportPublished", "ReportPublished"]
    with pytest.raises(DocumentNotFoundError):                 # thread not there yet: retryable
        s.process_summary({**data, "thread_id": "missing"})
    with pytest.raises(ValueError):
        s.process_summary({"summary_markdown": "x"})
    # webhook failure -> ReportDeliveryFailed, report still published
    s.notify_enabled, s.webhook_url = True, "http://127.0.0.1:9/unreachable"
    s.process_summary({**data, "thread_id": "t2", "summary_id": "cd" * 32})
    kinds = [e["event_type"] for e in pub.get_events()]
    assert kinds[-2:] == ["ReportDeliveryFailed", "ReportPublished"]
    assert pub.get_events("ReportPublished")[-1]["data"]["notified"] is False


def test_routes_validation_and_health(svc):
    s, _ = svc
    app = create_app(s, extra_routes=reporting_routes)
    c = TestClient(app)
    assert c.get("/readyz").status_code == 503                 # not started
    s.start()
    assert c.get("/readyz").json() == {"status": "ready", "service": "reporting"}
    assert c.get("/api/reports", params={"sort_by": "thread_start_date", "sort_order": "asc"}).json()["count"] == 5
    for bad in ({"sort_by": "subject"}, {"sort_order": "up"}, {"limit": 0}, {"skip": -1}, {"min_messages": -1}):
        assert c.get("/api/reports", params=bad).status_code == 422, bad
    assert c.get("/api/threads", params={"sort_by": "subject"}).status_code == 422
    assert c.get("/api/reports/search", params={"topic": "x"}).status_code == 503     # no vector store
    # a consumer thread that died: unhealthy and not ready (reference reporting/main.py:79-121)
    t = threading.Thread(target=lambda: None)
    t.start()
    t.join()
    s.consumer_thread = t
    assert c.get("/health").json()["status"] == "unhealthy"
    assert c.get("/readyz").status_code == 503
