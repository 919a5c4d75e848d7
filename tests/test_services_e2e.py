"""Whole pipeline through the services and the in-process bus (the reference's docker-compose CI
job, .github/workflows/docker-compose-ci.yml: create source -> trigger -> poll reports), CPU,
mock LLM and the tiny HIP-encoder architecture on the CPU reference path."""
import os
import shutil

from fastapi.testclient import TestClient

from copilot_for_consensus_amd.bus import NoopPublisher
from copilot_for_consensus_amd.contracts.registry import default_provider
from copilot_for_consensus_amd.embedding import HipEncoderProvider
from copilot_for_consensus_amd.services.base import create_app
from copilot_for_consensus_amd.services.ingestion import ingestion_routes
from copilot_for_consensus_amd.services.node import Node
from copilot_for_consensus_amd.services.reporting import reporting_routes
from copilot_for_consensus_amd.summarization import MockSummarizer
from copilot_for_consensus_amd.vectorstore import HipFlatIndex

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "sample.mbox")
ENV = {"DOCUMENT_STORE_TYPE": "inmemory", "MESSAGE_BUS_TYPE": "inproc", "METRICS_TYPE": "prometheus",
       "LOG_TYPE": "silent", "ERROR_REPORTER_TYPE": "silent", "EMBEDDING_BACKEND_TYPE": "mock",
       "VECTOR_STORE_TYPE": "inmemory", "LLM_BACKEND_TYPE": "mock", "ARCHIVE_STORE_TYPE": "inmemory",
       "SECRET_PROVIDER_TYPE": "env"}


def _node(tmp_path):
    emb = HipEncoderProvider(model_name="tiny", device="cpu")
    return Node(env=ENV, embedding_provider=emb, vector_store=HipFlatIndex(emb.dimension, device="cpu"),
                summarizer=MockSummarizer(mock_latency_ms=0))


def test_pipeline_via_rest_and_bus(tmp_path):
    node = _node(tmp_path)
    node.start(threaded=False)
    app = create_app(node.services["reporting"], extra_routes=reporting_routes)
    ingestion_routes(app, node.services["ingestion"], None)
    c = TestClient(app)
    src_dir = tmp_path / "src"
    src_dir.mkdir()
    shutil.copy(FIX, src_dir / "list.mbox")
    r = c.post("/api/sources", json={"name": "wg", "source_type": "local", "url": str(src_dir)})
    assert r.status_code == 201, r.text
    r = c.post("/api/sources/wg/trigger")
    assert r.status_code == 200 and len(r.json()["archive_ids"]) == 1
    first = r.json()["archive_ids"]
    node.drain()
    # a manual re-trigger forces re-ingestion (reference trigger_ingestion deletes the source's
    # archive records first); the deterministic ids keep every downstream write idempotent
    assert c.post("/api/sources/wg/trigger").json()["archive_ids"] == first
    node.drain()
    reports = c.get("/api/reports", params={"limit": 100}).json()["reports"]
    assert len(reports) == 2
    threads = c.get("/api/threads").json()["threads"]
    assert all(t["summary_id"] for t in threads)
    rep = c.get(f"/api/reports/{reports[0]['_id']}").json()
    assert rep["content_markdown"].startswith("# Summary")
    assert c.get(f"/api/threads/{rep['thread_id']}/summary").status_code == 200
    msgs = c.get("/api/messages", params={"thread_id": rep["thread_id"]}).json()["messages"]
    assert len(msgs) == 5
    chunks = c.get("/api/chunks", params={"thread_id": rep["thread_id"]}).json()["chunks"]
    assert chunks and all(ch["embedding_generated"] for ch in chunks)
    assert c.get("/api/sources").json()["sources"] == ["wg"]
    # semantic search returns the summarised threads
    hits = c.get("/api/reports/search", params={"topic": msgs[0]["body_normalized"][:200], "min_score": 0.0}).json()
    assert hits["count"] >= 1
    assert c.get("/health").json()["status"] == "healthy"
    assert "copilot_" in c.get("/metrics").text
    # filters
    assert c.get("/api/reports", params={"min_messages": 6}).json()["count"] == 0
    assert c.get("/api/reports", params={"source": "wg"}).json()["count"] == 2


def test_events_are_schema_valid_and_cascade_delete(tmp_path):
    node = _node(tmp_path)
    rec = NoopPublisher()
    for s in node.services.values():  # tap every publisher
        inner = s.publisher

        def tap(exchange, rk, ev, inner=inner):
            rec.publish(exchange, rk, ev)
            inner.publish(exchange, rk, ev)
        s.publisher = type("Tap", (), {"publish": staticmethod(tap)})()
    node.start(threaded=False)
    ing = node.services["ingestion"]
    src_dir = tmp_path / "s2"
    src_dir.mkdir()
    shutil.copy(FIX, src_dir / "a.mbox")
    ing.create_source({"name": "s2", "source_type": "local", "url": str(src_dir)})
    ing.trigger_ingestion("s2")
    node.drain()
    sp = default_provider()
    types = {e["event_type"] for e in rec.get_events()}
    assert {"ArchiveIngested", "JSONParsed", "ChunksPrepared", "EmbeddingsGenerated", "SummarizationRequested",
            "SummaryComplete", "ReportPublished"} <= types
    for e in rec.get_events():
        assert sp.validate_event(e) == [], (e["event_type"], sp.validate_event(e))
    assert node.store.count_documents("messages") == 10
    res = ing.delete_source_cascade("s2")
    node.drain()
    assert res["archives_deleted"] == 1
    assert node.store.count_documents("messages") == 0
    assert node.store.count_documents("chunks") == 0
    assert any(e["event_type"] == "SourceCleanupProgress" for e in rec.get_events())


def test_threaded_consumers(tmp_path):
    import time
    node = _node(tmp_path)
    node.start(threaded=True)
    try:
        ing = node.services["ingestion"]
        src = tmp_path / "s3"
        src.mkdir()
        shutil.copy(FIX, src / "a.mbox")
        ing.create_source({"name": "s3", "source_type": "local", "url": str(src)})
        ing.trigger_ingestion("s3")
        deadline = time.time() + 60
        while time.time() < deadline and node.store.count_documents("summaries") < 2:
            time.sleep(0.05)
        assert node.store.count_documents("summaries") == 2
    finally:
        node.stop()
