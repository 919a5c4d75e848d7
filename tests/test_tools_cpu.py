"""Operational tools: retry job, failed-queue manager, exporters, log mining, schema check,
gateway generation, StartupRequeue."""
import json
from datetime import datetime, timedelta, timezone

import pytest

from copilot_for_consensus_amd.bus import InProcBroker, InProcPublisher, InProcSubscriber, NoopPublisher
from copilot_for_consensus_amd.contracts.registry import default_provider
from copilot_for_consensus_amd.observability import PrometheusMetricsCollector
from copilot_for_consensus_amd.services.startup import StartupRequeue
from copilot_for_consensus_amd.storage.document_store import InMemoryDocumentStore
from copilot_for_consensus_amd.tools.exporters import PipelineExporter
from copilot_for_consensus_amd.tools.failed_queues import FailedQueueManager, InProcFailedQueues
from copilot_for_consensus_amd.tools.log_mining import Drain, mine, normalize_message
from copilot_for_consensus_amd.tools.retry_job import RetryStuckDocumentsJob


def _store():
    s = InMemoryDocumentStore()
    s.insert_document("archives", {"_id": "a1a1a1a1a1a1a1a1", "status": "pending", "source": "list", "file_hash": "abababababababababababababababababababababababababababababababab",
                                   "file_size_bytes": 10})
    s.insert_document("archives", {"_id": "a2a2a2a2a2a2a2a2", "status": "completed"})
    s.insert_document("archives", {"_id": "a3a3a3a3a3a3a3a3", "status": "processing", "attemptCount": 3})
    s.insert_document("messages", {"_id": "0101010101010101", "archive_id": "a2a2a2a2a2a2a2a2", "thread_id": "0101010101010101"})
    s.insert_document("messages", {"_id": "0202020202020202", "archive_id": "a2a2a2a2a2a2a2a2", "thread_id": "0101010101010101"})
    s.insert_document("chunks", {"_id": "0c0c0c0c0c0c0c0c", "message_doc_id": "0101010101010101", "thread_id": "0101010101010101", "embedding_generated": False})
    return s


def test_retry_job_requeues_with_backoff_and_caps():
    s, pub = _store(), NoopPublisher()
    clock = [datetime(2025, 1, 1, tzinfo=timezone.utc)]
    job = RetryStuckDocumentsJob(s, pub, base_delay_seconds=300, stuck_threshold_hours=24, clock=lambda: clock[0])
    r = job.run_once()
    assert r["archives"]["requeued"] == 1 and r["archives"]["max_retries_exceeded"] == 1
    assert r["messages"]["requeued"] == 1 and r["chunks"]["requeued"] == 1
    assert s.get_document("archives", "a3a3a3a3a3a3a3a3")["status"] == "failed_max_retries"
    assert s.get_document("archives", "a1a1a1a1a1a1a1a1")["attemptCount"] == 1
    prov = default_provider()
    for ev in pub.get_events():
        assert prov.validate_event(ev) == [], ev
    # backoff: 1st retry after 300 s
    clock[0] += timedelta(seconds=100)
    assert job.run_once()["archives"]["skipped_backoff"] == 1
    clock[0] += timedelta(seconds=300)
    assert job.run_once()["archives"]["requeued"] == 1
    assert job.backoff_seconds(10) == 3600


def test_failed_queue_manager_inproc():
    broker = InProcBroker(max_redeliveries=1)
    fq = FailedQueueManager(InProcFailedQueues(broker))
    pub = InProcPublisher(broker)
    from copilot_for_consensus_amd.contracts.events import Event
    ev = Event.create("ParsingFailed", archive_id="a1a1a1a1a1a1a1a1", error_message="boom", error_type="X", retry_count=0,
                      failed_at="2025-01-01T00:00:00Z").to_dict()
    pub.publish("copilot.events", "parsing.failed", ev)
    q = {d["queue"]: d for d in fq.list_failed_queues()}
    assert q["parsing.failed"]["message_count"] == 1 and q["parsing.failed"]["target"] == "archive.ingested"
    assert fq.inspect_messages("parsing.failed")[0]["event_id"] == ev["event_id"]
    # requeue moves it to the mapped routing key
    sub = InProcSubscriber(broker, queue_name="parsing")
    got = []
    sub.subscribe("ParsingFailed", got.append, routing_key="archive.ingested")
    assert fq.requeue_messages("parsing.failed", dry_run=True) == 1
    assert fq.requeue_messages("parsing.failed") == 1
    sub.drain()
    assert len(got) == 1 and fq.list_failed_queues()[0]["message_count"] == 0
    pub.publish("copilot.events", "parsing.failed", ev)
    assert fq.purge_messages("parsing.failed") == 1


def test_exporter_renders_prometheus_text():
    txt = PipelineExporter(_store()).render()
    assert 'copilot_document_status_count{collection="archives",database="copilot",status="pending"} 1.0' in txt
    assert 'copilot_chunks_embedding_status_count{database="copilot",embedding_generated="false"} 1.0' in txt


def test_log_mining_templates():
    assert normalize_message("at 2025-01-01T00:00:00Z from 10.0.0.1 id 42") == "at <TS> from <IP> id <NUM>"
    lines = [json.dumps({"service": "parsing", "message": f"parsed archive {i} in {i * 3} ms"}) for i in range(20)]
    lines += ["embedding | failed to connect to host qdrant port 6333"] * 2
    lines += ["a totally unique line"]
    rep = mine(lines, group_by_service=True)
    top = rep["templates"][0]
    assert top["count"] == 20 and top["service"] == "parsing" and "<NUM>" in top["template"]
    assert rep["meta"]["services"] == ["embedding", "parsing"]
    assert any(t["template"] == "a totally unique line" for t in rep["anomalies"]["rare_templates"])
    d = Drain()
    a = d.add("user alice logged in")
    b = d.add("user bob logged in")
    assert a is b and a.template == "user <*> logged in"


def test_schema_registry_check_and_export(tmp_path):
    from copilot_for_consensus_amd.tools.schemas import check, export_all
    assert check() == []
    files = export_all(tmp_path)
    assert (tmp_path / "events" / "ArchiveIngested.schema.json").exists()
    assert (tmp_path / "configs" / "services" / "parsing.json").exists() and len(files) > 25


def test_gateway_generation(tmp_path):
    from copilot_for_consensus_amd.tools.gateway import main
    assert main(["--out", str(tmp_path)]) == 0
    g = json.loads((tmp_path / "gateway.openapi.json").read_text())
    for p in ("/reporting/api/reports/search", "/ingestion/api/sources/{name}/trigger", "/auth/.well-known/jwks.json",
              "/ingestion/api/uploads", "/reporting/api/threads/{thread_id}/summary"):
        assert p in g["paths"], p
    conf = (tmp_path / "nginx.conf").read_text()
    assert "location /reporting/" in conf and "client_max_body_size 100m" in conf
    # cloud gateways (reference infra/gateway/{aws,azure,gcp}_adapter.py): every operation routed
    cf = json.loads((tmp_path / "aws" / "cloudformation.json").read_text())
    body = cf["Resources"]["Api"]["Properties"]["Body"]
    trig = body["paths"]["/ingestion/api/sources/{name}/trigger"]["post"]["x-amazon-apigateway-integration"]
    assert trig["uri"] == "http://ingestion:8080/api/sources/{name}/trigger"
    assert trig["requestParameters"] == {"integration.request.path.name": "method.request.path.name"}
    apim = json.loads((tmp_path / "azure" / "apim.json").read_text())
    assert "validate-jwt" in apim["resources"][1]["properties"]["value"]
    assert json.loads(apim["resources"][0]["properties"]["value"])["paths"] == g["paths"]
    gcp = json.loads((tmp_path / "gcp" / "api_config.json").read_text())
    search = gcp["paths"]["/reporting/api/reports/search"]["get"]
    assert search["x-google-backend"]["address"] == "http://reporting:8080/api/reports/search"
    assert search["security"] == [{"copilot_jwt": []}]
    assert "security" not in gcp["paths"]["/auth/.well-known/jwks.json"]["get"]


def test_cloud_gateway_with_public_backend(tmp_path):
    from copilot_for_consensus_amd.tools import gateway as G
    spec = {"openapi": "3.1.0", "paths": {"/reporting/api/reports/{report_id}": {"get": {
        "parameters": [{"name": "report_id", "in": "path"}]}}}}
    cf = G.aws_cloudformation(spec, "https://api.example.org")
    op = cf["Resources"]["Api"]["Properties"]["Body"]["paths"]["/reporting/api/reports/{report_id}"]["get"]
    assert op["x-amazon-apigateway-integration"]["uri"] == "https://api.example.org/reporting/api/reports/{report_id}"
    assert G.validate_cloud_config(spec, "aws", cf) == []
    assert G.validate_cloud_config(spec, "gcp", {"paths": {"/x": {"get": {}}}}) == ["GET /x"]


def test_startup_requeue_generic():
    s, pub = _store(), NoopPublisher()
    m = PrometheusMetricsCollector()
    n = StartupRequeue(s, pub, m).requeue_incomplete(
        "chunks", {"embedding_generated": False}, "ChunksPrepared", "chunks.prepared", "_id",
        lambda c: dict(message_doc_ids=[c["message_doc_id"]], chunk_count=1, chunk_ids=[c["_id"]], chunks_ready=True,
                       chunking_strategy="requeue", avg_chunk_size_tokens=0))
    assert n == 1 and default_provider().validate_event(pub.get_events()[0]) == []
    assert "startup_requeue_documents_total" in m.render()


def test_ui_served():
    from fastapi import FastAPI
    from fastapi.testclient import TestClient
    from copilot_for_consensus_amd.ui import ui_routes
    app = FastAPI()
    ui_routes(app)
    c = TestClient(app)
    r = c.get("/ui")
    assert r.status_code == 200 and "Copilot for Consensus" in r.text and "/api/reports/search" in r.text
    # reference ui/src/routes: Login, Callback, AdminDashboard / PendingAssignments / UserRolesList
    for route in ("async login(q)", "async callback(q)", "async admin(q)", "async summary(_, id)", "/admin/role-assignments/pending",
                  "/admin/users/search"):
        assert route in r.text, route
    # ReportsList / DiscussionsList filters + paging, MessageDetail chunks, UserRolesList
    for needle in ("message_start_date", "max_participants", "sort_order", "thread_start_date", "first_message_date",
                   "/api/chunks?message_doc_id=", "/roles`", "function pager"):
        assert needle in r.text, needle
    assert c.get("/", follow_redirects=False).status_code in (302, 307)


def test_ui_script_parses(tmp_path):
    """The page's script is valid JavaScript (node --check; ``??`` rewritten for old node versions)."""
    import re
    import shutil
    import subprocess
    node = shutil.which("node")
    if node is None:
        pytest.skip("node not installed")
    from copilot_for_consensus_amd.ui import INDEX
    html = INDEX.read_text(encoding="utf-8")
    js = re.search(r"<script>(.*)</script>", html, re.S).group(1).replace("??", "||")
    f = tmp_path / "ui.js"
    f.write_text(js)
    r = subprocess.run([node, "--check", str(f)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr


def test_deploy_artifacts(tmp_path):
    from copilot_for_consensus_amd.tools.deploy import main, rabbitmq_definitions
    d = rabbitmq_definitions()
    b = {(x["destination"], x["routing_key"]) for x in d["bindings"]}
    assert ("parsing", "archive.ingested") in b and ("summarization", "summarization.requested") in b
    assert ("parsing.failed", "parsing.failed") in b
    assert any(e["type"] == "topic" and e["name"] == "copilot.events" for e in d["exchanges"])
    assert main(["--out", str(tmp_path)]) == 0
    assert "histogram_quantile(0.95" in (tmp_path / "prometheus" / "alerts.yml").read_text()
    assert "services.main node" in (tmp_path / "docker-compose.yml").read_text()
