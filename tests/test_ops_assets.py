"""Generated operations assets (tools/ops_assets.py, tools/deploy.py): the eight alert groups, the
eleven dashboards, Loki/Promtail, the Mongo bootstrap and the Kubernetes manifests -- every alert
and panel must read a metric that this framework (or a standard exporter) actually emits."""
from __future__ import annotations

import json
import re
from pathlib import Path

import pytest
import yaml

from copilot_for_consensus_amd.contracts.documents import collections_config
from copilot_for_consensus_amd.tools import ops_assets as ops
from copilot_for_consensus_amd.tools.deploy import SERVICE_PORTS, main, rabbitmq_definitions

PKG = Path(__file__).resolve().parents[1] / "copilot_for_consensus_amd"
STANDARD_PREFIXES = ("rabbitmq_", "mongodb_", "process_", "up")


def _emitted_metrics() -> set[str]:
    """Metric names the package emits: literal names in increment/observe/gauge calls and the
    exporter, plus the per-service f-string families expanded over the services."""
    src = "\n".join(p.read_text() for p in PKG.rglob("*.py"))
    names = set(re.findall(r"(?:increment|observe|gauge)\(\s*\"([a-z_]+)\"", src))
    names |= set(re.findall(r"_fmt\(\"([a-z_]+)\"", src))
    names |= set(re.findall(r"\"(copilot_[a-z_]+)\"", src))
    fam = set(re.findall(r"f\"\{(?:self\.name|service_name|service\.name)\}_([a-z_]+)\"", src))
    for svc in SERVICE_PORTS:
        names |= {f"{svc}_{s}" for s in fam}
    gpu = set(re.findall(r"gauge\(f\"summarization_gpu_\{k\}\"", src))
    assert gpu, "GPU gauge family not found"
    names |= {f"summarization_gpu_{k}" for k in ("decode_tokens_per_second", "prefill_tokens_per_second",
                                                 "ttft_seconds", "hbm_used_bytes", "kv_cache_bytes",
                                                 "prefix_cached_tokens")}
    return names


def _check_exprs(exprs, known):
    for e in exprs:
        for m in ops.metric_names(e):
            base = re.sub(r"_(bucket|sum|count)$", "", m)
            assert base in known or m in known or m.startswith(STANDARD_PREFIXES), (m, e)


def test_gpu_gauges_exist_in_summarizer():
    src = (PKG / "summarization" / "__init__.py").read_text()
    for k in ("decode_tokens_per_second", "prefill_tokens_per_second", "kv_cache_bytes"):
        assert k in src


def test_alert_groups_read_emitted_metrics():
    groups = ops.alert_groups()
    assert set(groups) == {"slo_latency", "slo_errors", "document_processing", "failed_queues", "queue_lag",
                           "retry_policy", "service_health", "resource_limits"}
    known = _emitted_metrics()
    seen = set()
    for stem, body in groups.items():
        rules = body["groups"][0]["rules"]
        assert rules, stem
        for r in rules:
            assert {"alert", "expr", "for", "labels", "annotations"} <= set(r)
            assert r["labels"]["severity"] in ("warning", "critical")
            assert r["alert"] not in seen
            seen.add(r["alert"])
        _check_exprs([r["expr"] for r in rules], known)
    # YAML round trip
    assert yaml.safe_load(yaml.safe_dump(groups["slo_latency"])) == groups["slo_latency"]


def test_dashboards_cover_the_reference_views():
    d = ops.dashboards()
    assert set(d) == {"document-processing-status", "failed-queues", "logs-overview", "mongodb-status",
                      "pipeline-flow", "queue-status", "resource-usage", "retry-policy", "service-metrics",
                      "system-health", "vectorstore-status"}
    known = _emitted_metrics()
    uids = set()
    for name, dash in d.items():
        assert dash["uid"] not in uids
        uids.add(dash["uid"])
        for p in dash["panels"]:
            assert p["targets"], (name, p["title"])
            if p["datasource"]["type"] == "prometheus":
                _check_exprs([t["expr"] for t in p["targets"]], known)
    assert all(p["datasource"]["type"] == "loki" for p in d["logs-overview"]["panels"])


def test_logs_configs():
    lc, pc = ops.loki_config(), ops.promtail_config()
    assert lc["server"]["http_listen_port"] == 3100
    assert pc["clients"][0]["url"].startswith("http://loki:3100")
    stages = pc["scrape_configs"][0]["pipeline_stages"]
    assert stages[0]["json"]["expressions"]["level"] == "level"


def test_mongo_init_and_store_indexes():
    js = ops.mongo_init_js()
    cfg = collections_config()
    for c in cfg["collections"]:
        assert f'"name": "{c["name"]}"' in js
        for i in c.get("indexes", []):
            assert i["options"]["name"] in js
    # MongoDocumentStore.ensure_collections against the stand-in pymongo (tests/fake_pymongo.py)
    import fake_pymongo
    mp = pytest.MonkeyPatch()
    try:
        server = fake_pymongo.install(mp)
        server.dbs["copilot"] = {"messages": fake_pymongo._CollData()}
        from copilot_for_consensus_amd.storage.document_store import MongoDocumentStore
        st = MongoDocumentStore(host="h")
        st.connect()
        assert st.ensure_collections() == sum(len(c.get("indexes", [])) for c in cfg["collections"])
    finally:
        mp.undo()
    assert {c["name"] for c in cfg["collections"]} <= set(server.dbs["copilot"])
    assert "name" in server.dbs["copilot"]["sources"].unique


def test_k8s_manifests():
    ms = ops.k8s_manifests(tp=2)
    deps = {m["metadata"]["name"]: m for m in ms if m["kind"] == "Deployment"}
    assert set(SERVICE_PORTS) <= set(deps)
    for svc, n in ops.GPU_SERVICES.items():
        lim = deps[svc]["spec"]["template"]["spec"]["containers"][0]["resources"]["limits"]["amd.com/gpu"]
        assert lim == (2 if svc == "summarization" else n)
    assert "resources" not in deps["parsing"]["spec"]["template"]["spec"]["containers"][0]
    queues = {q["name"] for q in rabbitmq_definitions()["queues"]}
    scalers = [m for m in ms if m["kind"] == "ScaledObject"]
    assert {s["spec"]["scaleTargetRef"]["name"] for s in scalers} == set(ops.BUS_SERVICES)
    for s in scalers:
        trig = s["spec"]["triggers"][0]["metadata"]
        assert trig["queueName"] in queues and trig["value"] == "5"
    docs = list(yaml.safe_load_all(ops.k8s_yaml()))
    assert len(docs) == len(ops.k8s_manifests())


def test_deploy_writes_everything(tmp_path):
    assert main(["--out", str(tmp_path)]) == 0
    assert len(list((tmp_path / "prometheus" / "alerts").glob("*.yml"))) == 8
    assert len(list((tmp_path / "grafana" / "dashboards").glob("*.json"))) == 12
    for f in (tmp_path / "grafana" / "dashboards").glob("*.json"):
        json.loads(f.read_text())
    assert "alerts/*.yml" in (tmp_path / "prometheus" / "prometheus.yml").read_text()
    compose = (tmp_path / "docker-compose.yml").read_text()
    assert "mongo-init.js" in compose and "loki" in compose and "promtail" in compose
    assert (tmp_path / "k8s" / "copilot-mi355x.yaml").exists()
