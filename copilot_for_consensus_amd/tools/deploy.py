"""Deployment artefacts derived from the code, so they cannot drift from it.

Parity target: infra/rabbitmq/definitions.json (one topic exchange ``copilot.events``, a durable
queue per consumer bound to its routing keys), infra/prometheus/prometheus.yml (+ alert rules for
the documented SLOs, infra/prometheus/alerts/slo_latency.yml) and the docker-compose service
topology of the reference.  Here:

* RabbitMQ definitions come from each service's ``subscriptions()`` (queue = service name, one
  binding per subscribed event's routing key) plus one ``<routing key>`` queue per *Failed event
  for the failed-queue tooling, and dead-letter policies (the reference has none);
* Prometheus config scrapes every service's ``/metrics`` and the pipeline exporter; alert rules
  carry the reference's SLO thresholds (parse P95 > 5 s, chunk > 2 s, embed > 10 s, summarize
  > 30 s, reporting API > 0.5 s);
* docker-compose: one MI355X node runs the whole pipeline in one process (``node``) with the GPU
  devices mapped; the per-service form is emitted too for multi-host deployments, with the
  reference's RabbitMQ + MongoDB (docker-compose.yml) or with this framework's native broker,
  document store server and HIP vector store (docker-compose.native.yml);
* the eight alert groups, eleven Grafana dashboards, Loki/Promtail, the Mongo bootstrap script and
  the Kubernetes manifests come from :mod:`.ops_assets`.

    python -m copilot_for_consensus_amd.tools.deploy --out deploy

Reference lines: prometheus.yml:19-26 (push model), :23-60 (scrape jobs);
alerts/slo_latency.yml:18-305.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

from ..contracts.events import EVENT_SPECS, EXCHANGE, routing_key_for

SERVICE_PORTS = {"ingestion": 8001, "parsing": 8002, "chunking": 8003, "embedding": 8004, "orchestrator": 8005,
                 "summarization": 8006, "reporting": 8007, "auth": 8090}

SLO_RULES = [  # (service, histogram, p95 threshold seconds) from the reference's alert rules
    ("parsing", "parsing_event_processing_seconds", 5.0),
    ("chunking", "chunking_event_processing_seconds", 2.0),
    ("embedding", "embedding_event_processing_seconds", 10.0),
    ("summarization", "summarization_event_processing_seconds", 30.0),
    ("reporting", "reporting_event_processing_seconds", 0.5),
]


def _subscriptions() -> dict[str, list[str]]:
    from .gateway import _MOCK_ENV
    from ..services.node import Node
    node = Node(env=_MOCK_ENV)
    return {name: sorted(svc.subscriptions()) for name, svc in node.services.items() if svc.subscriptions()}


def rabbitmq_definitions() -> dict:
    subs = _subscriptions()
    queues, bindings = [], []
    dlx = f"{EXCHANGE}.dlx"
    for svc, events in sorted(subs.items()):
        queues.append({"name": svc, "vhost": "/", "durable": True, "auto_delete": False,
                       "arguments": {"x-dead-letter-exchange": dlx, "x-dead-letter-routing-key": f"{svc}.dlq"}})
        queues.append({"name": f"{svc}.dlq", "vhost": "/", "durable": True, "auto_delete": False, "arguments": {}})
        bindings.append({"source": dlx, "vhost": "/", "destination": f"{svc}.dlq", "destination_type": "queue",
                         "routing_key": f"{svc}.dlq", "arguments": {}})
        for et in events:
            bindings.append({"source": EXCHANGE, "vhost": "/", "destination": svc, "destination_type": "queue",
                             "routing_key": routing_key_for(et), "arguments": {}})
    for et in sorted(EVENT_SPECS):
        if et.endswith("Failed"):
            rk = routing_key_for(et)
            queues.append({"name": rk, "vhost": "/", "durable": True, "auto_delete": False, "arguments": {}})
            bindings.append({"source": EXCHANGE, "vhost": "/", "destination": rk, "destination_type": "queue",
                             "routing_key": rk, "arguments": {}})
    return {"vhosts": [{"name": "/"}],
            "exchanges": [{"name": EXCHANGE, "vhost": "/", "type": "topic", "durable": True, "auto_delete": False,
                           "internal": False, "arguments": {}},
                          {"name": dlx, "vhost": "/", "type": "direct", "durable": True, "auto_delete": False,
                           "internal": False, "arguments": {}}],
            "queues": queues, "bindings": bindings,
            "policies": [{"vhost": "/", "name": "delivery-limit", "pattern": "^(?!.*\\.dlq$).*",
                          "apply-to": "queues", "definition": {"delivery-limit": 8}, "priority": 0}]}


def prometheus_config() -> str:
    lines = ["global:", "  scrape_interval: 15s", "  evaluation_interval: 15s", "rule_files:", "  - alerts.yml",
             "  - alerts/*.yml", "scrape_configs:"]
    for svc, port in SERVICE_PORTS.items():
        lines += [f"  - job_name: {svc}", "    static_configs:", f"      - targets: ['{svc}:{port}']"]
    lines += ["  - job_name: pipeline-exporter", "    static_configs:", "      - targets: ['exporter:9502']",
              "  - job_name: pushgateway", "    honor_labels: true", "    static_configs:",
              "      - targets: ['pushgateway:9091']"]
    return "\n".join(lines) + "\n"


def alert_rules() -> str:
    lines = ["groups:", "  - name: slo_latency", "    rules:"]
    for svc, hist, thr in SLO_RULES:
        lines += [f"      - alert: {svc.capitalize()}LatencyP95High",
                  f"        expr: histogram_quantile(0.95, sum(rate({hist}_bucket[5m])) by (le)) > {thr}",
                  "        for: 5m", "        labels: {severity: warning}",
                  f"        annotations: {{summary: '{svc} p95 latency above {thr}s'}}"]
    lines += ["  - name: pipeline_health", "    rules:",
              "      - alert: DocumentsStuck",
              "        expr: max(copilot_document_age_seconds{status=~'pending|processing'}) > 3600",
              "        for: 15m", "        labels: {severity: warning}",
              "        annotations: {summary: 'documents pending/processing for over an hour'}"]
    return "\n".join(lines) + "\n"


def grafana_dashboard() -> dict:
    """One dashboard over the pipeline + GPU metrics (the reference ships 11 Grafana JSON files;
    the panels here cover its service-health, latency and document-state views plus the MI355X
    engine figures)."""
    def panel(i, title, expr, unit="short", kind="timeseries"):
        return {"id": i, "type": kind, "title": title, "gridPos": {"h": 8, "w": 12, "x": 12 * (i % 2), "y": 8 * (i // 2)},
                "fieldConfig": {"defaults": {"unit": unit}, "overrides": []},
                "targets": [{"expr": e, "refId": chr(65 + j)} for j, e in enumerate([expr] if isinstance(expr, str) else expr)]}
    ps = [
        panel(0, "Threads summarized / s", "sum(rate(summarization_tokens_total{type='completion'}[5m])) / 512"),
        panel(1, "Summarization batch latency p50 / p95",
              ["histogram_quantile(0.5, sum(rate(summarization_latency_seconds_bucket[5m])) by (le))",
               "histogram_quantile(0.95, sum(rate(summarization_latency_seconds_bucket[5m])) by (le))"], "s"),
        panel(2, "Decode tokens / s (GPU)", "summarization_gpu_decode_tokens_per_second"),
        panel(3, "Prefill tokens / s (GPU)", "summarization_gpu_prefill_tokens_per_second"),
        panel(4, "Time to first token", "summarization_gpu_ttft_seconds", "s"),
        panel(5, "HBM used", ["summarization_gpu_hbm_used_bytes", "summarization_gpu_kv_cache_bytes"], "bytes"),
        panel(6, "Stage latency p95", [f"histogram_quantile(0.95, sum(rate({h}_bucket[5m])) by (le))"
                                       for _, h, _ in SLO_RULES], "s"),
        panel(7, "Documents by status", "sum by (collection, status) (copilot_document_status_count)"),
        panel(8, "Chunks awaiting embedding", "copilot_chunks_embedding_status_count{embedding_generated='false'}"),
        panel(9, "Prefix-cache hit tokens / batch", "summarization_gpu_prefix_cached_tokens"),
    ]
    return {"title": "Copilot for Consensus - MI355X", "uid": "cfc-mi355x", "schemaVersion": 39, "version": 1,
            "time": {"from": "now-6h", "to": "now"}, "refresh": "30s", "panels": ps}


def compose() -> str:
    gpu = ["    devices: ['/dev/kfd', '/dev/dri']", "    group_add: ['video', 'render']", "    ipc: host",
           "    shm_size: 64g", "    environment:", "      - HSA_ENABLE_IPC_MODE_LEGACY=0"]
    base_env = ["      - MESSAGE_BUS_TYPE=rabbitmq", "      - RABBITMQ_HOST=messagebus", "      - DOCUMENT_STORE_TYPE=mongodb",
                "      - MONGODB_HOST=documentdb", "      - METRICS_TYPE=prometheus"]
    out = ["services:",
           "  # single MI355X node: every stage in one process on the in-process bus (recommended)",
           "  node:", "    image: copilot-for-consensus-amd:latest", "    profiles: ['node']",
           "    command: python -m copilot_for_consensus_amd.services.main node --port 8080",
           "    ports: ['8080:8080']"] + gpu + ["      - DOCUMENT_STORE_TYPE=inmemory", "      - MESSAGE_BUS_TYPE=inproc"]
    out += ["  messagebus:", "    image: rabbitmq:3-management", "    profiles: ['services']",
            "    volumes: ['./rabbitmq/definitions.json:/etc/rabbitmq/definitions.json:ro']",
            "    environment:", "      - RABBITMQ_SERVER_ADDITIONAL_ERL_ARGS=-rabbitmq_management load_definitions "
            "\"/etc/rabbitmq/definitions.json\"",
            "  documentdb:", "    image: mongo:7", "    profiles: ['services']",
            "    volumes: ['./mongo/mongo-init.js:/docker-entrypoint-initdb.d/mongo-init.js:ro']"]
    for svc, port in SERVICE_PORTS.items():
        out += [f"  {svc}:", "    image: copilot-for-consensus-amd:latest", "    profiles: ['services']",
                f"    command: python -m copilot_for_consensus_amd.services.main {svc} --port {port}",
                f"    ports: ['{port}:{port}']"]
        if svc in ("embedding", "summarization", "reporting"):
            out += gpu + base_env[:]
        else:
            out += ["    environment:"] + base_env
        out += ["    depends_on: [messagebus, documentdb]"]
    out += ["  prometheus:", "    image: prom/prometheus", "    profiles: ['services', 'node']",
            "    volumes: ['./prometheus:/etc/prometheus:ro']", "    ports: ['9090:9090']",
            "  grafana:", "    image: grafana/grafana", "    profiles: ['services', 'node']",
            "    volumes: ['./grafana/dashboards:/var/lib/grafana/dashboards:ro']", "    ports: ['3000:3000']",
            "  loki:", "    image: grafana/loki", "    profiles: ['services', 'node']",
            "    command: -config.file=/etc/loki/loki-config.yml",
            "    volumes: ['./loki:/etc/loki:ro']", "    ports: ['3100:3100']",
            "  promtail:", "    image: grafana/promtail", "    profiles: ['services', 'node']",
            "    command: -config.file=/etc/promtail/promtail-config.yml",
            "    volumes: ['./promtail:/etc/promtail:ro', '/var/run/docker.sock:/var/run/docker.sock:ro']"]
    return "\n".join(out) + "\n"


def compose_native() -> str:
    """One service per container with this framework's own infrastructure in place of RabbitMQ,
    MongoDB and Qdrant: the native broker (csrc/broker), the document store server (WAL +
    snapshots) and the HIP index behind Qdrant's REST API, each on a persistent volume."""
    gpu = ["    devices: ['/dev/kfd', '/dev/dri']", "    group_add: ['video', 'render']", "    ipc: host"]
    env = ["      - MESSAGE_BUS_TYPE=cfcbroker", "      - CFC_BROKER_HOST=messagebus", "      - CFC_BROKER_PORT=5680",
           "      - DOCUMENT_STORE_TYPE=cfcstore", "      - CFC_DOCSTORE_HOST=documentdb", "      - CFC_DOCSTORE_PORT=27027",
           "      - VECTOR_STORE_TYPE=qdrant", "      - QDRANT_HOST=vectorstore", "      - QDRANT_PORT=6333",
           "      - ARCHIVE_STORE_TYPE=local", "      - ARCHIVE_BASE_PATH=/data/raw_archives",
           "      - METRICS_TYPE=prometheus", "      - HSA_ENABLE_IPC_MODE_LEGACY=0"]
    img = "    image: copilot-for-consensus-amd:latest"
    out = ["services:",
           "  messagebus:", img, "    command: python -m copilot_for_consensus_amd.services.main broker --port 5680 "
           "--data-dir /data/broker", "    volumes: ['broker:/data/broker']",
           "    healthcheck: {test: ['CMD', 'python', '-c', \"import socket; socket.create_connection(('localhost', 5680))\"]}",
           "  documentdb:", img, "    command: python -m copilot_for_consensus_amd.services.main docstore --port 27027 "
           "--data-dir /data/docstore", "    volumes: ['docstore:/data/docstore']",
           "  vectorstore:", img, "    command: python -m copilot_for_consensus_amd.services.main vectorstore --port 6333 "
           "--data-dir /data/vectors", "    volumes: ['vectors:/data/vectors']"] + gpu + \
          ["    environment:", "      - VECTOR_STORE_DEVICE=cuda", "      - HSA_ENABLE_IPC_MODE_LEGACY=0"]
    out += ["  llm:", img, "    command: python -m copilot_for_consensus_amd.services.main llm --port 8081",
            "    profiles: ['llm-server']", "    ports: ['8081:8081']"] + gpu + \
           ["    environment:", "      - LLM_MODEL_PRESET=mistral-7b", "      - HSA_ENABLE_IPC_MODE_LEGACY=0",
            "    # the llama-cpp / ollama containers' role: LLM_BACKEND_TYPE=llamacpp, LLAMACPP_ENDPOINT=http://llm:8081"]
    for svc, port in SERVICE_PORTS.items():
        if svc == "auth":
            continue
        out += [f"  {svc}:", img, f"    command: python -m copilot_for_consensus_amd.services.main {svc} --port {port}",
                f"    ports: ['{port}:{port}']"]
        if svc in ("embedding", "summarization", "reporting"):
            out += gpu
        out += ["    environment:"] + env
        if svc in ("ingestion", "parsing"):
            out += ["    volumes: ['archives:/data/raw_archives']"]
        out += ["    depends_on: [messagebus, documentdb, vectorstore]", "    restart: unless-stopped"]
    out += ["volumes:", "  broker: {}", "  docstore: {}", "  vectors: {}", "  archives: {}"]
    return "\n".join(out) + "\n"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Write RabbitMQ definitions, Prometheus config/alerts, compose file")
    ap.add_argument("--out", default="deploy")
    a = ap.parse_args(argv)
    out = Path(a.out)
    (out / "rabbitmq").mkdir(parents=True, exist_ok=True)
    (out / "prometheus").mkdir(parents=True, exist_ok=True)
    (out / "rabbitmq" / "definitions.json").write_text(json.dumps(rabbitmq_definitions(), indent=2) + "\n")
    (out / "prometheus" / "prometheus.yml").write_text(prometheus_config())
    (out / "prometheus" / "alerts.yml").write_text(alert_rules())
    (out / "docker-compose.yml").write_text(compose())
    (out / "docker-compose.native.yml").write_text(compose_native())
    (out / "grafana" / "dashboards").mkdir(parents=True, exist_ok=True)
    (out / "grafana" / "dashboards" / "copilot-mi355x.json").write_text(json.dumps(grafana_dashboard(), indent=2) + "\n")
    from . import ops_assets as ops
    import yaml
    (out / "prometheus" / "alerts").mkdir(parents=True, exist_ok=True)
    for stem, rules in ops.alert_groups().items():
        (out / "prometheus" / "alerts" / f"{stem}.yml").write_text(yaml.safe_dump(rules, sort_keys=False))
    for stem, dash in ops.dashboards().items():
        (out / "grafana" / "dashboards" / f"{stem}.json").write_text(json.dumps(dash, indent=2) + "\n")
    for sub, fname, body in (("loki", "loki-config.yml", ops.loki_config()),
                             ("promtail", "promtail-config.yml", ops.promtail_config())):
        (out / sub).mkdir(parents=True, exist_ok=True)
        (out / sub / fname).write_text(yaml.safe_dump(body, sort_keys=False))
    (out / "mongo").mkdir(parents=True, exist_ok=True)
    (out / "mongo" / "mongo-init.js").write_text(ops.mongo_init_js())
    (out / "k8s").mkdir(parents=True, exist_ok=True)
    (out / "k8s" / "copilot-mi355x.yaml").write_text(ops.k8s_yaml())
    print(f"wrote deployment files under {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
