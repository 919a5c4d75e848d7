"""Operations assets generated from the code: Prometheus alert groups, Grafana dashboards, Loki /
Promtail configs, the Mongo collection/index bootstrap script and Kubernetes manifests.

Parity targets in the reference (behaviour, not text):

* infra/prometheus/alerts/*.yml -- eight alert files (document_processing, failed_queues,
  queue_lag, resource_limits, retry_policy, service_health, slo_errors, slo_latency).  The same
  eight groups are emitted here, written against the metric names THIS framework exports
  (``<service>_event_processing_seconds``, ``<service>_events_failed_total``,
  ``<service>_http_request_duration_seconds``, the pipeline exporter's ``copilot_*`` gauges) plus
  ``rabbitmq_*`` / ``up`` from the standard exporters; resource_limits gains the MI355X HBM gauges.
* infra/grafana/dashboards/*.json -- eleven dashboards; the same eleven views are generated here
  (logs-overview reads Loki), plus the GPU engine dashboard of :func:`.deploy.grafana_dashboard`.
* infra/loki/loki-config.yml, infra/promtail/promtail-config.yml -- single-binary Loki and a
  Promtail that tails container logs and parses this framework's JSON log lines.
* infra/init/mongo-init.js -- creates the collections and indexes listed in
  collections.config.json (here generated from :func:`contracts.documents.collections_config`).
* infra/azure/*.bicep (Container Apps with Service Bus queue-length scale rules) -- this framework
  targets MI355X nodes, so the equivalent is Kubernetes: one Deployment per service, the GPU stages
  requesting ``amd.com/gpu`` (AMD GPU device plugin), and KEDA ScaledObjects that scale each
  consumer on its RabbitMQ queue length (the Container Apps rule ``messageCount: 5``,
  containerapps.bicep:262-263).
"""
from __future__ import annotations

import json
import re

import yaml

from ..contracts.documents import collections_config
from .deploy import SERVICE_PORTS, SLO_RULES, rabbitmq_definitions

BUS_SERVICES = ("parsing", "chunking", "embedding", "orchestrator", "summarization", "reporting")
GPU_SERVICES = {"embedding": 1, "summarization": 1, "reporting": 1}
MAIN_QUEUE_DEPTH = {"parsing": (500, 2000), "chunking": (500, 2000), "embedding": (1000, 5000),
                    "orchestrator": (500, 2000), "summarization": (200, 1000)}


def _rule(alert: str, expr: str, for_: str, severity: str, summary: str) -> dict:
    return {"alert": alert, "expr": expr, "for": for_, "labels": {"severity": severity},
            "annotations": {"summary": summary}}


def _p(q: float, hist: str, window: str = "5m") -> str:
    return f"histogram_quantile({q}, sum(rate({hist}_bucket[{window}])) by (le))"


def alert_groups() -> dict[str, dict]:
    """{file stem: Prometheus rule file} for the eight alert groups."""
    g: dict[str, list[dict]] = {k: [] for k in ("slo_latency", "slo_errors", "document_processing", "failed_queues",
                                                "queue_lag", "retry_policy", "service_health", "resource_limits")}
    # --- latency SLOs (reference slo_latency.yml thresholds)
    for svc, hist, thr in SLO_RULES:
        g["slo_latency"].append(_rule(f"{svc.capitalize()}LatencyP95High", f"{_p(0.95, hist)} > {thr}", "5m",
                                      "warning", f"{svc} p95 latency above {thr}s"))
    g["slo_latency"] += [
        _rule("EmbeddingLatencyP99Critical", f"{_p(0.99, 'embedding_event_processing_seconds')} > 60", "5m",
              "critical", "embedding p99 latency above 60s"),
        _rule("SummarizationLatencyP99Critical", f"{_p(0.99, 'summarization_event_processing_seconds')} > 120", "5m",
              "critical", "summarization p99 latency above 120s"),
        _rule("IngestionAPILatencyHigh", f"{_p(0.95, 'ingestion_http_request_duration_seconds')} > 0.5", "5m",
              "warning", "ingestion API p95 above 500ms"),
        _rule("ReportingAPILatencyHigh", f"{_p(0.95, 'reporting_http_request_duration_seconds')} > 0.2", "5m",
              "warning", "reporting API p95 above 200ms"),
        _rule("ReportingAPILatencyCritical", f"{_p(0.95, 'reporting_http_request_duration_seconds')} > 0.5", "5m",
              "critical", "reporting API p95 above 500ms"),
    ]
    # --- error-rate SLOs
    for svc in BUS_SERVICES:
        err = (f"sum(rate({svc}_events_failed_total[5m])) / "
               f"clamp_min(sum(rate({svc}_events_processed_total[5m])) + sum(rate({svc}_events_failed_total[5m])), 1e-9)")
        g["slo_errors"].append(_rule(f"{svc.capitalize()}ErrorRateHigh", f"{err} > 0.05", "10m", "warning",
                                     f"{svc}: more than 5% of events fail"))
    for svc in ("ingestion", "reporting"):
        g["slo_errors"].append(_rule(
            f"{svc.capitalize()}APIErrorRateHigh",
            f"sum(rate({svc}_http_requests_total{{status=~'5..'}}[5m])) / "
            f"clamp_min(sum(rate({svc}_http_requests_total[5m])), 1e-9) > 0.01", "10m", "warning",
            f"{svc} API 5xx rate above 1%"))
    g["slo_errors"].append(_rule(
        "ErrorBudgetBurnRateHigh",
        "sum(rate({__name__=~'.+_events_failed_total'}[1h])) / "
        "clamp_min(sum(rate({__name__=~'.+_events_processed_total'}[1h])), 1e-9) > 0.0144", "15m", "critical",
        "error budget (99% success) burning 14.4x too fast"))
    # --- documents (pipeline exporter)
    g["document_processing"] += [
        _rule("DocumentsStuckPending", "max(copilot_document_age_seconds{status='pending'}) > 3600", "15m", "warning",
              "documents pending for over an hour"),
        _rule("DocumentsStuckProcessing", "max(copilot_document_age_seconds{status='processing'}) > 1800", "15m",
              "warning", "documents processing for over 30 minutes"),
        _rule("HighDocumentAttemptCount", "max(copilot_document_attempt_count) > 3", "15m", "warning",
              "documents needing more than 3 attempts on average"),
        _rule("FailedDocumentsAccumulating", "sum(copilot_document_status_count{status=~'failed.*'}) > 10", "30m",
              "warning", "failed documents accumulating"),
        _rule("LowEmbeddingCompletionRate",
              "sum(copilot_chunks_embedding_status_count{embedding_generated='false'}) / "
              "clamp_min(sum(copilot_chunks_embedding_status_count), 1) > 0.5", "30m", "warning",
              "more than half of the chunks have no embedding"),
    ]
    # --- failed-event queues (RabbitMQ exporter names; in-process node: copilot_queue_messages)
    for name, thr, sev in (("Warning", 10, "warning"), ("Critical", 100, "critical"), ("Emergency", 1000, "critical")):
        g["failed_queues"].append(_rule(
            f"FailedQueue{name}",
            f"max by (queue) (rabbitmq_queue_messages{{queue=~'.*failed'}} or copilot_queue_messages{{queue=~'.*failed'}}) > {thr}",
            "5m", sev, f"a *.failed queue holds more than {thr} messages"))
    g["failed_queues"].append(_rule(
        "FailedQueueStagnant", "min by (queue) (copilot_queue_messages{queue=~'.*failed'}) > 0 and "
        "delta(copilot_queue_messages{queue=~'.*failed'}[24h]) >= 0", "1h", "warning",
        "failed messages not drained for 24h"))
    # --- queue lag
    for svc, (hi, crit) in MAIN_QUEUE_DEPTH.items():
        depth = f"(rabbitmq_queue_messages{{queue='{svc}'}} or copilot_queue_messages{{queue='{svc}'}})"
        g["queue_lag"] += [_rule(f"{svc.capitalize()}QueueDepthHigh", f"max({depth}) > {hi}", "10m", "warning",
                                 f"{svc} queue deeper than {hi}"),
                           _rule(f"{svc.capitalize()}QueueDepthCritical", f"max({depth}) > {crit}", "10m", "critical",
                                 f"{svc} queue deeper than {crit}")]
    g["queue_lag"] += [
        _rule("NoQueueConsumers", "(copilot_queue_consumers == 0) and on(queue) (copilot_queue_messages > 0)", "5m",
              "critical", "messages waiting on a queue nobody consumes"),
        _rule("DeadLetterQueueGrowing", "delta(copilot_queue_messages{queue=~'.*\\\\.dlq'}[30m]) > 0", "30m", "warning",
              "dead-letter queue growing"),
        _rule("QueueGrowingRapidly", "deriv(copilot_queue_messages[10m]) > 5", "10m", "warning",
              "a queue grows by more than 5 messages/s"),
    ]
    # --- retry policy (retry/ metrics)
    g["retry_policy"] += [
        _rule("MaxRetriesExceededCritical", "sum(increase({__name__=~'.+_event_dlq_total'}[15m])) > 0", "0m",
              "critical", "events exhausted their retries and went to the DLQ"),
        _rule("HighRetryRate", "sum(rate({__name__=~'.+_event_retry_attempts_total'}[5m])) > 1", "15m", "warning",
              "more than one retry per second"),
        _rule("StartupRequeueErrors", "increase(startup_requeue_errors_total[1h]) > 0", "0m", "warning",
              "startup requeue could not republish incomplete work"),
    ]
    # --- service health
    g["service_health"] += [
        _rule("ServiceDown", "up == 0", "2m", "critical", "{{ $labels.job }} is down"),
        _rule("PipelineExporterScrapeErrors", "increase(copilot_document_exporter_scrape_errors_total[15m]) > 0", "15m",
              "warning", "the pipeline exporter cannot read the document store"),
        _rule("NoEventsProcessed",
              "sum(rate({__name__=~'.+_events_processed_total'}[30m])) == 0 and "
              "sum(copilot_queue_messages{queue!~'.*(failed|dlq)'}) > 0", "30m", "warning",
              "work is queued but no stage processes events"),
    ]
    # --- resources: MI355X HBM + host process
    g["resource_limits"] += [
        _rule("GpuHbmNearlyFull", "max by (device) (copilot_gpu_hbm_used_bytes / copilot_gpu_hbm_total_bytes) > 0.95",
              "10m", "warning", "GPU {{ $labels.device }} HBM above 95%"),
        _rule("KvCacheNearlyFull", "summarization_gpu_kv_cache_bytes / clamp_min(copilot_gpu_hbm_total_bytes, 1) > 0.9",
              "10m", "warning", "KV cache uses more than 90% of HBM"),
        _rule("DecodeStalled", "summarization_gpu_decode_tokens_per_second == 0 and "
              "on() (max(copilot_queue_messages{queue='summarization'}) > 0)", "10m", "critical",
              "summarization queued but the GPU engine decodes nothing"),
        _rule("ServiceMemoryUsageHigh", "process_resident_memory_bytes > 200e9", "10m", "warning",
              "a service process holds more than 200 GB of host memory"),
    ]
    return {k: {"groups": [{"name": k, "rules": v}]} for k, v in g.items()}


# ---------------------------------------------------------------------------- dashboards
def _panel(i: int, title: str, exprs, unit: str = "short", kind: str = "timeseries", ds: str = "prometheus") -> dict:
    exprs = [exprs] if isinstance(exprs, str) else list(exprs)
    return {"id": i, "type": kind, "title": title, "datasource": {"type": ds},
            "gridPos": {"h": 8, "w": 12, "x": 12 * (i % 2), "y": 8 * (i // 2)},
            "fieldConfig": {"defaults": {"unit": unit}, "overrides": []},
            "targets": [{"expr": e, "refId": chr(65 + j)} for j, e in enumerate(exprs)]}


def _dash(uid: str, title: str, panels: list[tuple]) -> dict:
    return {"title": title, "uid": uid, "schemaVersion": 39, "version": 1, "time": {"from": "now-6h", "to": "now"},
            "refresh": "30s", "tags": ["copilot"], "panels": [_panel(i, *p) for i, p in enumerate(panels)]}


def dashboards() -> dict[str, dict]:
    stages = BUS_SERVICES
    ev = lambda n: [f"sum(rate({s}_{n}[5m]))" for s in stages]  # noqa: E731
    return {
        "document-processing-status": _dash("cfc-docs", "Document processing status", [
            ("Documents by collection / status", "sum by (collection, status) (copilot_document_status_count)"),
            ("Collection sizes", "copilot_collection_document_count"),
            ("Oldest pending / processing (s)", "max by (collection, status) (copilot_document_age_seconds)", "s"),
            ("Average attempts", "copilot_document_attempt_count"),
            ("Chunks with / without embeddings", "copilot_chunks_embedding_status_count")]),
        "failed-queues": _dash("cfc-failed", "Failed-event queues", [
            ("Messages per failed queue", "copilot_queue_messages{queue=~'.*failed'}"),
            ("Dead-letter queues", "copilot_queue_messages{queue=~'.*\\\\.dlq'}"),
            ("RabbitMQ failed queues", "rabbitmq_queue_messages{queue=~'.*failed'}"),
            ("Events sent to DLQ / 15m", "sum by (__name__) (increase({__name__=~'.+_event_dlq_total'}[15m]))")]),
        "logs-overview": _dash("cfc-logs", "Logs overview", [
            ("Log lines by service", "sum by (service) (count_over_time({job='copilot'}[5m]))", "short", "timeseries",
             "loki"),
            ("Errors by service", "sum by (service) (count_over_time({job='copilot', level='ERROR'}[5m]))", "short",
             "timeseries", "loki"),
            ("Recent errors", "{job='copilot', level='ERROR'}", "short", "logs", "loki")]),
        "mongodb-status": _dash("cfc-mongo", "Document store", [
            ("Documents per collection", "copilot_collection_document_count"),
            ("MongoDB up", "mongodb_up", "short", "stat"),
            ("MongoDB connections", "mongodb_connections{state='current'}"),
            ("Operations / s", "sum by (type) (rate(mongodb_op_counters_total[5m]))")]),
        "pipeline-flow": _dash("cfc-flow", "Pipeline flow", [
            ("Events processed / s by stage", ev("events_processed_total")),
            ("Events failed / s by stage", ev("events_failed_total")),
            ("Events published / s by stage", ev("events_published_total")),
            ("Threads summarized / s", "sum(rate(summarization_events_processed_total[5m]))"),
            ("Messages parsed / s", "sum(rate(parsing_messages_parsed_total[5m]))"),
            ("Chunks created / embedded per s", ["sum(rate(chunking_chunks_created_total[5m]))",
                                                 "sum(rate(embedding_chunks_processed_total[5m]))"])]),
        "queue-status": _dash("cfc-queues", "Queues", [
            ("Queue depth", "copilot_queue_messages"),
            ("Consumers per queue", "copilot_queue_consumers"),
            ("RabbitMQ queue depth", "rabbitmq_queue_messages"),
            ("RabbitMQ unacked", "rabbitmq_queue_messages_unacked")]),
        "resource-usage": _dash("cfc-resources", "Resources (MI355X + host)", [
            ("HBM used per GPU", "copilot_gpu_hbm_used_bytes", "bytes"),
            ("KV cache", "summarization_gpu_kv_cache_bytes", "bytes"),
            ("Decode / prefill tokens per s", ["summarization_gpu_decode_tokens_per_second",
                                               "summarization_gpu_prefill_tokens_per_second"]),
            ("Vector index device bytes", "copilot_vectorstore_device_bytes", "bytes"),
            ("Process resident memory", "process_resident_memory_bytes", "bytes"),
            ("Process CPU", "rate(process_cpu_seconds_total[5m])")]),
        "retry-policy": _dash("cfc-retry", "Retry policy", [
            ("Retry attempts / s", "sum by (__name__) (rate({__name__=~'.+_event_retry_attempts_total'}[5m]))"),
            ("Retry successes / s", "sum by (__name__) (rate({__name__=~'.+_event_retry_success_total'}[5m]))"),
            ("Non-retryable errors / s",
             "sum by (__name__) (rate({__name__=~'.+_event_non_retryable_errors_total'}[5m]))"),
            ("Startup requeues", ["increase(startup_requeue_documents_total[1h])",
                                  "increase(startup_requeue_errors_total[1h])"])]),
        "service-metrics": _dash("cfc-services", "Service latency", [
            (f"{s} event latency p50 / p95", [_p(0.5, f"{s}_event_processing_seconds"),
                                              _p(0.95, f"{s}_event_processing_seconds")], "s")
            for s in stages] + [
            ("API latency p95", [_p(0.95, "ingestion_http_request_duration_seconds"),
                                 _p(0.95, "reporting_http_request_duration_seconds")], "s")]),
        "system-health": _dash("cfc-health", "System health", [
            ("Targets up", "up", "short", "stat"),
            ("Failed-event ratio (1h)", "sum(rate({__name__=~'.+_events_failed_total'}[1h])) / "
             "clamp_min(sum(rate({__name__=~'.+_events_processed_total'}[1h])), 1e-9)", "percentunit"),
            ("Exporter scrape errors", "copilot_document_exporter_scrape_errors_total"),
            ("API 5xx / s", "sum by (__name__) (rate({__name__=~'.+_http_requests_total', status=~'5..'}[5m]))")]),
        "vectorstore-status": _dash("cfc-vectors", "Vector store", [
            ("Vectors indexed", "copilot_vectorstore_vectors", "short", "stat"),
            ("Index bytes in HBM", "copilot_vectorstore_device_bytes", "bytes"),
            ("Chunks awaiting embedding", "copilot_chunks_embedding_status_count{embedding_generated='false'}"),
            ("Topic-search latency p95", _p(0.95, "reporting_http_request_duration_seconds"), "s")]),
    }


# ---------------------------------------------------------------------------- logs
def loki_config() -> dict:
    return {"auth_enabled": False,
            "server": {"http_listen_port": 3100},
            "common": {"path_prefix": "/loki", "replication_factor": 1, "ring": {"kvstore": {"store": "inmemory"}},
                       "storage": {"filesystem": {"chunks_directory": "/loki/chunks",
                                                  "rules_directory": "/loki/rules"}}},
            "schema_config": {"configs": [{"from": "2024-01-01", "store": "tsdb", "object_store": "filesystem",
                                           "schema": "v13", "index": {"prefix": "index_", "period": "24h"}}]},
            "limits_config": {"retention_period": "168h", "allow_structured_metadata": True},
            "compactor": {"working_directory": "/loki/compactor", "retention_enabled": True,
                          "delete_request_store": "filesystem"}}


def promtail_config() -> dict:
    """Tails the containers' stdout and lifts the JSON log fields (observability.StdoutLogger:
    ``level``, ``logger``/``service``, ``message``) into Loki labels."""
    return {"server": {"http_listen_port": 9080, "grpc_listen_port": 0},
            "positions": {"filename": "/tmp/positions.yaml"},
            "clients": [{"url": "http://loki:3100/loki/api/v1/push"}],
            "scrape_configs": [{
                "job_name": "copilot",
                "docker_sd_configs": [{"host": "unix:///var/run/docker.sock", "refresh_interval": "10s"}],
                "relabel_configs": [
                    {"source_labels": ["__meta_docker_container_name"], "regex": "/(.*)", "target_label": "container"},
                    {"target_label": "job", "replacement": "copilot"}],
                "pipeline_stages": [
                    {"json": {"expressions": {"level": "level", "service": "logger", "message": "message"}}},
                    {"labels": {"level": None, "service": None}},
                    {"output": {"source": "message"}}]}]}


# ---------------------------------------------------------------------------- Mongo
def mongo_init_js() -> str:
    cfg = collections_config()
    return "\n".join([
        "// Generated by copilot_for_consensus_amd.tools.ops_assets: collections + indexes of",
        "// contracts.documents.collections_config() (validation stays in the application's schema layer).",
        "const dbName = process.env.MONGO_APP_DB || 'copilot';",
        "const database = db.getSiblingDB(dbName);",
        f"const config = {json.dumps(cfg, indent=2)};",
        "for (const def of config.collections) {",
        "  if (!database.getCollectionNames().includes(def.name)) { database.createCollection(def.name); }",
        "  for (const spec of (def.indexes || [])) { database.getCollection(def.name).createIndex(spec.keys, spec.options || {}); }",
        "}",
        "print(`copilot collections ready in '${dbName}'`);", ""])


# ---------------------------------------------------------------------------- Kubernetes
def k8s_manifests(image: str = "copilot-for-consensus-amd:latest", namespace: str = "copilot",
                  max_replicas: int = 8, tp: int = 1) -> list[dict]:
    """Namespace, shared ConfigMap, a Deployment + Service per service (GPU stages request
    ``amd.com/gpu``), KEDA ScaledObjects on each consumer's RabbitMQ queue, and the single-node
    alternative (every stage in one pod on the in-process bus, one engine per GPU)."""
    queues = {q["name"] for q in rabbitmq_definitions()["queues"]}
    meta = lambda name, **kw: {"name": name, "namespace": namespace, **kw}  # noqa: E731
    env_cfg = {"MESSAGE_BUS_TYPE": "rabbitmq", "RABBITMQ_HOST": "messagebus", "DOCUMENT_STORE_TYPE": "mongodb",
               "MONGODB_HOST": "documentdb", "METRICS_TYPE": "prometheus", "LOG_TYPE": "stdout",
               "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    out: list[dict] = [
        {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": namespace}},
        {"apiVersion": "v1", "kind": "ConfigMap", "metadata": meta("copilot-env"), "data": env_cfg},
    ]

    def container(name, args, port, gpus=0):
        c = {"name": name, "image": image, "command": ["python", "-m", "copilot_for_consensus_amd.services.main"],
             "args": args, "ports": [{"containerPort": port}], "envFrom": [{"configMapRef": {"name": "copilot-env"}}],
             "readinessProbe": {"httpGet": {"path": "/readyz", "port": port}, "periodSeconds": 10},
             "livenessProbe": {"httpGet": {"path": "/health", "port": port}, "periodSeconds": 30}}
        if gpus:
            c["resources"] = {"limits": {"amd.com/gpu": gpus}}
            c["volumeMounts"] = [{"name": "dshm", "mountPath": "/dev/shm"}]
        return c

    def deployment(name, cont, replicas=1):
        spec = {"containers": [cont]}
        if "resources" in cont:
            spec["volumes"] = [{"name": "dshm", "emptyDir": {"medium": "Memory"}}]
            spec["nodeSelector"] = {"amd.com/gpu.product-name": "AMD_Instinct_MI355X"}
        return {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": meta(name, labels={"app": name}),
                "spec": {"replicas": replicas, "selector": {"matchLabels": {"app": name}},
                         "template": {"metadata": {"labels": {"app": name}}, "spec": spec}}}

    for svc, port in SERVICE_PORTS.items():
        gpus = GPU_SERVICES.get(svc, 0) * (tp if svc == "summarization" else 1)
        out.append(deployment(svc, container(svc, [svc, "--port", str(port)], port, gpus)))
        out.append({"apiVersion": "v1", "kind": "Service", "metadata": meta(svc),
                    "spec": {"selector": {"app": svc}, "ports": [{"port": port, "targetPort": port}]}})
        if svc in BUS_SERVICES and svc in queues:
            out.append({"apiVersion": "keda.sh/v1alpha1", "kind": "ScaledObject", "metadata": meta(f"{svc}-scaler"),
                        "spec": {"scaleTargetRef": {"name": svc}, "minReplicaCount": 1,
                                 "maxReplicaCount": max_replicas if svc in GPU_SERVICES else 2 * max_replicas,
                                 "triggers": [{"type": "rabbitmq", "metadata": {
                                     "queueName": svc, "mode": "QueueLength", "value": "5",
                                     "hostFromEnv": "RABBITMQ_URL"}}]}})
    node = container("node", ["node", "--port", "8080"], 8080, gpus=8)
    node["env"] = [{"name": "MESSAGE_BUS_TYPE", "value": "inproc"}, {"name": "DOCUMENT_STORE_TYPE", "value": "mongodb"}]
    nd = deployment("node", node, replicas=0)
    nd["metadata"]["annotations"] = {"copilot/mode": "single-node alternative: scale to 1 instead of the per-service "
                                                     "deployments"}
    out.append(nd)
    return out


def k8s_yaml(**kw) -> str:
    return "---\n".join(yaml.safe_dump(m, sort_keys=False) for m in k8s_manifests(**kw))


def metric_names(expr: str) -> set[str]:
    """Metric identifiers referenced by a PromQL expression (used by the tests to check every alert
    and panel reads a metric this framework or a standard exporter emits)."""
    body = re.sub(r"'[^']*'|\"[^\"]*\"|\{[^}]*\}|\[[^\]]*\]", " ", expr)
    body = re.sub(r"(?<![A-Za-z0-9_])\d+(\.\d+)?([eE][-+]?\d+)?", " ", body)    # numeric literals (1e-9, 200e9)
    words = set(re.findall(r"[a-zA-Z_:][a-zA-Z0-9_:]*", body))
    funcs = {"histogram_quantile", "sum", "rate", "by", "le", "max", "min", "clamp_min", "increase", "delta", "deriv",
             "and", "or", "on", "count_over_time", "e9", "queue", "collection", "status", "device", "type", "job",
             "service", "__name__", "labels", "bool"}
    return {w for w in words if w not in funcs and not w[0].isdigit()}
