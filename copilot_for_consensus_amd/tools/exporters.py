"""Prometheus exporters for pipeline state.

Parity target: scripts/document_processing_exporter.py (copilot_document_status_count,
..._processing_duration_seconds, ..._age_seconds, ..._attempt_count, chunks embedding status,
scrape errors), mongo_doc_count_exporter.py / mongo_collstats_exporter.py (per-collection counts)
and qdrant_exporter.py (vector counts) of the reference.  One collector reads any DocumentStore
and VectorStore (in-proc or Mongo) -- plus the GPU-resident index's HBM footprint -- and renders
the Prometheus text format; ``serve`` exposes it on /metrics (stdlib http.server).

Reference: scripts/document_processing_exporter.py:37-67 (gauges), mongo_doc_count_exporter.py,
qdrant_exporter.py.
"""
from __future__ import annotations

import argparse
import collections
import sys
import threading
import time
from datetime import datetime, timezone
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

COLLECTIONS = ("archives", "messages", "threads", "chunks", "summaries", "sources")


def _ts(v):
    if v is None:
        return None
    if isinstance(v, datetime):
        return v if v.tzinfo else v.replace(tzinfo=timezone.utc)
    try:
        t = datetime.fromisoformat(str(v).replace("Z", "+00:00"))
        return t if t.tzinfo else t.replace(tzinfo=timezone.utc)
    except ValueError:
        return None


def _fmt(name, labels: dict, value) -> str:
    lab = ",".join(f'{k}="{str(v).replace(chr(34), chr(39))}"' for k, v in sorted(labels.items()))
    return f"{name}{{{lab}}} {float(value)}" if lab else f"{name} {float(value)}"


class PipelineExporter:
    def __init__(self, store, vector_store=None, database: str = "copilot", broker=None, gpus: bool = False):
        self.store, self.vectors, self.db = store, vector_store, database
        self.broker = broker          # in-process broker: queue depth / consumer gauges
        self.gpus = gpus              # per-device HBM gauges (torch.cuda.mem_get_info)
        self.scrape_errors = 0

    def collect(self) -> list[str]:
        out = []
        now = datetime.now(timezone.utc)
        for coll in COLLECTIONS:
            try:
                docs = self.store.query_documents(coll, {}, limit=1 << 30)
            except Exception:
                self.scrape_errors += 1
                continue
            out.append(_fmt("copilot_collection_document_count", {"database": self.db, "collection": coll}, len(docs)))
            by_status = collections.Counter(d.get("status", "none") for d in docs)
            for st, n in by_status.items():
                out.append(_fmt("copilot_document_status_count", {"database": self.db, "collection": coll,
                                                                  "status": st}, n))
            ages = collections.defaultdict(float)
            for d in docs:
                t = _ts(d.get("lastAttemptTime") or d.get("updated_at") or d.get("created_at"))
                if t is not None and d.get("status") in ("pending", "processing"):
                    ages[d["status"]] = max(ages[d["status"]], (now - t).total_seconds())
            for st, a in ages.items():
                out.append(_fmt("copilot_document_age_seconds", {"database": self.db, "collection": coll,
                                                                 "status": st}, a))
            att = [int(d.get("attemptCount", 0)) for d in docs if "attemptCount" in d]
            if att:
                out.append(_fmt("copilot_document_attempt_count", {"database": self.db, "collection": coll},
                                sum(att) / len(att)))
            if coll == "chunks":
                emb = collections.Counter(bool(d.get("embedding_generated")) for d in docs)
                for k in (True, False):
                    out.append(_fmt("copilot_chunks_embedding_status_count",
                                    {"database": self.db, "embedding_generated": str(k).lower()}, emb.get(k, 0)))
        if self.vectors is not None:
            try:
                out.append(_fmt("copilot_vectorstore_vectors", {}, self.vectors.count()))
                X = getattr(self.vectors, "_X", None)
                if X is not None:
                    out.append(_fmt("copilot_vectorstore_device_bytes", {"device": str(X.device)},
                                    X.numel() * X.element_size()))
            except Exception:
                self.scrape_errors += 1
        if self.broker is not None:
            try:
                consumers = self.broker.consumer_counts()
                for q, depth in sorted(self.broker.queues().items()):
                    out.append(_fmt("copilot_queue_messages", {"queue": q}, depth))
                    out.append(_fmt("copilot_queue_consumers", {"queue": q}, consumers.get(q, 0)))
                details = getattr(self.broker, "queue_details", None)
                for q, v in sorted((details() if details else {}).items()):   # native broker counters
                    out.append(_fmt("copilot_queue_messages_unacked", {"queue": q}, v["unacked"]))
                    out.append(_fmt("copilot_queue_dead_lettered_total", {"queue": q}, v["dead_lettered"]))
                    out.append(_fmt("copilot_queue_redelivered_total", {"queue": q}, v["redelivered"]))
            except Exception:
                self.scrape_errors += 1
        if self.gpus:
            try:
                import torch
                for i in range(torch.cuda.device_count()):
                    free, total = torch.cuda.mem_get_info(i)
                    out.append(_fmt("copilot_gpu_hbm_used_bytes", {"device": i}, total - free))
                    out.append(_fmt("copilot_gpu_hbm_total_bytes", {"device": i}, total))
            except Exception:
                self.scrape_errors += 1
        out.append(_fmt("copilot_document_exporter_scrape_errors_total", {}, self.scrape_errors))
        return out

    def render(self) -> str:
        return "\n".join(self.collect()) + "\n"

    def serve(self, port: int = 9502, host: str = "0.0.0.0") -> ThreadingHTTPServer:
        exporter = self

        class H(BaseHTTPRequestHandler):
            def do_GET(self):
                if self.path.rstrip("/") not in ("/metrics", ""):
                    self.send_response(404)
                    self.end_headers()
                    return
                body = exporter.render().encode()
                self.send_response(200)
                self.send_header("Content-Type", "text/plain; version=0.0.4")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *a):
                pass

        srv = ThreadingHTTPServer((host, port), H)
        threading.Thread(target=srv.serve_forever, daemon=True).start()
        return srv


def main(argv=None) -> int:
    from ..config.loader import load_adapter_config
    from ..storage.document_store import create_document_store
    ap = argparse.ArgumentParser(description="Pipeline document-state Prometheus exporter")
    ap.add_argument("--port", type=int, default=9502)
    a = ap.parse_args(argv)
    bus = load_adapter_config("message_bus")
    broker = None
    if bus.driver_name == "cfcbroker":
        from ..bus.cfcbroker import CfcBrokerMonitor
        broker = CfcBrokerMonitor(bus.driver_config["broker_host"], bus.driver_config["broker_port"])
    store = create_document_store(load_adapter_config("document_store"))
    store.connect()
    PipelineExporter(store, broker=broker).serve(a.port)
    while True:
        time.sleep(3600)


if __name__ == "__main__":
    sys.exit(main())
