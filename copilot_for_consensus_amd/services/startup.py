"""Forward progress after a crash/restart: republish work for documents left incomplete.

Parity target: adapters/copilot_startup/copilot_startup/startup_requeue.py (StartupRequeue :19,
``requeue_incomplete(collection, query, event_type, routing_key, id_field, build_event_data, limit)``
:44, ``publish_event`` helper, metrics ``startup_requeue_documents_total`` /
``startup_requeue_errors_total``).  The services' own ``requeue_incomplete`` hooks
(services/processing.py) group documents into batched events; this class is the generic
per-document form the reference exposes, usable by scripts and custom services.

Reference: adapters/copilot_startup/copilot_startup/startup_requeue.py:19-44 (StartupRequeue).
"""
from __future__ import annotations

from typing import Any, Callable

from ..contracts.events import Event
from ..observability import get_logger

EXCHANGE = "copilot.events"


class StartupRequeue:
    def __init__(self, document_store, publisher, metrics_collector=None, logger=None):
        self.document_store = document_store
        self.publisher = publisher
        self.metrics_collector = metrics_collector
        self.log = logger or get_logger("startup")

    def _event(self, event_type: str, data: dict[str, Any]) -> dict:
        return Event.create(event_type, **data).to_dict()

    def publish_event(self, event_type: str, routing_key: str, event_data: dict[str, Any]) -> None:
        self.publisher.publish(EXCHANGE, routing_key, self._event(event_type, event_data))

    def requeue_incomplete(self, collection: str, query: dict[str, Any], event_type: str, routing_key: str,
                           id_field: str, build_event_data: Callable[[dict], dict], limit: int = 1000) -> int:
        try:
            docs = self.document_store.query_documents(collection, query, limit=limit)
        except Exception as e:
            if self.metrics_collector:
                self.metrics_collector.increment("startup_requeue_errors_total", 1,
                                                 tags={"collection": collection, "error_type": type(e).__name__})
            self.log.error("startup requeue query failed", collection=collection, error=repr(e))
            raise
        done = 0
        for d in docs:
            try:
                self.publish_event(event_type, routing_key, build_event_data(d))
                done += 1
            except Exception as e:  # one bad document must not block the rest
                self.log.error("requeue failed", collection=collection, id=d.get(id_field, "unknown"), error=repr(e))
        if self.metrics_collector and done:
            self.metrics_collector.increment("startup_requeue_documents_total", done, tags={"collection": collection})
        self.log.info("startup requeue", collection=collection, found=len(docs), requeued=done)
        return done
