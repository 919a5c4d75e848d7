"""Shared service scaffolding.

Every bus-driven service of the reference has the same process model: build adapters
from typed config, start a non-daemon consumer thread (``service.start()`` + blocking
``subscriber.start_consuming()``), run uvicorn on the main thread with ``/health``, ``/readyz``,
``/stats`` and ``/.well-known/configuration-schema`` (e.g. parsing/main.py:101-145,303-318).
:class:`BaseService` + :func:`create_app` + :func:`run_service` provide exactly that, with
handlers wrapped in the event-retry policy and every stage instrumented with the reference's
metric names.
"""
from __future__ import annotations

import threading
import time
from typing import Any, Callable

from ..bus import EventPublisher, EventSubscriber
from ..contracts.events import EXCHANGE, Event
from ..observability import ErrorReporter, Logger, MetricsCollector, NoOpMetricsCollector, SilentErrorReporter
from ..observability import SilentLogger
from ..retry import RetryConfig, RetryExhaustedError, handle_event_with_retry


class BaseService:
    name = "service"

    def __init__(self, publisher: EventPublisher, subscriber: EventSubscriber | None, document_store,
                 metrics: MetricsCollector | None = None, logger: Logger | None = None,
                 error_reporter: ErrorReporter | None = None, retry_config: RetryConfig | None = None):
        self.publisher = publisher
        self.subscriber = subscriber
        self.store = document_store
        self.metrics = metrics or NoOpMetricsCollector()
        self.log = logger or SilentLogger()
        self.errors = error_reporter or SilentErrorReporter()
        self.retry_config = retry_config or RetryConfig()
        self.stats: dict[str, Any] = {"events_processed": 0, "events_failed": 0, "started_at": None,
                                      "last_event_at": None}
        self._ready = threading.Event()
        self._lock = threading.Lock()
        self.consumer_thread: threading.Thread | None = None   # set by whoever runs the consume loop

    # ---------------------------------------------------------------- events
    def publish(self, event_type: str, **data) -> dict:
        ev = Event.create(event_type, **data).to_dict()
        self.publisher.publish(EXCHANGE, Event(event_type).routing_key, ev)
        self.metrics.increment(f"{self.name}_events_published_total", tags={"event_type": event_type})
        return ev

    def subscriptions(self) -> dict[str, Callable[[dict], None]]:
        """event_type -> handler(event dict); override."""
        return {}

    def _wrap(self, event_type: str, fn: Callable[[dict], None]) -> Callable[[dict], None]:
        def handler(event: dict) -> None:
            t = time.perf_counter()
            try:
                handle_event_with_retry(fn, event, self.retry_config,
                                        idempotency_key=f"{self.name}-{event.get('event_id')}",
                                        metrics_collector=self.metrics, error_reporter=self.errors,
                                        service_name=self.name)
                with self._lock:
                    self.stats["events_processed"] += 1
                    self.stats["last_event_at"] = time.time()
                self.metrics.increment(f"{self.name}_events_processed_total", tags={"event_type": event_type})
            except RetryExhaustedError as e:
                with self._lock:
                    self.stats["events_failed"] += 1
                self.metrics.increment(f"{self.name}_events_failed_total", tags={"event_type": event_type})
                self.log.error("retry exhausted", event_type=event_type, error=str(e))
                self.on_failure(event_type, event, e)
            except Exception as e:
                with self._lock:
                    self.stats["events_failed"] += 1
                self.metrics.increment(f"{self.name}_events_failed_total", tags={"event_type": event_type})
                self.log.error("handler failed", event_type=event_type, error=repr(e))
                self.on_failure(event_type, event, e)
                raise
            finally:
                self.metrics.observe(f"{self.name}_event_processing_seconds", time.perf_counter() - t,
                                     tags={"event_type": event_type})
                self.metrics.safe_push()
        return handler

    def on_failure(self, event_type: str, event: dict, error: Exception) -> None:
        """Publish the stage's *Failed event; override."""

    def requeue_incomplete(self) -> int:
        """Startup forward-progress hook (copilot_startup); override."""
        return 0

    def start(self) -> None:
        if self.subscriber is not None:
            for et, fn in self.subscriptions().items():
                self.subscriber.subscribe(et, self._wrap(et, fn))
        self.stats["started_at"] = time.time()
        try:
            n = self.requeue_incomplete()
            if n:
                self.log.info("requeued incomplete work on startup", count=n)
        except Exception as e:  # startup requeue is best effort (reference startup_requeue.py)
            self.log.warning("startup requeue failed", error=repr(e))
        self._ready.set()

    def is_ready(self) -> bool:
        return self._ready.is_set()

    def consumer_alive(self) -> bool | None:
        """None when no consume thread was started (synchronous / drain mode), else its liveness."""
        return None if self.consumer_thread is None else self.consumer_thread.is_alive()

    def get_stats(self) -> dict:
        with self._lock:
            return dict(self.stats)


def own_gpu_stream() -> None:
    """Give the calling thread its own HIP stream (PyTorch's current stream is per thread): the
    services of one node share the GPU, and on the default stream every service's kernels (an
    embedding batch, the orchestrator's scoring) would queue behind the LLM's decode bursts."""
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.set_stream(torch.cuda.Stream())
    except (ImportError, RuntimeError):
        pass


def create_app(service: BaseService, extra_routes: Callable | None = None, config_schema: dict | None = None,
               auth_dependency=None):
    """FastAPI app with the health/readiness/stats/config-schema routes every service exposes."""
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import PlainTextResponse

    app = FastAPI(title=f"copilot-for-consensus {service.name}")

    @app.middleware("http")
    async def _request_metrics(request, call_next):
        # per-route latency + status counts (the API latency / error-rate SLO alerts read these)
        t = time.perf_counter()
        status = 500
        try:
            resp = await call_next(request)
            status = resp.status_code
            return resp
        finally:
            route = getattr(request.scope.get("route"), "path", "unmatched")
            tags = {"method": request.method, "route": route}
            service.metrics.observe(f"{service.name}_http_request_duration_seconds", time.perf_counter() - t, tags=tags)
            service.metrics.increment(f"{service.name}_http_requests_total", tags={**tags, "status": str(status)})

    @app.get("/health")
    def health():
        # a bus-driven service whose consumer thread died is unhealthy (reference reporting/main.py:79-103)
        alive = service.consumer_alive()
        out = {"status": "unhealthy" if alive is False else "healthy", "service": service.name,
               "events_processed": service.stats["events_processed"], "subscriber_thread_alive": alive}
        sched = getattr(service, "scheduler", None)
        if service.name == "ingestion":   # reference ingestion/main.py health(): scheduler + source counts
            srcs = service.list_sources()
            out.update(scheduler_running=bool(sched and sched.is_running), sources_configured=len(srcs),
                       sources_enabled=sum(1 for x in srcs if x.get("enabled", True)),
                       total_files_ingested=service.stats.get("files_ingested", 0))
        return out

    @app.get("/readyz")
    def readyz():
        if not service.is_ready():
            raise HTTPException(503, "Service not initialized")
        if service.consumer_alive() is False:
            raise HTTPException(503, "Subscriber thread not running")
        return {"status": "ready", "service": service.name}

    @app.get("/stats")
    def stats():
        return service.get_stats()

    @app.get("/.well-known/configuration-schema")
    def cfg_schema():
        if config_schema is None:
            from ..config.loader import config_json_schema
            return config_json_schema(service.name)
        return config_schema

    @app.get("/metrics", response_class=PlainTextResponse)
    def metrics():
        render = getattr(service.metrics, "render", None)
        return render() if render else ""

    if extra_routes is not None:
        extra_routes(app, service, auth_dependency)
    return app


def run_service(service: BaseService, app, host: str = "0.0.0.0", port: int = 8000) -> None:
    """Consumer thread (non-daemon) + uvicorn on the main thread (reference main.py pattern)."""
    import uvicorn

    from ..observability import uvicorn_log_config

    def consume():
        service.start()
        if hasattr(service, "start_async"):
            service.start_async()
        if service.subscriber is not None:
            service.subscriber.start_consuming()

    t = threading.Thread(target=consume, name=f"{service.name}-consumer", daemon=False)
    if service.subscriber is not None:
        service.consumer_thread = t
    t.start()
    try:
        uvicorn.run(app, host=host, port=port, log_config=uvicorn_log_config())
    finally:
        if service.subscriber is not None:
            service.subscriber.stop_consuming()
        t.join(timeout=10)
        if hasattr(service, "stop_async"):
            service.stop_async()
