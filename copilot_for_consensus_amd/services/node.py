"""Service assembly: build any service from typed config, or a whole single-node deployment.

``build_service(name, cfg, ...)`` wires a service from ``get_config(name)`` exactly like the
reference mains (e.g. parsing/main.py:152-318): adapters from their discriminant env vars, the
validating bus decorators, JWT middleware.  :class:`Node` runs every stage in ONE process on the
in-process broker (the MI355X single-node deployment: one node, one bus, GPU models loaded once),
with one consumer thread per service -- the compose topology of the reference without its
network hops.  ``python -m copilot_for_consensus_amd.services.main <service>`` runs one service
per process (uvicorn + consumer thread) for a distributed deployment.
"""
from __future__ import annotations

import threading

from ..archive import create_archive_store
from ..bus import InProcBroker, create_publisher, create_subscriber
from ..chunking import create_chunker
from ..config.loader import env_is_set, get_config
from ..consensus import create_consensus_detector
from ..embedding import create_embedding_provider
from ..observability import create_error_reporter, create_logger, create_metrics_collector
from ..retry import RetryConfig
from ..storage.document_store import create_document_store
from ..summarization import create_llm_backend
from ..vectorstore import create_vector_store
from .base import own_gpu_stream
from .ingestion import IngestionService
from .processing import ChunkingService, EmbeddingService, OrchestratorService, ParsingService, SummarizationService
from .reporting import ReportingService


class Node:
    """All pipeline services in one process, sharing the broker, stores and GPU models."""

    # adapters each service needs (so a one-service process builds only its own: the summarization
    # process alone loads the LLM, only embedding / reporting load the encoder)
    NEEDS = {"ingestion": {"archives"}, "parsing": {"archives"}, "chunking": set(),
             "embedding": {"embedder", "vectors"}, "orchestrator": {"vectors"}, "summarization": {"summarizer"},
             "reporting": {"embedder", "vectors"}}

    def __init__(self, env: dict | None = None, broker: InProcBroker | None = None, document_store=None,
                 archive_store=None, embedding_provider=None, vector_store=None, summarizer=None,
                 retry_config: RetryConfig | None = None, services=None):
        names = [s for s in self.NEEDS if services is None or s in services]
        need = set().union(*(self.NEEDS[s] for s in names))
        self.broker = broker or InProcBroker()
        cfgs = {s: get_config(s, env=env) for s in names}
        self.cfgs = cfgs
        c0 = cfgs[names[0]]
        self.store = document_store or create_document_store(c0.document_store)
        self.archives = archive_store or (create_archive_store(cfgs.get("ingestion", c0).archive_store)
                                          if "archives" in need else None)
        self.metrics = create_metrics_collector(c0.metrics)
        self.logger = create_logger(c0.logger)
        self.errors = create_error_reporter(c0.error_reporter)
        ecfg = cfgs.get("embedding", c0)
        self.embedder = embedding_provider or (create_embedding_provider(ecfg.embedding_backend)
                                               if "embedder" in need else None)
        if vector_store is not None or "vectors" not in need:
            self.vectors = vector_store
        else:
            dim = int(self.embedder.dimension) if self.embedder is not None else \
                int(ecfg.vector_store.driver_config.get("dimension") or
                    ecfg.vector_store.driver_config.get("vector_size") or 384)
            self.vectors = create_vector_store(ecfg.vector_store, dimension=dim)
        # a DP-sharded index (parallel/dp_node.py) reads chunk texts from this node's store by id
        attach = getattr(self.vectors, "attach_document_store", None)
        if callable(attach):
            attach(self.store)
        self.summarizer = summarizer or (create_llm_backend(cfgs["summarization"].llm_backend)
                                         if "summarizer" in need else None)
        rcfg = next((c.event_retry for c in cfgs.values() if hasattr(c, "event_retry")), None)
        retry = retry_config or (RetryConfig.from_adapter(rcfg) if rcfg is not None else RetryConfig())
        common = dict(metrics=self.metrics, logger=self.logger, error_reporter=self.errors, retry_config=retry)

        def pub(name):
            return create_publisher(cfgs[name].message_bus, broker=self.broker)

        def sub(name):
            return create_subscriber(cfgs[name].message_bus, broker=self.broker, queue_name=name)

        build = {
            "ingestion": lambda: IngestionService(
                pub("ingestion"), self.store, self.archives,
                storage_path=cfgs["ingestion"].storage_path if env_is_set("INGESTION_STORAGE_PATH", env) else None,
                max_retries=cfgs["ingestion"].max_retries, **common),
            "parsing": lambda: ParsingService(pub("parsing"), sub("parsing"), self.store, self.archives, **common),
            "chunking": lambda: ChunkingService(pub("chunking"), sub("chunking"), self.store,
                                                create_chunker(cfgs["chunking"].chunker), **common),
            "embedding": lambda: EmbeddingService(pub("embedding"), sub("embedding"), self.store, self.embedder,
                                                  self.vectors, max_retries=cfgs["embedding"].max_retries,
                                                  retry_backoff_seconds=0.1, **common),
            "orchestrator": lambda: OrchestratorService(
                pub("orchestrator"), sub("orchestrator"), self.store, self.vectors, top_k=cfgs["orchestrator"].top_k,
                context_window_tokens=cfgs["orchestrator"].context_window_tokens,
                chunk_selection_strategy=cfgs["orchestrator"].chunk_selection_strategy,
                system_prompt_path=cfgs["orchestrator"].system_prompt_path,
                user_prompt_path=cfgs["orchestrator"].user_prompt_path,
                consensus_detector=create_consensus_detector(cfgs["orchestrator"].consensus_detector), **common),
            "summarization": lambda: SummarizationService(
                pub("summarization"), sub("summarization"), self.store, self.summarizer,
                citation_count=cfgs["summarization"].citation_count,
                context_window_tokens=cfgs["summarization"].context_window_tokens,
                max_batch_threads=cfgs["summarization"].max_batch_threads,
                batch_wait_ms=cfgs["summarization"].batch_wait_ms, retry_delay_seconds=0.1,
                continuous=cfgs["summarization"].continuous_batching,
                min_admit=cfgs["summarization"].min_admit, admit_wait_ms=cfgs["summarization"].admit_wait_ms,
                **common),
            "reporting": lambda: ReportingService(
                pub("reporting"), sub("reporting"), self.store, self.vectors, self.embedder,
                notify_enabled=cfgs["reporting"].notify_enabled,
                notify_webhook_url=cfgs["reporting"].notify_webhook_url, **common),
        }
        self.services = {n: build[n]() for n in names}
        self._threads: list[threading.Thread] = []
        self._connected = False

    def connect(self, services=None) -> None:
        """Connect the document store and every (or the named) service's publisher / subscriber.
        Raises on the first failure -- the entry point turns that into exit code 1, the reference's
        fail-fast start-up (parsing/tests/test_startup_validation.py:115-165)."""
        if self._connected:
            return
        self.store.connect()
        for name, svc in self.services.items():
            if services is not None and name not in services:
                continue
            for end in (svc.publisher, svc.subscriber):
                if end is not None and hasattr(end, "connect"):
                    end.connect()
        self._connected = True

    def start(self, threaded: bool = True) -> None:
        self.connect()
        for s in self.services.values():
            s.start()
            if threaded and hasattr(s, "start_async"):
                s.start_async()        # the summarizer's continuous engine / micro-batcher
        if threaded:
            self.start_scheduler()
        if threaded:
            for name, s in self.services.items():
                if s.subscriber is not None:
                    def consume(sub=s.subscriber):
                        own_gpu_stream()
                        sub.start_consuming()
                    t = threading.Thread(target=consume, name=f"{name}-consumer", daemon=True)
                    s.consumer_thread = t
                    t.start()
                    self._threads.append(t)

    def start_scheduler(self) -> bool:
        """Periodic ingestion of every enabled source (reference ingestion/main.py:374-385), in the
        node and in a standalone ``main ingestion`` process alike; INGESTION_SCHEDULE_INTERVAL_SECONDS
        <= 0 turns it off.  Returns whether a scheduler is running."""
        ing = self.services.get("ingestion")
        if ing is None:
            return False
        from .ingestion import IngestionScheduler
        interval = self.cfgs["ingestion"].schedule_interval_seconds
        if interval and interval > 0 and getattr(ing, "scheduler", None) is None:
            ing.scheduler = IngestionScheduler(ing, interval_seconds=interval)
            ing.scheduler.start()
        return getattr(ing, "scheduler", None) is not None and ing.scheduler.is_running

    def stop(self) -> None:
        ing = self.services.get("ingestion")
        if ing is not None and getattr(ing, "scheduler", None) is not None:
            ing.scheduler.stop()
        for s in self.services.values():
            if s.subscriber is not None:
                s.subscriber.stop_consuming()
        for t in self._threads:
            t.join(timeout=5)
        for s in self.services.values():
            if hasattr(s, "stop_async"):
                s.stop_async()

    def http_app(self, auth_base: str = "/auth"):
        """The all-in-one HTTP front in the gateway's layout (deploy/gateway/nginx.conf):
        ``/reporting/...`` and ``/ingestion/...`` are the two services' APIs (both define
        ``/api/sources`` -- thread-source names vs the ingestion source records -- so they cannot
        share one path space), ``/ui`` the web UI wired to those prefixes.  The reporting API also
        answers at the root for clients of a single reporting service."""
        from ..ui import ui_routes
        from .base import create_app
        from .ingestion import ingestion_routes
        from .reporting import reporting_routes
        root = create_app(self.services["reporting"], extra_routes=reporting_routes)
        root.mount("/reporting", create_app(self.services["reporting"], extra_routes=reporting_routes))
        if "ingestion" in self.services:
            root.mount("/ingestion", create_app(self.services["ingestion"], extra_routes=ingestion_routes))
        ui_routes(root, bases={"reporting": "/reporting", "ingestion": "/ingestion", "auth": auth_base})
        return root

    def drain(self, max_rounds: int = 1000) -> int:
        """Synchronous mode: process queued events stage by stage until the bus is quiet."""
        total = 0
        for _ in range(max_rounds):
            n = 0
            for s in self.services.values():
                if s.subscriber is not None:
                    n += s.subscriber.drain()
            total += n
            if n == 0:
                break
        return total
