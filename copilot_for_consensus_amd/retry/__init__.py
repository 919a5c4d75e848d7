"""In-handler event retry (API of adapters/copilot_event_retry: handle_event_with_retry
event_handler.py:48, RetryConfig / RetryPolicy retry_policy.py:14,78).

Exponential backoff with full jitter (delay(n) = U[0, min(base * factor^(n-1), cap)] for the
n-th attempt, first attempt immediate), TTL abandonment, retry only on :class:`RetryableError`
(including :class:`DocumentNotFoundError`: the eventual-consistency race where an event arrives
before its document is queryable), DLQ diagnostics on exhaustion, metric names
``<service>_event_retry_*`` / ``<service>_event_dlq_total`` as in the reference.
"""
from __future__ import annotations

import dataclasses
import logging
import random
import time
from datetime import datetime, timezone
from typing import Any, Callable

log = logging.getLogger(__name__)


class RetryableError(Exception):
    """A transient failure: retry with backoff."""


class DocumentNotFoundError(RetryableError):
    """The document an event refers to is not (yet) visible."""


@dataclasses.dataclass
class RetryConfig:
    max_attempts: int = 8
    base_delay_ms: int = 250
    backoff_factor: float = 2.0
    max_delay_ms: int = 60000
    ttl_seconds: int = 1800
    use_jitter: bool = True

    @classmethod
    def from_adapter(cls, cfg) -> "RetryConfig":
        if cfg is None:
            return cls()
        d = getattr(cfg, "driver_config", cfg) or {}
        kw = {k: v for k, v in d.items() if k in {f.name for f in dataclasses.fields(cls)} and v is not None}
        return cls(**kw)


@dataclasses.dataclass
class RetryContext:
    attempt_number: int = 1
    start_time: datetime = dataclasses.field(default_factory=lambda: datetime.now(timezone.utc))
    last_exception: Exception | None = None
    idempotency_key: str | None = None
    metadata: dict[str, Any] = dataclasses.field(default_factory=dict)

    def elapsed_seconds(self) -> float:
        return (datetime.now(timezone.utc) - self.start_time).total_seconds()


# one jitter RNG for every policy: a policy is built per handled event, and random.Random() seeds
# itself from os.urandom each time (thousands of events per batch in the node)
_JITTER_RNG = random.Random()


class RetryPolicy:
    def __init__(self, config: RetryConfig | None = None, sleeper: Callable[[float], None] = time.sleep,
                 rng: random.Random | None = None):
        self.config = config or RetryConfig()
        self._sleep = sleeper
        self._rng = rng or _JITTER_RNG

    def calculate_delay_ms(self, attempt_number: int) -> int:
        if attempt_number <= 1:
            return 0
        cap = min(int(self.config.base_delay_ms * self.config.backoff_factor ** (attempt_number - 1)),
                  self.config.max_delay_ms)
        return self._rng.randint(0, cap) if self.config.use_jitter else cap

    def should_retry(self, ctx: RetryContext, exc: Exception) -> bool:
        if not isinstance(exc, RetryableError):
            return False
        if ctx.attempt_number >= self.config.max_attempts:
            return False
        return ctx.elapsed_seconds() < self.config.ttl_seconds

    def sleep(self, delay_ms: int) -> None:
        if delay_ms > 0:
            self._sleep(delay_ms / 1000.0)


class RetryExhaustedError(Exception):
    def __init__(self, message: str, context: RetryContext, dlq_info: dict):
        super().__init__(message)
        self.context = context
        self.dlq_info = dlq_info


def _dlq_info(event, ctx, cfg) -> dict:
    return {"event_id": event.get("event_id"), "event_type": event.get("event_type"),
            "attempts": ctx.attempt_number, "elapsed_seconds": round(ctx.elapsed_seconds(), 3),
            "idempotency_key": ctx.idempotency_key,
            "last_error": repr(ctx.last_exception), "last_error_type": type(ctx.last_exception).__name__,
            "max_attempts": cfg.max_attempts, "ttl_seconds": cfg.ttl_seconds, **ctx.metadata}


def handle_event_with_retry(handler: Callable[[dict], Any], event: dict, config: RetryConfig | None = None,
                            idempotency_key: str | None = None, metrics_collector=None, error_reporter=None,
                            service_name: str = "unknown", policy: RetryPolicy | None = None) -> None:
    policy = policy or RetryPolicy(config)
    ctx = RetryContext(idempotency_key=idempotency_key,
                       metadata={"service": service_name, "event_type_name": event.get("event_type")})
    et = event.get("event_type", "unknown")
    while True:
        try:
            if metrics_collector:
                metrics_collector.increment(f"{service_name}_event_retry_attempts_total",
                                            tags={"attempt": str(ctx.attempt_number), "event_type": et})
            handler(event)
            if metrics_collector:
                metrics_collector.increment(f"{service_name}_event_retry_success_total",
                                            tags={"attempts": str(ctx.attempt_number), "event_type": et})
                metrics_collector.observe(f"{service_name}_event_retry_latency_ms", ctx.elapsed_seconds() * 1000,
                                          tags={"event_type": et})
            return
        except RetryableError as e:
            ctx.last_exception = e
            if not policy.should_retry(ctx, e):
                info = _dlq_info(event, ctx, policy.config)
                if metrics_collector:
                    metrics_collector.increment(f"{service_name}_event_dlq_total",
                                                tags={"reason": type(e).__name__, "event_type": et})
                if error_reporter:
                    error_reporter.report(e, context=info)
                raise RetryExhaustedError(f"Retry exhausted after {ctx.attempt_number} attempts", ctx, info) from e
            delay = policy.calculate_delay_ms(ctx.attempt_number + 1)
            log.warning("retryable error on attempt %d, retrying in %d ms: %s", ctx.attempt_number, delay, e)
            if metrics_collector:
                metrics_collector.increment(f"{service_name}_event_retry_count_total",
                                            tags={"reason": type(e).__name__, "event_type": et})
            policy.sleep(delay)
            ctx.attempt_number += 1
        except Exception as e:
            if metrics_collector:
                metrics_collector.increment(f"{service_name}_event_non_retryable_errors_total",
                                            tags={"error_type": type(e).__name__, "event_type": et})
            if error_reporter:
                error_reporter.report(e, context={"service": service_name, "event": event,
                                                  "attempt": ctx.attempt_number})
            raise


def retry_with_backoff(fn: Callable[[], Any], attempts: int, base_seconds: float, cap_seconds: float = 60.0,
                       retry_on: tuple = (Exception,), sleeper: Callable[[float], None] = time.sleep):
    """Service-level retry used by embedding/summarization (base * 2^n capped, reference
    embedding/app/service.py:366-371, summarization/app/service.py:395-402)."""
    last = None
    for n in range(attempts):
        try:
            return fn()
        except retry_on as e:  # noqa: PERF203
            last = e
            if n + 1 < attempts:
                sleeper(min(base_seconds * (2 ** n), cap_seconds))
    raise last
