"""Logging, metrics, error reporting and tracing spans.

* Logger (adapters/copilot_logging): ``StdoutLogger`` emits one JSON object per line
  (timestamp, level, logger, message, **kv) -- stdout_logger.py:64-93; ``SilentLogger``.
* MetricsCollector (adapters/copilot_metrics base.py:20-64): increment / observe / gauge /
  safe_push.  ``PrometheusMetricsCollector`` keeps counters, gauges and histograms in-process and
  renders the Prometheus text exposition format (services can serve ``/metrics`` -- the reference
  only pushes); ``PushGatewayMetricsCollector`` PUTs that text to a Pushgateway; ``NoOp``.
  Metric names are the reference's (``<svc>_event_retry_*``, ``embedding_generation_duration_seconds``,
  ``summarization_latency_seconds`` ...).  GPU metrics (tokens/s, TTFT, HBM) are gauges here.
* ErrorReporter (adapters/copilot_error_reporting): console / silent / sentry(optional).
* ``span`` -- a timing context manager recorded into a histogram and, on a GPU, bracketed with a
  roctx range when the ROCm tracer is importable (rocprofv3 --marker-trace shows pipeline stages).
"""
from __future__ import annotations

import collections
import contextlib
import json
import logging
import os
import re
import sys
import threading
import time
import traceback
import urllib.request
from abc import ABC, abstractmethod
from datetime import datetime, timezone
from typing import Any

# ------------------------------------------------------------------------------------- logging

_LEVELS = {"DEBUG": 10, "INFO": 20, "WARNING": 30, "ERROR": 40, "CRITICAL": 50}


class Logger(ABC):
    @abstractmethod
    def log(self, level: str, message: str, **kw) -> None: ...

    def debug(self, m, **kw): self.log("DEBUG", m, **kw)
    def info(self, m, **kw): self.log("INFO", m, **kw)
    def warning(self, m, **kw): self.log("WARNING", m, **kw)
    def error(self, m, **kw): self.log("ERROR", m, **kw)

    def exception(self, m, **kw):
        kw["traceback"] = traceback.format_exc()
        self.log("ERROR", m, **kw)


class StdoutLogger(Logger):
    def __init__(self, level: str = "INFO", name: str | None = None, stream=None, **_):
        lv = str(level).upper()
        lv = "WARNING" if lv == "WARN" else lv
        if lv not in _LEVELS:
            raise ValueError(f"Invalid log level {level!r}; choose one of {', '.join(_LEVELS)}")
        self.level = _LEVELS[lv]
        self.name = name or "copilot"
        self.stream = stream or sys.stdout
        self._lock = threading.Lock()

    def log(self, level, message, **kw):
        level = str(level).upper()
        level = "WARNING" if level == "WARN" else level
        if _LEVELS.get(level, 20) < self.level:
            return
        rec = {"timestamp": datetime.now(timezone.utc).isoformat().replace("+00:00", "Z"), "level": level,
               "logger": self.name, "message": message}
        for k, v in kw.items():
            rec[k] = v if isinstance(v, (str, int, float, bool, type(None), list, dict)) else repr(v)
        line = json.dumps(rec, default=str)
        with self._lock:
            self.stream.write(line + "\n")
            self.stream.flush()


class SilentLogger(Logger):
    """Records instead of printing (tests inspect what a service logged)."""

    def __init__(self, **_):
        self.records: list[tuple[str, str, dict]] = []

    def log(self, level, message, **kw):
        if len(self.records) < 10000:
            self.records.append((str(level).upper(), message, kw))

    def get_logs(self, level: str | None = None) -> list[tuple[str, str, dict]]:
        return [r for r in self.records if level is None or r[0] == level.upper()]

    def has_log(self, message: str, level: str | None = None) -> bool:
        return any(message in r[1] for r in self.get_logs(level))

    def clear(self) -> None:
        self.records.clear()


_default_logger: Logger | None = None


def create_logger(cfg=None, **overrides) -> Logger:
    name = str(getattr(cfg, "driver_name", cfg) or "stdout").strip().lower()
    kw = {k: v for k, v in dict(getattr(cfg, "driver_config", {}) or {}).items() if v is not None}
    kw.update(overrides)
    cls = {"stdout": StdoutLogger, "silent": SilentLogger}.get(name)
    if cls is None:
        raise ValueError(f"unknown logger driver {name!r} (stdout or silent)")
    return cls(**kw)


def set_default_logger(lg: Logger) -> None:
    global _default_logger
    _default_logger = lg


_fallback_loggers: dict[str | None, Logger] = {}


def get_logger(name: str | None = None) -> Logger:
    """The process default (``set_default_logger``) if one is set, else a stdout logger cached by
    name, so modules calling ``get_logger(__name__)`` repeatedly share one instance."""
    if _default_logger is not None:
        return _default_logger
    lg = _fallback_loggers.get(name)
    if lg is None:
        lg = _fallback_loggers[name] = StdoutLogger(name=name)
    return lg


def uvicorn_log_config(level: str = "INFO") -> dict:
    """uvicorn dictConfig emitting JSON lines (reference copilot_logging/uvicorn_config.py)."""
    fmt = '{"timestamp":"%(asctime)s","level":"%(levelname)s","logger":"%(name)s","message":"%(message)s"}'
    return {"version": 1, "disable_existing_loggers": False,
            "formatters": {"json": {"format": fmt}},
            "handlers": {"default": {"class": "logging.StreamHandler", "formatter": "json", "stream": "ext://sys.stdout"}},
            # access logs at WARNING: health probes and normal requests stay out of the log stream
            "loggers": {"uvicorn": {"handlers": ["default"], "level": level},
                        "uvicorn.error": {"handlers": ["default"], "level": level, "propagate": False},
                        "uvicorn.access": {"handlers": ["default"], "level": "WARNING", "propagate": False}}}


# ------------------------------------------------------------------------------------- metrics

def _key(name, tags):
    return (name, tuple(sorted((str(k), str(v)) for k, v in (tags or {}).items())))


_NAME_OK = re.compile(r"[^a-zA-Z0-9_:]")


def _metric_name(name: str) -> str:
    """Prometheus metric / label names: [a-zA-Z_:][a-zA-Z0-9_:]* (other characters become '_')."""
    n = _NAME_OK.sub("_", str(name))
    return n if n and not n[0].isdigit() else "_" + n


def _label_value(v) -> str:
    """Exposition-format escaping of a label value: backslash, double quote, newline."""
    return str(v).replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n")


DEFAULT_BUCKETS = (0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60, 120, 300)


class MetricsCollector(ABC):
    @abstractmethod
    def increment(self, name: str, value: float = 1.0, tags: dict | None = None) -> None: ...

    @abstractmethod
    def observe(self, name: str, value: float, tags: dict | None = None) -> None: ...

    @abstractmethod
    def gauge(self, name: str, value: float, tags: dict | None = None) -> None: ...

    def push(self) -> None:
        pass

    def safe_push(self) -> None:
        try:
            self.push()
        except Exception:  # metrics must never break the pipeline
            pass


class NoOpMetricsCollector(MetricsCollector):
    def __init__(self, **_):
        pass

    def increment(self, name, value=1.0, tags=None): pass
    def observe(self, name, value, tags=None): pass
    def gauge(self, name, value, tags=None): pass


class PrometheusMetricsCollector(MetricsCollector):
    def __init__(self, namespace: str = "copilot", raise_on_error: bool = False, buckets=DEFAULT_BUCKETS, **_):
        self.namespace = namespace
        self.buckets = tuple(buckets)
        self._lock = threading.Lock()
        self.counters: dict = collections.defaultdict(float)
        self.gauges: dict = {}
        self.hist: dict = {}

    def _n(self, name):
        name = _metric_name(name)
        return f"{self.namespace}_{name}" if self.namespace and not name.startswith(self.namespace + "_") else name

    def increment(self, name, value=1.0, tags=None):
        with self._lock:
            self.counters[_key(self._n(name), tags)] += value

    def gauge(self, name, value, tags=None):
        with self._lock:
            self.gauges[_key(self._n(name), tags)] = float(value)

    def observe(self, name, value, tags=None):
        with self._lock:
            k = _key(self._n(name), tags)
            h = self.hist.get(k)
            if h is None:
                h = self.hist[k] = [[0] * len(self.buckets), 0.0, 0]
            for i, b in enumerate(self.buckets):
                if value <= b:
                    h[0][i] += 1
            h[1] += value
            h[2] += 1

    def get_counter(self, name, tags=None) -> float:
        return self.counters.get(_key(self._n(name), tags), 0.0)

    @staticmethod
    def _labels(tags, extra=None):
        items = list(tags) + (extra or [])
        return "{" + ",".join(f'{_metric_name(k)}="{_label_value(v)}"' for k, v in items) + "}" if items else ""

    def render(self) -> str:
        """Prometheus text exposition format 0.0.4: one ``# TYPE`` line per metric family, then
        its samples (label values escaped)."""
        out = []
        typed = set()

        def family(n, kind):
            if n not in typed:
                typed.add(n)
                out.append(f"# TYPE {n} {kind}")

        with self._lock:
            for (n, t), v in sorted(self.counters.items()):
                family(n, "counter")
                out.append(f"{n}{self._labels(t)} {v}")
            for (n, t), v in sorted(self.gauges.items()):
                family(n, "gauge")
                out.append(f"{n}{self._labels(t)} {v}")
            for (n, t), (counts, s, c) in sorted(self.hist.items()):
                family(n, "histogram")
                for b, cnt in zip(self.buckets, counts):
                    out.append(f"{n}_bucket{self._labels(t, [('le', b)])} {cnt}")
                out.append(f"{n}_bucket{self._labels(t, [('le', '+Inf')])} {c}")
                out.append(f"{n}_sum{self._labels(t)} {s}")
                out.append(f"{n}_count{self._labels(t)} {c}")
        return "\n".join(out) + "\n"


def _push_segment(key, value) -> tuple[str, str]:
    """Pushgateway grouping-key path segment: URL-escaped, or ``key@base64/<urlsafe b64>`` when
    the value contains '/' or is empty (the Pushgateway's own encoding for such values)."""
    import base64
    import urllib.parse
    v = str(value)
    if "/" in v or v == "":
        return f"{key}@base64", base64.urlsafe_b64encode(v.encode()).decode() or "="
    return str(key), urllib.parse.quote(v, safe="")


class PushGatewayMetricsCollector(PrometheusMetricsCollector):
    def __init__(self, gateway: str | None = None, job: str = "copilot", namespace: str = "copilot",
                 raise_on_error: bool = False, grouping_key: dict | None = None, **_):
        super().__init__(namespace)
        self.gateway, self.job = gateway, job
        if isinstance(grouping_key, str):  # env/config form: JSON object or "k=v,k2=v2"
            gk = grouping_key.strip()
            grouping_key = json.loads(gk) if gk.startswith("{") else dict(
                kv.split("=", 1) for kv in gk.split(",") if "=" in kv)
        self.grouping_key = grouping_key or {}
        self.raise_on_error = raise_on_error

    def push(self):
        if not self.gateway:
            return
        url = self.gateway.rstrip("/")
        if not url.startswith("http"):
            url = "http://" + url
        url += f"/metrics/job/{_push_segment('job', self.job)[1]}" + "".join(
            "/{}/{}".format(*_push_segment(k, v)) for k, v in self.grouping_key.items())
        req = urllib.request.Request(url, data=self.render().encode(), method="PUT",
                                     headers={"Content-Type": "text/plain; version=0.0.4"})
        try:
            urllib.request.urlopen(req, timeout=5).read()
        except Exception:
            if self.raise_on_error:
                raise


def create_metrics_collector(cfg=None, **overrides) -> MetricsCollector:
    name = str(getattr(cfg, "driver_name", cfg) or "noop").strip().lower()
    kw = {k: v for k, v in dict(getattr(cfg, "driver_config", {}) or {}).items() if v is not None}
    kw.update(overrides)
    if name == "noop":
        return NoOpMetricsCollector()
    if name == "prometheus":
        return PrometheusMetricsCollector(**kw)
    if name == "pushgateway":
        return PushGatewayMetricsCollector(**kw)
    if name == "azure_monitor":
        from ..cloud.azure import AzureMonitorMetricsCollector
        return AzureMonitorMetricsCollector(**kw)
    raise ValueError(f"unknown metrics driver {name!r}")


# ------------------------------------------------------------------------------ error reporting

class ErrorReporter(ABC):
    @abstractmethod
    def report(self, error: BaseException, context: dict | None = None) -> None: ...

    def capture_message(self, message: str, level: str = "error", context: dict | None = None) -> None:
        self.report(RuntimeError(message), context)


class ConsoleErrorReporter(ErrorReporter):
    def __init__(self, logger_name: str | None = None, logger: Logger | None = None, **_):
        self.logger = logger or StdoutLogger(name=logger_name or "errors", stream=sys.stderr)
        self.reported: list[tuple[BaseException, dict]] = []

    def report(self, error, context=None):
        self.reported.append((error, dict(context or {})))
        self.logger.error(f"{type(error).__name__}: {error}", context=context or {})


class SilentErrorReporter(ErrorReporter):
    def __init__(self, **_):
        self.reported: list[tuple[BaseException, dict]] = []

    def report(self, error, context=None):
        self.reported.append((error, dict(context or {})))


class SentryErrorReporter(ErrorReporter):
    """Sentry (sentry_error_reporter.py:13 of the reference); sentry-sdk is imported on construction."""

    def __init__(self, dsn: str | None = None, environment: str = "production", traces_sample_rate: float = 0.0,
                 **_):
        try:
            import sentry_sdk
        except ImportError as e:
            raise ImportError("sentry error reporting needs the 'sentry-sdk' package, which is not installed") from e
        self._sdk = sentry_sdk
        sentry_sdk.init(dsn=dsn, environment=environment, traces_sample_rate=traces_sample_rate)

    def report(self, error, context=None):
        with self._sdk.push_scope() as scope:
            for k, v in (context or {}).items():
                scope.set_extra(k, v)
            self._sdk.capture_exception(error)

    def capture_message(self, message, level="info", context=None):
        self._sdk.capture_message(message, level=level)


def create_error_reporter(cfg=None, **overrides) -> ErrorReporter:
    name = str(getattr(cfg, "driver_name", cfg) or "console").strip().lower()
    kw = {k: v for k, v in dict(getattr(cfg, "driver_config", {}) or {}).items() if v is not None}
    kw.update(overrides)
    if name == "console":
        return ConsoleErrorReporter(**kw)
    if name == "silent":
        return SilentErrorReporter()
    if name == "sentry":
        return SentryErrorReporter(**kw)
    raise ValueError(f"unknown error reporter {name!r}")


# ------------------------------------------------------------------------------------- tracing

def _load_roctx():
    """roctx ranges (shown by ``rocprofv3 --marker-trace``) through the ROCm tracer library."""
    import ctypes
    import os
    for name in ("libroctx64.so", os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "libroctx64.so")):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            return (lambda n: lib.roctxRangePushA(n.encode())), (lambda: lib.roctxRangePop())
        except (OSError, AttributeError):
            continue
    return None, None


_rpush, _rpop = _load_roctx() if os.environ.get("CFC_ROCTX", "1") != "0" else (None, None)


@contextlib.contextmanager
def span(name: str, metrics: MetricsCollector | None = None, tags: dict | None = None, sync_device=None):
    """Time a pipeline stage; observes ``<name>_duration_seconds`` and marks a roctx range."""
    if _rpush:
        _rpush(name)
    t = time.perf_counter()
    try:
        yield
    finally:
        if sync_device is not None:
            import torch
            torch.cuda.synchronize(sync_device)
        if metrics is not None:
            metrics.observe(f"{name}_duration_seconds", time.perf_counter() - t, tags)
        if _rpop:
            _rpop()


del logging
