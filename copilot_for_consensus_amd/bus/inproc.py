"""In-process topic-exchange broker -- the default single-node transport.

Replaces RabbitMQ (rabbitmq_publisher.py / rabbitmq_subscriber.py of the reference) when every
stage runs in one process per node: same exchange/queue/routing-key model, persistent-until-acked
semantics, ack on callback success, nack+requeue on callback failure (rabbitmq_subscriber.py:
537-539) -- with a redelivery limit after which the message goes to ``<queue>.dlq`` (the
reference only counts a DLQ metric), and malformed messages dropped (acked).

Thread-safe: publishers may run on any thread; each subscriber's ``start_consuming`` blocks its
own thread.  ``drain()`` processes everything queued synchronously (tests, batch pipelines).
"""
from __future__ import annotations

import collections
import copy
import json
import threading
from typing import Any

from ..contracts.events import EXCHANGE, ROUTING_KEYS
from .base import Callback, EventPublisher, EventSubscriber, topic_matches
from .validating import EventValidationError


class _Queue:
    def __init__(self, name: str):
        self.name = name
        self.bindings: set[tuple[str, str]] = set()  # (exchange, pattern)
        self.items: collections.deque = collections.deque()
        self.cv = threading.Condition()


class InProcBroker:
    def __init__(self, max_redeliveries: int = 5):
        self._lock = threading.RLock()
        self._queues: dict[str, _Queue] = {}
        self.max_redeliveries = max_redeliveries
        self.published = 0
        self.dead_letters: dict[str, list] = collections.defaultdict(list)
        self._consumers: collections.Counter = collections.Counter()

    def declare_queue(self, name: str) -> _Queue:
        with self._lock:
            q = self._queues.get(name)
            if q is None:
                q = self._queues[name] = _Queue(name)
            return q

    def bind(self, queue: str, exchange: str, pattern: str) -> None:
        self.declare_queue(queue).bindings.add((exchange, pattern))

    def publish(self, exchange: str, routing_key: str, body: bytes) -> int:
        with self._lock:
            targets = [q for q in self._queues.values()
                       if any(ex == exchange and topic_matches(p, routing_key) for ex, p in q.bindings)]
            self.published += 1
        for q in targets:
            with q.cv:
                q.items.append([routing_key, body, 0])
                q.cv.notify()
        return len(targets)

    def queue_depth(self, name: str) -> int:
        q = self._queues.get(name)
        return len(q.items) if q else 0

    def queues(self) -> dict[str, int]:
        return {n: len(q.items) for n, q in self._queues.items()}

    def consumer_counts(self) -> dict[str, int]:
        """Active consumers per queue (management-API ``consumers`` field)."""
        with self._lock:
            return {n: self._consumers[n] for n in self._queues}

    def _consumer(self, queue: str, delta: int) -> None:
        with self._lock:
            self._consumers[queue] = max(0, self._consumers[queue] + delta)


_default_broker: InProcBroker | None = None
_default_lock = threading.Lock()


def default_broker() -> InProcBroker:
    global _default_broker
    with _default_lock:
        if _default_broker is None:
            _default_broker = InProcBroker()
        return _default_broker


def reset_default_broker() -> None:
    global _default_broker
    with _default_lock:
        _default_broker = None


class InProcPublisher(EventPublisher):
    def __init__(self, broker: InProcBroker | None = None, exchange: str = EXCHANGE, **_):
        self.broker = broker or default_broker()
        self.exchange = exchange
        self.connected = False

    def connect(self) -> None:
        self.connected = True

    def publish(self, exchange: str, routing_key: str, event: dict[str, Any]) -> None:
        # serialise like a real transport: subscribers never share the publisher's objects
        self.broker.publish(exchange or self.exchange, routing_key, json.dumps(event).encode())


class InProcSubscriber(EventSubscriber):
    def __init__(self, broker: InProcBroker | None = None, queue_name: str | None = None, exchange: str = EXCHANGE,
                 **_):
        self.broker = broker or default_broker()
        self.exchange = exchange
        self.queue_name = queue_name or f"q-{id(self):x}"
        self.queue = self.broker.declare_queue(self.queue_name)
        self.callbacks: dict[str, Callback] = {}
        self._stop = threading.Event()
        self.processed = 0
        self.failed = 0

    def subscribe(self, event_type: str, callback: Callback, routing_key: str | None = None,
                  exchange: str | None = None) -> None:
        self.callbacks[event_type] = callback
        key = routing_key or ROUTING_KEYS.get(event_type, event_type)
        self.broker.bind(self.queue_name, exchange or self.exchange, key)

    def _handle(self, item) -> None:
        routing_key, body, redeliveries = item
        try:
            event = json.loads(body)
            event_type = event["event_type"]
        except (ValueError, KeyError, TypeError):
            self.failed += 1  # malformed: ack (drop), like the reference
            return
        cb = self.callbacks.get(event_type)
        if cb is None:
            return
        try:
            cb(copy.deepcopy(event))
            self.processed += 1
        except Exception as e:
            self.failed += 1
            # a schema-invalid event fails the same way on every delivery: dead-letter it at once
            poison = isinstance(e, EventValidationError)
            if poison or redeliveries + 1 >= self.broker.max_redeliveries:
                self.broker.dead_letters[self.queue_name].append(event)
            else:
                with self.queue.cv:  # nack + requeue at the tail
                    self.queue.items.append([routing_key, body, redeliveries + 1])
                    self.queue.cv.notify()

    def _pop(self, timeout: float | None):
        with self.queue.cv:
            if not self.queue.items:
                self.queue.cv.wait(timeout)
            return self.queue.items.popleft() if self.queue.items else None

    def drain(self, max_items: int | None = None) -> int:
        """Process queued events synchronously on the calling thread; returns count handled."""
        n = 0
        while max_items is None or n < max_items:
            with self.queue.cv:
                item = self.queue.items.popleft() if self.queue.items else None
            if item is None:
                break
            self._handle(item)
            n += 1
        return n

    def start_consuming(self) -> None:
        self._stop.clear()
        self.broker._consumer(self.queue_name, +1)
        try:
            while not self._stop.is_set():
                item = self._pop(0.05)
                if item is not None:
                    self._handle(item)
        finally:
            self.broker._consumer(self.queue_name, -1)

    def stop_consuming(self) -> None:
        self._stop.set()
        with self.queue.cv:
            self.queue.cv.notify_all()


class NoopPublisher(EventPublisher):
    """Records events (reference noop_publisher.py:16,47-79)."""

    def __init__(self, **_):
        self.published_events: list[dict] = []
        self.connected = False

    def connect(self) -> None:
        self.connected = True

    def disconnect(self) -> None:
        self.connected = False

    def publish(self, exchange: str, routing_key: str, event: dict[str, Any]) -> None:
        self.published_events.append({"exchange": exchange, "routing_key": routing_key, "event": copy.deepcopy(event)})

    def get_events(self, event_type: str | None = None) -> list[dict]:
        evs = [p["event"] for p in self.published_events]
        return [e for e in evs if event_type is None or e.get("event_type") == event_type]

    def clear_events(self) -> None:
        self.published_events.clear()


class CountingPublisher(EventPublisher):
    """Counts events per type without retaining payloads (long-running batch pipelines)."""

    def __init__(self, **_):
        self.counts: dict[str, int] = collections.Counter()
        self.bytes = 0

    def publish(self, exchange: str, routing_key: str, event: dict[str, Any]) -> None:
        self.counts[event.get("event_type", "?")] += 1


class NoopSubscriber(EventSubscriber):
    """Callbacks driven by ``inject_event`` (reference noop_subscriber.py:18,101-123)."""

    def __init__(self, **_):
        self.callbacks: dict[str, Callback] = {}
        self.routing_keys: dict[str, str | None] = {}
        self.connected = False
        self.consuming = False
        self._stop = threading.Event()

    def connect(self) -> None:
        self.connected = True

    def disconnect(self) -> None:
        self.connected = False

    def subscribe(self, event_type: str, callback: Callback, routing_key: str | None = None,
                  exchange: str | None = None) -> None:
        self.callbacks[event_type] = callback
        self.routing_keys[event_type] = routing_key

    def start_consuming(self) -> None:
        self.consuming = True
        self._stop.clear()
        self._stop.wait()

    def stop_consuming(self) -> None:
        self.consuming = False
        self._stop.set()

    def inject_event(self, event: dict[str, Any]) -> None:
        et = event.get("event_type")
        if not et:
            raise ValueError("Event must have 'event_type' field")
        cb = self.callbacks.get(et)
        if cb:
            cb(event)

    def get_subscriptions(self) -> list[str]:
        return list(self.callbacks)
