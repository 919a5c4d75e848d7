"""Driver for the native cfc-broker (``MESSAGE_BUS_TYPE=cfcbroker``) + admin / failed-queue client.

The broker (csrc/broker/cfc_broker.cpp, built to ``_lib/cfc-broker``) is the RabbitMQ replacement
for running the services as separate processes on one node: a topic exchange, durable journaled
queues, publisher confirms, prefetch, ack / nack(requeue) and a redelivery limit with ``<queue>.dlq``
dead-letter queues.  This module keeps the reference's publisher / subscriber behaviour
(rabbitmq_publisher.py:148-156 confirms + persistent publish, :389-406 reconnect-and-retry-once;
rabbitmq_subscriber.py:376-476 reconnecting consume loop, :504-560 ack on success, nack+requeue on
callback error, ack (drop) of malformed JSON) on top of the broker's length-prefixed TCP protocol.
"""
from __future__ import annotations

import itertools
import json
import os
import select
import socket
import struct
import subprocess
import threading
import time
import uuid
from collections import deque
from pathlib import Path
from typing import Any

from ..contracts.events import EXCHANGE, ROUTING_KEYS
from .base import Callback, EventPublisher, EventSubscriber

PROTOCOL_VERSION = 1
OP_HELLO, OP_OK, OP_ERR = 1, 2, 3
OP_DECLARE, OP_BIND, OP_UNBIND, OP_DELETE, OP_PURGE = 10, 11, 12, 13, 14
OP_PUBLISH, OP_CONFIRM = 20, 21
OP_CONSUME, OP_CANCEL, OP_DELIVER, OP_ACK, OP_NACK = 30, 31, 32, 33, 34
OP_GET, OP_GET_OK, OP_PEEK, OP_PEEK_OK = 40, 41, 42, 43
OP_STATS, OP_STATS_OK = 50, 51
OP_PING, OP_PONG = 60, 61
_REPLIES = {OP_OK, OP_ERR, OP_CONFIRM, OP_GET_OK, OP_PEEK_OK, OP_STATS_OK, OP_PONG}

BROKER_BIN = Path(__file__).resolve().parent.parent / "_lib" / "cfc-broker"
DEFAULT_PORT = 5680


class BrokerError(RuntimeError):
    """The broker answered a request with an error."""


def _s(x: str | bytes) -> bytes:
    b = x.encode() if isinstance(x, str) else x
    if len(b) > 0xFFFF:
        raise ValueError("string field longer than 65535 bytes")
    return struct.pack(">H", len(b)) + b


def _blob(b: bytes) -> bytes:
    return struct.pack(">I", len(b)) + b


class _Cursor:
    def __init__(self, b: bytes):
        self.b, self.o = b, 0

    def u8(self) -> int:
        v = self.b[self.o]
        self.o += 1
        return v

    def u32(self) -> int:
        (v,) = struct.unpack_from(">I", self.b, self.o)
        self.o += 4
        return v

    def u64(self) -> int:
        (v,) = struct.unpack_from(">Q", self.b, self.o)
        self.o += 8
        return v

    def str(self) -> str:
        (n,) = struct.unpack_from(">H", self.b, self.o)
        self.o += 2 + n
        return self.b[self.o - n:self.o].decode("utf-8", "replace")

    def blob(self) -> bytes:
        n = self.u32()
        self.o += n
        return bytes(self.b[self.o - n:self.o])


class Delivery:
    __slots__ = ("tag", "redeliveries", "queue", "routing_key", "body")

    def __init__(self, tag, redeliveries, queue, routing_key, body):
        self.tag, self.redeliveries, self.queue, self.routing_key, self.body = tag, redeliveries, queue, routing_key, body


class Connection:
    """One TCP connection to the broker.  Requests are serialised by a lock; deliveries that arrive
    while a request waits for its reply are queued and handed out by :meth:`next_delivery`."""

    def __init__(self, host: str = "localhost", port: int = DEFAULT_PORT, timeout: float = 10.0,
                 name: str = "cfc-client"):
        self.host, self.port, self.timeout = host, int(port), timeout
        self.sock = socket.create_connection((host, self.port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.sock.setblocking(True)
        self._rbuf = bytearray()
        self._ids = itertools.count(1)
        self._lock = threading.RLock()
        self.deliveries: deque[Delivery] = deque()
        self.closed = False
        self.request(OP_HELLO, struct.pack(">I", PROTOCOL_VERSION) + _s(name))

    # ------------------------------------------------------------------ framing
    def _send(self, op: int, payload: bytes) -> None:
        self.sock.sendall(struct.pack(">IB", 1 + len(payload), op) + payload)

    def _read_frame(self, timeout: float | None) -> tuple[int, bytes] | None:
        deadline = None if timeout is None else time.monotonic() + timeout
        while True:
            if len(self._rbuf) >= 4:
                (n,) = struct.unpack_from(">I", self._rbuf, 0)
                if len(self._rbuf) >= 4 + n:
                    op = self._rbuf[4]
                    payload = bytes(self._rbuf[5:4 + n])
                    del self._rbuf[:4 + n]
                    return op, payload
            wait = None if deadline is None else max(0.0, deadline - time.monotonic())
            if wait is not None:
                r, _, _ = select.select([self.sock], [], [], wait)
                if not r:
                    return None
            chunk = self.sock.recv(1 << 16)
            if not chunk:
                self.closed = True
                raise ConnectionError("broker closed the connection")
            self._rbuf += chunk

    def _take_delivery(self, payload: bytes) -> None:
        c = _Cursor(payload)
        tag, red = c.u64(), c.u32()
        q, rk = c.str(), c.str()
        self.deliveries.append(Delivery(tag, red, q, rk, c.blob()))

    def request(self, op: int, payload: bytes, timeout: float | None = None) -> tuple[int, _Cursor]:
        rid = next(self._ids)
        with self._lock:
            self._send(op, struct.pack(">I", rid) + payload)
            deadline = time.monotonic() + (timeout or self.timeout)
            while True:
                fr = self._read_frame(max(0.0, deadline - time.monotonic()))
                if fr is None:
                    raise TimeoutError(f"broker did not answer op {op} within {timeout or self.timeout}s")
                rop, body = fr
                if rop == OP_DELIVER:
                    self._take_delivery(body)
                    continue
                c = _Cursor(body)
                if rop not in _REPLIES or c.u32() != rid:
                    raise ConnectionError(f"unexpected frame op={rop} from broker")
                if rop == OP_ERR:
                    raise BrokerError(c.str())
                return rop, c

    def next_delivery(self, timeout: float) -> Delivery | None:
        if self.deliveries:
            return self.deliveries.popleft()
        with self._lock:
            fr = self._read_frame(timeout)
            while fr is not None:
                op, body = fr
                if op == OP_DELIVER:
                    self._take_delivery(body)
                    break
                fr = self._read_frame(0.0)   # stray reply of a timed-out request: skip
        return self.deliveries.popleft() if self.deliveries else None

    # ------------------------------------------------------------------ operations
    def declare(self, queue: str, durable: bool = True, max_redeliveries: int = 0) -> int:
        _, c = self.request(OP_DECLARE, _s(queue) + struct.pack(">BI", 1 if durable else 0, max_redeliveries))
        return c.u32()

    def bind(self, queue: str, exchange: str, pattern: str) -> None:
        self.request(OP_BIND, _s(queue) + _s(exchange) + _s(pattern))

    def unbind(self, queue: str, exchange: str, pattern: str) -> None:
        self.request(OP_UNBIND, _s(queue) + _s(exchange) + _s(pattern))

    def delete(self, queue: str) -> int:
        return self.request(OP_DELETE, _s(queue))[1].u32()

    def purge(self, queue: str) -> int:
        return self.request(OP_PURGE, _s(queue))[1].u32()

    def publish(self, exchange: str, routing_key: str, body: bytes, timeout: float | None = None) -> int:
        """Returns the number of queues the message was routed to, once it is durable (confirm)."""
        _, c = self.request(OP_PUBLISH, _s(exchange) + _s(routing_key) + _blob(body), timeout)
        return c.u32()

    def consume(self, queue: str, prefetch: int = 1) -> None:
        self.request(OP_CONSUME, _s(queue) + struct.pack(">I", prefetch))

    def cancel(self, queue: str) -> None:
        self.request(OP_CANCEL, _s(queue))

    def ack(self, tag: int) -> None:
        with self._lock:
            self._send(OP_ACK, struct.pack(">Q", tag))

    def nack(self, tag: int, requeue: bool = True) -> None:
        with self._lock:
            self._send(OP_NACK, struct.pack(">QB", tag, 1 if requeue else 0))

    def get(self, queue: str) -> Delivery | None:
        """Remove and return the head of a queue (auto-acked), or None."""
        _, c = self.request(OP_GET, _s(queue))
        if not c.u8():
            return None
        red = c.u32()
        rk = c.str()
        return Delivery(0, red, queue, rk, c.blob())

    def peek(self, queue: str, limit: int = 10) -> list[Delivery]:
        _, c = self.request(OP_PEEK, _s(queue) + struct.pack(">I", limit))
        out = []
        for _ in range(c.u32()):
            red = c.u32()
            rk = c.str()
            out.append(Delivery(0, red, queue, rk, c.blob()))
        return out

    def stats(self) -> dict:
        return json.loads(self.request(OP_STATS, b"")[1].blob())

    def ping(self) -> float:
        t = time.perf_counter()
        self.request(OP_PING, b"")
        return time.perf_counter() - t

    def close(self) -> None:
        self.closed = True
        try:
            self.sock.close()
        except OSError:
            pass


def _endpoint(host, port, url):
    if url:
        rest = url.split("://", 1)[-1]
        host, _, p = rest.partition(":")
        port = int(p or DEFAULT_PORT)
    return host, int(port)


class CfcBrokerPublisher(EventPublisher):
    def __init__(self, broker_host: str = "localhost", broker_port: int = DEFAULT_PORT, broker_url: str | None = None,
                 exchange: str = EXCHANGE, confirm_timeout: float = 30.0, **_):
        self.host, self.port = _endpoint(broker_host, broker_port, broker_url)
        self.exchange, self.confirm_timeout = exchange, confirm_timeout
        self.conn: Connection | None = None
        self._lock = threading.Lock()
        self.unroutable = 0

    def connect(self) -> None:
        self.conn = Connection(self.host, self.port, name="publisher")

    def disconnect(self) -> None:
        if self.conn:
            self.conn.close()
            self.conn = None

    def publish(self, exchange: str, routing_key: str, event: dict[str, Any]) -> None:
        body = json.dumps(event).encode()
        with self._lock:
            for attempt in range(2):   # reconnect and retry once (rabbitmq_publisher.py:389-406)
                try:
                    if self.conn is None or self.conn.closed:
                        self.connect()
                    if self.conn.publish(exchange or self.exchange, routing_key, body, self.confirm_timeout) == 0:
                        self.unroutable += 1
                    return
                except (OSError, ConnectionError, TimeoutError):
                    if self.conn:
                        self.conn.close()
                    self.conn = None
                    if attempt:
                        raise


class CfcBrokerSubscriber(EventSubscriber):
    """One durable queue per service (the reference binds one queue per routing key per service,
    infra/rabbitmq/definitions.json), prefetch-limited, reconnecting consume loop."""

    def __init__(self, broker_host: str = "localhost", broker_port: int = DEFAULT_PORT, broker_url: str | None = None,
                 exchange: str = EXCHANGE, queue_name: str | None = None, queue_durable: bool = True,
                 prefetch_count: int = 1, max_redeliveries: int = 0, **_):
        self.host, self.port = _endpoint(broker_host, broker_port, broker_url)
        self.exchange = exchange
        self.queue_name = queue_name or f"q-{uuid.uuid4().hex[:12]}"
        self.durable = bool(queue_durable) and queue_name is not None
        self.prefetch, self.max_redeliveries = int(prefetch_count), int(max_redeliveries)
        self.callbacks: dict[str, Callback] = {}
        self.bindings: list[tuple[str, str]] = []
        self.conn: Connection | None = None
        self._consuming: Connection | None = None   # the connection a CONSUME was issued on
        self._stop = threading.Event()
        self.processed = self.failed = self.reconnects = 0

    def connect(self) -> None:
        conn = Connection(self.host, self.port, name=f"subscriber:{self.queue_name}")
        conn.declare(self.queue_name, self.durable, self.max_redeliveries)
        for ex, key in self.bindings:
            conn.bind(self.queue_name, ex, key)
        self.conn = conn

    def disconnect(self) -> None:
        if self.conn:
            self.conn.close()
            self.conn = None

    def subscribe(self, event_type: str, callback: Callback, routing_key: str | None = None,
                  exchange: str | None = None) -> None:
        self.callbacks[event_type] = callback
        b = (exchange or self.exchange, routing_key or ROUTING_KEYS.get(event_type, event_type))
        if b not in self.bindings:
            self.bindings.append(b)
            if self.conn is not None and not self.conn.closed:
                self.conn.bind(self.queue_name, *b)

    def _handle(self, d: Delivery) -> None:
        try:
            event = json.loads(d.body)
            cb = self.callbacks.get(event["event_type"])
        except (ValueError, KeyError, TypeError):
            self.failed += 1
            self.conn.ack(d.tag)        # malformed: drop, like the reference
            return
        if cb is None:
            self.conn.ack(d.tag)
            return
        try:
            cb(event)
        except Exception:   # noqa: BLE001 -- the callback's failure is the broker's redelivery signal
            self.failed += 1
            self.conn.nack(d.tag, requeue=True)
            return
        self.processed += 1
        self.conn.ack(d.tag)

    def _ensure(self) -> None:
        if self.conn is None or self.conn.closed:
            self.connect()
        if self._consuming is not self.conn:
            self.conn.consume(self.queue_name, self.prefetch)
            self._consuming = self.conn

    def drain(self, max_items: int | None = None, idle_timeout: float = 0.2) -> int:
        """Handle deliveries on the calling thread until none arrives for ``idle_timeout`` seconds."""
        self._ensure()
        n = 0
        while max_items is None or n < max_items:
            d = self.conn.next_delivery(idle_timeout)
            if d is None:
                break
            self._handle(d)
            n += 1
        return n

    def start_consuming(self) -> None:
        self._stop.clear()
        backoff = 0.5
        while not self._stop.is_set():
            try:
                self._ensure()
                backoff = 0.5
                while not self._stop.is_set():
                    d = self.conn.next_delivery(0.25)
                    if d is not None:
                        self._handle(d)
            except (OSError, ConnectionError, TimeoutError, BrokerError):
                if self.conn:
                    self.conn.close()
                self.conn = None
                self.reconnects += 1
                self._stop.wait(backoff)
                backoff = min(backoff * 2, 10.0)
        self.disconnect()

    def stop_consuming(self) -> None:
        self._stop.set()


class CfcBrokerFailedQueues:
    """tools/failed_queues.py backend: the ``*.failed`` routing-key queues and every ``.dlq``."""

    def __init__(self, host: str = "localhost", port: int = DEFAULT_PORT, exchange: str = EXCHANGE):
        from ..tools.failed_queues import failed_routing_keys
        self.conn = Connection(host, port, name="failed-queues")
        self.exchange = exchange
        for rk in failed_routing_keys():    # make failures observable from now on
            self.conn.declare(rk, True)
            self.conn.bind(rk, exchange, rk)

    def names(self) -> list[str]:
        from ..tools.failed_queues import failed_routing_keys
        qs = self.conn.stats()["queues"]
        return sorted(set(failed_routing_keys()) | {q for q, v in qs.items() if q.endswith(".dlq") and v["ready"]})

    def count(self, name: str) -> int:
        return int(self.conn.stats()["queues"].get(name, {}).get("ready", 0))

    def peek(self, name: str, limit: int) -> list[dict]:
        return [json.loads(d.body) for d in self.conn.peek(name, limit)]

    def pop(self, name: str) -> dict | None:
        d = self.conn.get(name)
        return None if d is None else json.loads(d.body)

    def publish(self, routing_key: str, event: dict) -> None:
        self.conn.publish(self.exchange, routing_key, json.dumps(event).encode())


class CfcBrokerMonitor:
    """Queue gauges for tools/exporters.py (the reference reads them from the RabbitMQ management
    API for its queue-lag alerts, infra/prometheus/alerts/queue_lag.yml)."""

    def __init__(self, host: str = "localhost", port: int = DEFAULT_PORT):
        self.host, self.port = host, int(port)
        self.conn: Connection | None = None

    def stats(self) -> dict:
        for attempt in range(2):
            try:
                if self.conn is None or self.conn.closed:
                    self.conn = Connection(self.host, self.port, name="monitor")
                return self.conn.stats()
            except (OSError, ConnectionError, TimeoutError):
                self.conn = None
                if attempt:
                    raise
        return {}

    def queues(self) -> dict[str, int]:
        return {q: v["ready"] for q, v in self.stats().get("queues", {}).items()}

    def consumer_counts(self) -> dict[str, int]:
        return {q: v["consumers"] for q, v in self.stats().get("queues", {}).items()}

    def queue_details(self) -> dict[str, dict]:
        return self.stats().get("queues", {})


def spawn_broker(port: int = 0, data_dir: str | os.PathLike | None = None, host: str = "127.0.0.1",
                 fsync: bool = True, max_redeliveries: int = 5, binary: str | os.PathLike | None = None,
                 timeout: float = 10.0) -> tuple[subprocess.Popen, int]:
    """Start a broker process; returns (process, port).  ``port=0`` picks a free port."""
    exe = Path(binary or BROKER_BIN)
    if not exe.exists():
        from .._build import build_broker
        build_broker(verbose=False)
    cmd = [str(exe), "--host", host, "--port", str(port), "--max-redeliveries", str(max_redeliveries),
           "--fsync", "always" if fsync else "never"]
    if data_dir is not None:
        cmd += ["--data-dir", str(data_dir)]
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=None, text=True)
    deadline = time.monotonic() + timeout
    line = ""
    while time.monotonic() < deadline:
        r, _, _ = select.select([proc.stdout], [], [], 0.1)
        if r:
            line = proc.stdout.readline()
            break
        if proc.poll() is not None:
            break
    if "listening on" not in line:
        proc.kill()
        raise RuntimeError(f"cfc-broker failed to start: {line!r}")
    return proc, int(line.rsplit(":", 1)[1])
