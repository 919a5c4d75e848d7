"""A stand-in for the ``pika`` SDK (absent from this image) backed by an in-memory AMQP broker.

Implements the part of pika's BlockingConnection API the RabbitMQ driver uses, with RabbitMQ's
semantics where the driver depends on them: topic exchanges, durable / exclusive / server-named
queues, bindings, publisher confirms with ``mandatory`` (UnroutableError when no queue is bound)
and broker nacks (NackError), per-channel prefetch, manual ack / nack(requeue), redelivery of a
closed channel's unacked messages (``redelivered`` set), and fault injection: ``BROKER.kill()``
drops every connection (the next call on it raises StreamLostError) and ``BROKER.up = False``
refuses new connections (AMQPConnectionError).
"""
from __future__ import annotations

import collections
import itertools
import threading
import time
import types

from copilot_for_consensus_amd.bus.base import topic_matches


class _Exc:
    class AMQPError(Exception):
        pass

    class AMQPConnectionError(AMQPError):
        pass

    class StreamLostError(AMQPConnectionError):
        pass

    class ConnectionClosedByBroker(AMQPConnectionError):
        pass

    class ChannelClosedByBroker(AMQPError):
        pass

    class ChannelWrongStateError(AMQPError):
        pass

    class UnroutableError(AMQPError):
        pass

    class NackError(AMQPError):
        pass


exceptions = types.SimpleNamespace(**{k: v for k, v in vars(_Exc).items() if not k.startswith("_")})


class PlainCredentials:
    def __init__(self, username, password):
        self.username, self.password = username, password


class ConnectionParameters:
    def __init__(self, host="localhost", port=5672, virtual_host="/", credentials=None, **kw):
        self.host, self.port, self.virtual_host, self.credentials, self.kw = host, port, virtual_host, credentials, kw


class BasicProperties:
    def __init__(self, delivery_mode=None, content_type=None, **_):
        self.delivery_mode, self.content_type = delivery_mode, content_type


class _Queue:
    def __init__(self, name, durable, exclusive_to=None):
        self.name, self.durable, self.exclusive_to = name, durable, exclusive_to
        self.ready: collections.deque = collections.deque()     # (body, redelivered)


class Broker:
    def __init__(self):
        self.lock = threading.RLock()
        self.reset()

    def reset(self):
        with self.lock:
            self.exchanges: dict[str, str] = {}
            self.queues: dict[str, _Queue] = {}
            self.bindings: list[tuple[str, str, str]] = []        # (exchange, queue, key)
            self.connections: list[BlockingConnection] = []
            self.up = True
            self.nack_next = 0
            self.published = 0
            self._names = itertools.count(1)

    def depth(self, queue: str) -> int:
        with self.lock:
            q = self.queues.get(queue)
            return len(q.ready) if q else 0

    def kill(self):
        """Network partition: every open connection dies; unacked deliveries go back to their queues."""
        with self.lock:
            for c in list(self.connections):
                c._die()

    def route(self, exchange, key) -> list[_Queue]:
        return [self.queues[q] for ex, q, k in self.bindings if ex == exchange and q in self.queues
                and topic_matches(k, key)]


BROKER = Broker()


class BlockingChannel:
    def __init__(self, conn):
        self.conn, self.is_open, self.confirm = conn, True, False
        self.prefetch = 0
        self.consumers: list[tuple[str, object, bool]] = []
        self.unacked: dict[int, tuple[_Queue, bytes]] = {}
        self._tags = itertools.count(1)

    @property
    def is_closed(self):
        return not self.is_open

    def _check(self):
        if self.conn._dead:
            raise exceptions.StreamLostError("connection lost")
        if not self.is_open:
            raise exceptions.ChannelWrongStateError("channel is closed")

    def close(self):
        with BROKER.lock:
            self._requeue_all()
            self.is_open = False

    def _requeue_all(self):
        for q, body in reversed(list(self.unacked.values())):
            q.ready.appendleft((body, True))
        self.unacked.clear()

    def confirm_delivery(self):
        self._check()
        self.confirm = True

    def exchange_declare(self, exchange, exchange_type="direct", durable=False, **_):
        self._check()
        with BROKER.lock:
            if BROKER.exchanges.setdefault(exchange, exchange_type) != exchange_type:
                raise exceptions.ChannelClosedByBroker(f"PRECONDITION_FAILED: exchange {exchange} type")

    def queue_declare(self, queue="", durable=False, exclusive=False, auto_delete=False, passive=False, **_):
        self._check()
        with BROKER.lock:
            name = queue or f"amq.gen-{next(BROKER._names)}"
            q = BROKER.queues.get(name)
            if passive:
                if q is None:
                    raise exceptions.ChannelClosedByBroker(f"NOT_FOUND - no queue '{name}'")
            elif q is None:
                q = BROKER.queues[name] = _Queue(name, durable, self.conn if exclusive else None)
            elif q.durable != durable:
                raise exceptions.ChannelClosedByBroker(f"PRECONDITION_FAILED: queue {name} durable")
        return types.SimpleNamespace(method=types.SimpleNamespace(queue=name, message_count=len(q.ready)))

    def queue_bind(self, queue, exchange, routing_key=None, **_):
        self._check()
        with BROKER.lock:
            if exchange not in BROKER.exchanges or queue not in BROKER.queues:
                raise exceptions.ChannelClosedByBroker("NOT_FOUND")
            b = (exchange, queue, routing_key or queue)
            if b not in BROKER.bindings:
                BROKER.bindings.append(b)

    def basic_qos(self, prefetch_count=0, **_):
        self._check()
        self.prefetch = int(prefetch_count)

    def basic_publish(self, exchange, routing_key, body, properties=None, mandatory=False):
        self._check()
        with BROKER.lock:
            if exchange not in BROKER.exchanges:
                raise exceptions.ChannelClosedByBroker(f"NOT_FOUND - no exchange '{exchange}'")
            if self.confirm and BROKER.nack_next:
                BROKER.nack_next -= 1
                raise exceptions.NackError("broker nacked the message")
            targets = BROKER.route(exchange, routing_key)
            if not targets and mandatory and self.confirm:
                raise exceptions.UnroutableError(f"unroutable: {exchange}/{routing_key}")
            for q in targets:
                q.ready.append((body if isinstance(body, bytes) else str(body).encode(), False))
            BROKER.published += 1

    def basic_consume(self, queue, on_message_callback, auto_ack=False, **_):
        self._check()
        with BROKER.lock:
            if queue not in BROKER.queues:
                raise exceptions.ChannelClosedByBroker("NOT_FOUND")
            tag = f"ctag-{next(BROKER._names)}"
            self.consumers.append((queue, on_message_callback, auto_ack))
        return tag

    def basic_ack(self, delivery_tag, multiple=False):
        self._check()
        with BROKER.lock:
            if self.unacked.pop(delivery_tag, None) is None:
                raise exceptions.ChannelClosedByBroker("PRECONDITION_FAILED - unknown delivery tag")

    def basic_nack(self, delivery_tag, multiple=False, requeue=True):
        self._check()
        with BROKER.lock:
            item = self.unacked.pop(delivery_tag, None)
            if item is None:
                raise exceptions.ChannelClosedByBroker("PRECONDITION_FAILED - unknown delivery tag")
            if requeue:
                item[0].ready.append((item[1], True))

    def basic_get(self, queue, auto_ack=False):
        self._check()
        with BROKER.lock:
            q = BROKER.queues.get(queue)
            if q is None:
                raise exceptions.ChannelClosedByBroker(f"NOT_FOUND - no queue '{queue}'")
            if not q.ready:
                return None, None, None
            body, redelivered = q.ready.popleft()
            tag = next(self._tags)
            if not auto_ack:
                self.unacked[tag] = (q, body)
            method = types.SimpleNamespace(delivery_tag=tag, redelivered=redelivered, message_count=len(q.ready))
            return method, BasicProperties(), body

    def _next_delivery(self):
        """One (callback, method, body) this channel may take now, or None (prefetch, empty queues)."""
        with BROKER.lock:
            for queue, cb, auto_ack in self.consumers:
                if not auto_ack and self.prefetch and len(self.unacked) >= self.prefetch:
                    return None
                q = BROKER.queues.get(queue)
                if q is None or not q.ready:
                    continue
                body, redelivered = q.ready.popleft()
                tag = next(self._tags)
                if not auto_ack:
                    self.unacked[tag] = (q, body)
                method = types.SimpleNamespace(delivery_tag=tag, redelivered=redelivered, routing_key=queue)
                return cb, method, body
        return None


class BlockingConnection:
    def __init__(self, parameters=None):
        with BROKER.lock:
            if not BROKER.up:
                raise exceptions.AMQPConnectionError("connection refused")
            BROKER.connections.append(self)
        self.params, self._dead, self._closed = parameters, False, False
        self.channels: list[BlockingChannel] = []

    @property
    def is_closed(self):
        return self._closed or self._dead

    @property
    def is_open(self):
        return not self.is_closed

    def channel(self):
        if self.is_closed:
            raise exceptions.StreamLostError("connection lost")
        ch = BlockingChannel(self)
        self.channels.append(ch)
        return ch

    def _die(self):
        self._dead = True
        for ch in self.channels:
            ch._requeue_all()
            ch.is_open = False
        self._drop_exclusive()

    def _drop_exclusive(self):
        with BROKER.lock:
            for name in [n for n, q in BROKER.queues.items() if q.exclusive_to is self]:
                del BROKER.queues[name]
                BROKER.bindings = [b for b in BROKER.bindings if b[1] != name]
            if self in BROKER.connections:
                BROKER.connections.remove(self)

    def close(self):
        if self._dead:
            raise exceptions.StreamLostError("connection lost")
        for ch in self.channels:
            if ch.is_open:
                ch.close()
        self._closed = True
        self._drop_exclusive()

    def process_data_events(self, time_limit=0):
        end = time.monotonic() + float(time_limit or 0)
        while True:
            if self._dead:
                raise exceptions.StreamLostError("connection lost")
            got = False
            for ch in list(self.channels):
                if not ch.is_open:
                    continue
                d = ch._next_delivery()
                if d is not None:
                    cb, method, body = d
                    cb(ch, method, BasicProperties(), body)
                    got = True
            if time.monotonic() >= end:
                return
            if not got:
                time.sleep(0.005)


def install(monkeypatch):
    """Make ``import pika`` resolve to this module (and reset the broker)."""
    import sys
    BROKER.reset()
    mod = sys.modules[__name__]
    monkeypatch.setitem(sys.modules, "pika", mod)
    monkeypatch.setitem(sys.modules, "pika.exceptions", exceptions)
    return BROKER
