"""RabbitMQ driver (needs ``pika``, which this image does not ship; tests drive it with a stand-in).

Deployment parity with the reference's default bus (rabbitmq_publisher.py:25, rabbitmq_subscriber.py:
28), same observable behaviour:

* publisher: durable topic exchange ``copilot.events``; persistent JSON messages published with
  ``mandatory=True`` under publisher confirms, so an unroutable message (no queue bound) raises
  ``UnroutableError`` and a broker nack raises ``NackError`` instead of being lost silently
  (rabbitmq_publisher.py:334-424); ``declare_queue(s)`` creates durable queues bound to their
  routing key and re-declares them after a reconnect (:239-301); a broken connection is reopened
  under an exponential-backoff circuit breaker with a cap on consecutive attempts (:185-250) and
  the publish retried once.
* subscriber: durable named queue (or an exclusive server-named one), one binding per subscribed
  routing key; ``prefetch_count`` unacked deliveries; manual acks; a callback that raises nacks
  the message back onto the queue (requeue), an envelope without ``event_type`` or with bad JSON
  is acked and dropped so it cannot block the queue, any other failure is nacked without requeue
  (dead-lettered by broker policy) -- rabbitmq_subscriber.py:504-560; acks / nacks on a channel
  that has closed meanwhile are swallowed (the broker redelivers) (:562-610); the consume loop
  reconnects on connection / channel loss, re-registering the consumer once per channel
  (:376-476).
"""
from __future__ import annotations

import json
import logging
import time
from typing import Any

from ..contracts.events import EXCHANGE, ROUTING_KEYS
from .base import Callback, EventPublisher, EventSubscriber

log = logging.getLogger(__name__)


def _pika():
    try:
        import pika  # type: ignore
    except ImportError as e:  # pragma: no cover - environment dependent
        raise ImportError("MESSAGE_BUS_TYPE=rabbitmq needs the 'pika' package; use MESSAGE_BUS_TYPE=cfcbroker "
                          "(native broker) or inproc") from e
    return pika


def _params(pika, host, port, username, password, heartbeat, blocked_connection_timeout):
    creds = pika.PlainCredentials(username or "guest", password or "guest")
    return pika.ConnectionParameters(host=host, port=int(port), credentials=creds, heartbeat=heartbeat,
                                     blocked_connection_timeout=blocked_connection_timeout,
                                     connection_attempts=3, retry_delay=2)


def _connection_errors(pika) -> tuple[type[BaseException], ...]:
    ex = pika.exceptions
    names = ("ChannelWrongStateError", "ChannelClosedByBroker", "ConnectionClosedByBroker", "AMQPConnectionError",
             "StreamLostError", "ChannelClosed", "ConnectionClosed")
    return tuple(getattr(ex, n) for n in names if hasattr(ex, n)) + (ConnectionError,)


class _Link:
    """Connection + channel with the reconnect circuit breaker both directions share."""

    def __init__(self, params, reconnect_delay: float, max_reconnect_attempts: int, clock=time.monotonic):
        self.params, self.delay, self.max_attempts, self.clock = params, float(reconnect_delay), \
            int(max_reconnect_attempts), clock
        self.conn = self.ch = None
        self.failures = 0
        self._last_attempt = None

    def is_open(self) -> bool:
        try:
            return (self.conn is not None and not self.conn.is_closed and self.ch is not None
                    and self.ch.is_open)
        except Exception:  # noqa: BLE001 -- a half-torn-down pika object counts as closed
            return False

    def close(self) -> None:
        for obj in (self.ch, self.conn):
            try:
                if obj is not None and obj.is_open:
                    obj.close()
            except Exception:  # noqa: BLE001
                pass
        self.conn = self.ch = None

    def may_retry(self) -> bool:
        """Throttle: the n-th consecutive attempt waits delay * 2^n (cap 60 s); give up after max."""
        if self.failures >= self.max_attempts:
            return False
        if self._last_attempt is None or self.failures == 0:
            return True
        return self.clock() - self._last_attempt >= min(self.delay * 2 ** self.failures, 60.0)

    def attempt(self, open_fn) -> bool:
        if not self.may_retry():
            return False
        self._last_attempt = self.clock()
        self.close()
        try:
            open_fn()
        except Exception as e:  # noqa: BLE001
            self.failures += 1
            log.warning("rabbitmq reconnect %d/%d failed: %s", self.failures, self.max_attempts, e)
            self.close()
            return False
        self.failures = 0
        return True


class RabbitMQPublisher(EventPublisher):
    def __init__(self, rabbitmq_host="messagebus", rabbitmq_port=5672, rabbitmq_username=None, rabbitmq_password=None,
                 exchange=EXCHANGE, exchange_type="topic", heartbeat=300, blocked_connection_timeout=600,
                 enable_publisher_confirms=True, reconnect_delay=1.0, max_reconnect_attempts=10, **_):
        self.pika = _pika()
        self.params = _params(self.pika, rabbitmq_host, rabbitmq_port, rabbitmq_username, rabbitmq_password, heartbeat,
                              blocked_connection_timeout)
        self.exchange, self.exchange_type, self.confirms = exchange, exchange_type, bool(enable_publisher_confirms)
        self.link = _Link(self.params, reconnect_delay, max_reconnect_attempts)
        self.declared: dict[str, tuple[str, str]] = {}
        self.published = 0

    @property
    def ch(self):
        return self.link.ch

    def connect(self) -> None:
        link = self.link
        link.conn = self.pika.BlockingConnection(self.params)
        link.ch = link.conn.channel()
        if self.confirms:
            link.ch.confirm_delivery()
        link.ch.exchange_declare(exchange=self.exchange, exchange_type=self.exchange_type, durable=True)

    def _reconnect(self) -> bool:
        if not self.link.attempt(self.connect):
            return False
        for q, (key, ex) in list(self.declared.items()):
            self.declare_queue(q, key, ex)
        return True

    def disconnect(self) -> None:
        self.link.close()

    def declare_queue(self, queue_name: str, routing_key: str | None = None, exchange: str | None = None) -> None:
        """Durable queue bound to ``routing_key`` (default: the queue name); remembered so a reconnect
        re-declares it before the next publish."""
        if not self.link.is_open():
            raise ConnectionError("not connected to RabbitMQ")
        key, ex = routing_key or queue_name, exchange or self.exchange
        self.link.ch.queue_declare(queue=queue_name, durable=True, auto_delete=False, exclusive=False)
        self.link.ch.queue_bind(exchange=ex, queue=queue_name, routing_key=key)
        self.declared[queue_name] = (key, ex)

    def declare_queues(self, queues: list[dict[str, str | None]]) -> bool:
        ok = True
        for q in queues:
            name = q.get("queue_name")
            if not name:
                ok = False
                continue
            try:
                self.declare_queue(name, q.get("routing_key"), q.get("exchange"))
            except Exception as e:  # noqa: BLE001 -- reported through the return value, like the reference
                log.error("declare %s failed: %s", name, e)
                ok = False
        return ok

    def _send(self, exchange: str, routing_key: str, body: bytes) -> None:
        props = self.pika.BasicProperties(delivery_mode=2, content_type="application/json")
        self.link.ch.basic_publish(exchange=exchange or self.exchange, routing_key=routing_key, body=body,
                                   properties=props, mandatory=True)

    def publish(self, exchange: str, routing_key: str, event: dict[str, Any]) -> None:
        body = json.dumps(event).encode()
        if not self.link.is_open() and not self._reconnect():
            raise ConnectionError("not connected to RabbitMQ and reconnection failed")
        try:
            self._send(exchange, routing_key, body)
        except _connection_errors(self.pika) as e:
            if not self._reconnect():
                raise ConnectionError(f"publish failed after connection error: {e}") from e
            self._send(exchange, routing_key, body)     # once; UnroutableError / NackError propagate
        self.published += 1


class RabbitMQSubscriber(EventSubscriber):
    def __init__(self, rabbitmq_host="messagebus", rabbitmq_port=5672, rabbitmq_username=None, rabbitmq_password=None,
                 exchange=EXCHANGE, exchange_name=None, exchange_type="topic", queue_name=None, queue_durable=True,
                 auto_ack=False, heartbeat=300, blocked_connection_timeout=600, prefetch_count=1,
                 reconnect_delay=1.0, max_reconnect_attempts=10, **_):
        self.pika = _pika()
        self.params = _params(self.pika, rabbitmq_host, rabbitmq_port, rabbitmq_username, rabbitmq_password, heartbeat,
                              blocked_connection_timeout)
        self.exchange, self.exchange_type = exchange_name or exchange, exchange_type
        self.queue_name, self.durable, self.auto_ack = queue_name, bool(queue_durable), bool(auto_ack)
        self.prefetch = int(prefetch_count)
        self.callbacks: dict[str, Callback] = {}
        self.bindings: list[tuple[str, str]] = []
        self.link = _Link(self.params, reconnect_delay, max_reconnect_attempts)
        self._stop = False
        self._consumer_channel = None
        self._connected_once = False
        self.stats = {"acked": 0, "requeued": 0, "rejected": 0, "dropped": 0, "reconnects": 0}

    @property
    def ch(self):
        return self.link.ch

    def connect(self) -> None:
        link = self.link
        link.conn = self.pika.BlockingConnection(self.params)
        link.ch = link.conn.channel()
        self._connected_once = True
        link.ch.exchange_declare(exchange=self.exchange, exchange_type=self.exchange_type, durable=True)
        if self.queue_name:
            link.ch.queue_declare(queue=self.queue_name, durable=self.durable)
        else:
            res = link.ch.queue_declare(queue="", exclusive=True, auto_delete=True)
            self.queue_name = res.method.queue
        for key, ex in self.bindings:
            link.ch.queue_bind(queue=self.queue_name, exchange=ex, routing_key=key)
        link.ch.basic_qos(prefetch_count=self.prefetch)

    def disconnect(self) -> None:
        self.link.close()

    def subscribe(self, event_type: str, callback: Callback, routing_key: str | None = None,
                  exchange: str | None = None) -> None:
        self.callbacks[event_type] = callback
        b = (routing_key or ROUTING_KEYS.get(event_type, event_type), exchange or self.exchange)
        if b not in self.bindings:
            self.bindings.append(b)
            if self.link.is_open():
                self.link.ch.queue_bind(queue=self.queue_name, exchange=b[1], routing_key=b[0])

    # -- delivery handling ---------------------------------------------------------------------
    def _settle(self, ch, tag, ok: bool, requeue: bool = True) -> None:
        if self.auto_ack:
            return
        try:
            if ok:
                ch.basic_ack(delivery_tag=tag)
            else:
                ch.basic_nack(delivery_tag=tag, requeue=requeue)
        except Exception as e:  # noqa: BLE001 -- channel closed under us: the broker redelivers
            log.warning("rabbitmq %s of delivery %s lost with the channel: %s", "ack" if ok else "nack", tag, e)

    def _on_message(self, ch, method, _props, body) -> None:
        tag = method.delivery_tag
        try:
            event = json.loads(body.decode("utf-8") if isinstance(body, (bytes, bytearray)) else body)
            etype = event.get("event_type") if isinstance(event, dict) else None
        except (ValueError, UnicodeDecodeError):
            self.stats["dropped"] += 1
            self._settle(ch, tag, True)          # malformed: ack so it cannot block the queue
            return
        if not etype:
            self.stats["dropped"] += 1
            self._settle(ch, tag, True)
            return
        cb = self.callbacks.get(etype)
        try:
            if cb is not None:
                cb(event)
        except Exception as e:  # noqa: BLE001 -- handler failure: back onto the queue for a retry
            log.error("callback for %s failed: %s", etype, e)
            self.stats["requeued"] += 1
            self._settle(ch, tag, False, requeue=True)
            return
        self.stats["acked"] += 1
        self._settle(ch, tag, True)

    # -- consume loop ----------------------------------------------------------------------------
    def _handled(self) -> int:
        st = self.stats
        return st["acked"] + st["requeued"] + st["dropped"]

    def _ensure_consumer(self) -> None:
        ch = self.link.ch
        if self._consumer_channel is not ch:              # one consumer per channel instance
            ch.basic_consume(queue=self.queue_name, on_message_callback=self._on_message, auto_ack=self.auto_ack)
            self._consumer_channel = ch

    def drain(self, quiet_s: float = 0.02) -> int:
        """Synchronous mode (Node.drain): handle deliveries until none arrives for ``quiet_s``."""
        if not self.link.is_open():
            self.connect()
        self._ensure_consumer()
        n0 = self._handled()
        while True:
            before = self._handled()
            self.link.conn.process_data_events(time_limit=quiet_s)
            if self._handled() == before:
                return self._handled() - n0

    def start_consuming(self) -> None:
        self._stop = False
        while not self._stop:
            if not self.link.is_open():
                if not self.link.attempt(self.connect):
                    time.sleep(0.1)
                    continue
                self.stats["reconnects"] += int(self._connected_once)
                self._connected_once = True
            try:
                self._ensure_consumer()
                while not self._stop:
                    self.link.conn.process_data_events(time_limit=0.2)
            except _connection_errors(self.pika) + (AssertionError,) as e:
                log.warning("rabbitmq consume loop lost its connection: %s; reconnecting", e)
                self.link.close()
                self._consumer_channel = None

    def stop_consuming(self) -> None:
        self._stop = True
