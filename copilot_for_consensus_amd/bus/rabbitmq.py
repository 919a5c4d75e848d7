"""RabbitMQ driver (optional; needs ``pika``, which this image does not ship).

Kept for deployment parity with the reference (rabbitmq_publisher.py:25, rabbitmq_subscriber.py:28):
topic exchange ``copilot.events``, durable queues bound per routing key, persistent messages with
publisher confirms, manual ack / nack(requeue) and a reconnecting consume loop.
"""
from __future__ import annotations

import json
import time
from typing import Any

from ..contracts.events import EXCHANGE, ROUTING_KEYS
from .base import Callback, EventPublisher, EventSubscriber


def _pika():
    try:
        import pika  # type: ignore
    except ImportError as e:  # pragma: no cover - environment dependent
        raise ImportError("MESSAGE_BUS_TYPE=rabbitmq needs the 'pika' package; use MESSAGE_BUS_TYPE=inproc "
                          "for single-node deployments") from e
    return pika


def _params(pika, host, port, username, password, heartbeat, blocked_connection_timeout):
    creds = pika.PlainCredentials(username or "guest", password or "guest")
    return pika.ConnectionParameters(host=host, port=int(port), credentials=creds, heartbeat=heartbeat,
                                     blocked_connection_timeout=blocked_connection_timeout)


class RabbitMQPublisher(EventPublisher):
    def __init__(self, rabbitmq_host="messagebus", rabbitmq_port=5672, rabbitmq_username=None, rabbitmq_password=None,
                 exchange=EXCHANGE, exchange_type="topic", heartbeat=300, blocked_connection_timeout=600, **_):
        self.pika = _pika()
        self.params = _params(self.pika, rabbitmq_host, rabbitmq_port, rabbitmq_username, rabbitmq_password, heartbeat,
                              blocked_connection_timeout)
        self.exchange, self.exchange_type = exchange, exchange_type
        self.conn = self.ch = None

    def connect(self) -> None:
        self.conn = self.pika.BlockingConnection(self.params)
        self.ch = self.conn.channel()
        self.ch.confirm_delivery()
        self.ch.exchange_declare(exchange=self.exchange, exchange_type=self.exchange_type, durable=True)

    def disconnect(self) -> None:
        if self.conn and self.conn.is_open:
            self.conn.close()

    def publish(self, exchange: str, routing_key: str, event: dict[str, Any]) -> None:
        body = json.dumps(event).encode()
        props = self.pika.BasicProperties(delivery_mode=2, content_type="application/json")
        for attempt in range(2):  # reconnect and retry once
            try:
                if self.ch is None or self.ch.is_closed:
                    self.connect()
                self.ch.basic_publish(exchange=exchange or self.exchange, routing_key=routing_key, body=body,
                                      properties=props, mandatory=False)
                return
            except Exception:
                if attempt:
                    raise
                self.ch = None


class RabbitMQSubscriber(EventSubscriber):
    def __init__(self, rabbitmq_host="messagebus", rabbitmq_port=5672, rabbitmq_username=None, rabbitmq_password=None,
                 exchange=EXCHANGE, queue_name=None, queue_durable=True, auto_ack=False, heartbeat=300,
                 blocked_connection_timeout=600, **_):
        self.pika = _pika()
        self.params = _params(self.pika, rabbitmq_host, rabbitmq_port, rabbitmq_username, rabbitmq_password, heartbeat,
                              blocked_connection_timeout)
        self.exchange, self.queue_name, self.durable, self.auto_ack = exchange, queue_name, queue_durable, auto_ack
        self.callbacks: dict[str, Callback] = {}
        self.bindings: list[str] = []
        self._stop = False
        self.conn = self.ch = None

    def connect(self) -> None:
        self.conn = self.pika.BlockingConnection(self.params)
        self.ch = self.conn.channel()
        self.ch.exchange_declare(exchange=self.exchange, exchange_type="topic", durable=True)
        res = self.ch.queue_declare(queue=self.queue_name or "", durable=self.durable, exclusive=not self.queue_name)
        self.queue_name = res.method.queue
        for key in self.bindings:
            self.ch.queue_bind(queue=self.queue_name, exchange=self.exchange, routing_key=key)

    def disconnect(self) -> None:
        if self.conn and self.conn.is_open:
            self.conn.close()

    def subscribe(self, event_type: str, callback: Callback, routing_key: str | None = None,
                  exchange: str | None = None) -> None:
        self.callbacks[event_type] = callback
        key = routing_key or ROUTING_KEYS.get(event_type, event_type)
        self.bindings.append(key)
        if self.ch is not None:
            self.ch.queue_bind(queue=self.queue_name, exchange=exchange or self.exchange, routing_key=key)

    def _on_message(self, ch, method, _props, body):
        try:
            event = json.loads(body)
            cb = self.callbacks.get(event.get("event_type"))
        except ValueError:
            ch.basic_ack(method.delivery_tag)  # malformed: drop
            return
        try:
            if cb:
                cb(event)
            if not self.auto_ack:
                ch.basic_ack(method.delivery_tag)
        except Exception:
            if not self.auto_ack:
                ch.basic_nack(method.delivery_tag, requeue=True)

    def start_consuming(self) -> None:
        self._stop = False
        backoff = 1.0
        while not self._stop:
            try:
                if self.ch is None or self.ch.is_closed:
                    self.connect()
                self.ch.basic_qos(prefetch_count=1)
                self.ch.basic_consume(queue=self.queue_name, on_message_callback=self._on_message,
                                      auto_ack=self.auto_ack)
                while not self._stop:
                    self.conn.process_data_events(time_limit=0.5)
                backoff = 1.0
            except Exception:
                self.ch = None
                time.sleep(backoff)
                backoff = min(backoff * 2, 30.0)

    def stop_consuming(self) -> None:
        self._stop = True
