"""Schema-validating bus decorators (reference validating_publisher.py:121,
validating_subscriber.py:30): every published / received event is checked against the generated
JSON Schema of its type; invalid events raise (publish) or are rejected before the callback."""
from __future__ import annotations

import logging
from typing import Any

from ..contracts.registry import SchemaProvider, default_provider
from .base import Callback, EventPublisher, EventSubscriber

log = logging.getLogger(__name__)


class EventValidationError(ValueError):
    def __init__(self, event_type: str, errors: list[str]):
        super().__init__(f"{event_type}: {'; '.join(errors[:5])}")
        self.event_type = event_type
        self.errors = errors


class ValidatingEventPublisher(EventPublisher):
    def __init__(self, publisher: EventPublisher, schema_provider: SchemaProvider | None = None, strict: bool = True):
        self._inner = publisher
        self._schemas = schema_provider or default_provider()
        self.strict = strict

    def publish(self, exchange: str, routing_key: str, event: dict[str, Any]) -> None:
        errs = self._schemas.validate_event(event)
        if errs and self.strict:
            raise EventValidationError(str(event.get("event_type")), errs)
        self._inner.publish(exchange, routing_key, event)

    def connect(self) -> None:
        self._inner.connect()

    def disconnect(self) -> None:
        self._inner.disconnect()

    def __getattr__(self, name):
        return getattr(self._inner, name)


class ValidatingEventSubscriber(EventSubscriber):
    def __init__(self, subscriber: EventSubscriber, schema_provider: SchemaProvider | None = None, strict: bool = True):
        self._inner = subscriber
        self._schemas = schema_provider or default_provider()
        self.strict = strict
        self.rejected: list[tuple[dict, list[str]]] = []

    def subscribe(self, event_type: str, callback: Callback, routing_key: str | None = None,
                  exchange: str | None = None) -> None:
        def wrapper(event: dict[str, Any]) -> None:
            errs = self._schemas.validate_event(event)
            if errs:
                # strict: raise (the transport dead-letters it); non-strict: log and skip the
                # callback (reference validating_subscriber.py wrapper)
                self.rejected.append((event, errs))
                if self.strict:
                    raise EventValidationError(event_type, errs)
                log.warning("skipping invalid %s event: %s", event_type, "; ".join(errs[:3]))
                return
            callback(event)

        self._inner.subscribe(event_type, wrapper, routing_key=routing_key, exchange=exchange)

    def start_consuming(self) -> None:
        self._inner.start_consuming()

    def stop_consuming(self) -> None:
        self._inner.stop_consuming()

    def connect(self) -> None:
        self._inner.connect()

    def disconnect(self) -> None:
        self._inner.disconnect()

    def __getattr__(self, name):
        return getattr(self._inner, name)
