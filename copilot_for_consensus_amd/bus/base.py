"""Message-bus interfaces (API of adapters/copilot_message_bus/copilot_message_bus/base.py:15-94).

``EventPublisher.publish(exchange, routing_key, event)`` and ``EventSubscriber.subscribe(
event_type, callback, routing_key=None, exchange=None) / start_consuming() / stop_consuming()``
keep the reference's signatures so services are written exactly as there.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Callable

Callback = Callable[[dict[str, Any]], None]


class EventPublisher(ABC):
    @abstractmethod
    def publish(self, exchange: str, routing_key: str, event: dict[str, Any]) -> None:
        """Publish ``event`` (envelope dict); raises on failure."""

    def connect(self) -> None:
        pass

    def disconnect(self) -> None:
        pass


class EventSubscriber(ABC):
    @abstractmethod
    def subscribe(self, event_type: str, callback: Callback, routing_key: str | None = None,
                  exchange: str | None = None) -> None:
        ...

    @abstractmethod
    def start_consuming(self) -> None:
        """Block, dispatching events to callbacks, until stop_consuming()."""

    @abstractmethod
    def stop_consuming(self) -> None:
        ...

    def connect(self) -> None:
        pass

    def disconnect(self) -> None:
        pass


def topic_matches(pattern: str, key: str) -> bool:
    """AMQP topic match: '*' = exactly one word, '#' = zero or more words."""
    p, k = pattern.split("."), key.split(".")

    def rec(i: int, j: int) -> bool:
        if i == len(p):
            return j == len(k)
        if p[i] == "#":
            return any(rec(i + 1, jj) for jj in range(j, len(k) + 1))
        if j == len(k):
            return False
        return (p[i] == "*" or p[i] == k[j]) and rec(i + 1, j + 1)

    return rec(0, 0)
