"""Operate on failed-event queues: list / inspect / export / requeue / purge.

Parity target: scripts/manage_failed_queues.py of the reference (FailedQueueManager :40 with
QUEUE_MAPPINGS :44-52, list :98, inspect :125, export :183, requeue :230 with --dry-run, purge
:303 with --limit/--confirm).  Two backends behind one manager:
  * :class:`InProcFailedQueues` -- the in-process broker: ``<queue>.dlq`` dead letters (events that
    exhausted redeliveries) plus queues bound to the ``*.failed`` routing keys;
  * :class:`RabbitMQFailedQueues` -- pika ``basic_get`` / ``basic_publish`` (import-gated);
  * ``bus.cfcbroker.CfcBrokerFailedQueues`` -- the native broker (``--backend cfcbroker``).
Requeue republishes each message on the target routing key (the mapping, ``--target``, or for a
dead letter its own routing key) and removes it from the failed queue only after the publish.

Reference: scripts/manage_failed_queues.py:98-303 (list / inspect / export / requeue / purge).
"""
from __future__ import annotations

import argparse
import json
import sys
from datetime import datetime, timezone
from typing import Any

from ..contracts.events import EVENT_SPECS, routing_key_for

EXCHANGE = "copilot.events"

QUEUE_MAPPINGS = {
    "archive.ingestion.failed": "archive.ingested",
    "parsing.failed": "archive.ingested",
    "chunking.failed": "json.parsed",
    "embedding.generation.failed": "chunks.prepared",
    "summarization.failed": "summarization.requested",
    "orchestration.failed": "embeddings.generated",
    "report.delivery.failed": "summary.complete",
}


def failed_routing_keys() -> list[str]:
    return sorted(routing_key_for(t) for t in EVENT_SPECS if t.endswith("Failed"))


class InProcFailedQueues:
    def __init__(self, broker):
        self.broker = broker
        for rk in failed_routing_keys():       # make failures observable from now on
            if rk not in broker.queues():
                broker.declare_queue(rk)
                broker.bind(rk, EXCHANGE, rk)

    def names(self) -> list[str]:
        return sorted(set(failed_routing_keys()) | {f"{q}.dlq" for q, v in self.broker.dead_letters.items() if v})

    def _items(self, name: str) -> list:
        if name.endswith(".dlq"):
            return self.broker.dead_letters[name[:-4]]
        return self.broker.declare_queue(name).items

    @staticmethod
    def _decode(it) -> dict:
        if isinstance(it, list):          # live queue entry: [routing_key, body, redeliveries]
            it = it[1]
        return json.loads(it) if isinstance(it, (bytes, str)) else it

    def peek(self, name: str, limit: int) -> list[dict]:
        return [self._decode(it) for it in list(self._items(name))[:limit]]

    def pop(self, name: str) -> dict | None:
        items = self._items(name)
        if not items:
            return None
        return self._decode(items.popleft() if hasattr(items, "popleft") else items.pop(0))

    def count(self, name: str) -> int:
        return len(self._items(name))

    def publish(self, routing_key: str, event: dict) -> None:
        self.broker.publish(EXCHANGE, routing_key, json.dumps(event).encode())


class RabbitMQFailedQueues:
    def __init__(self, host="localhost", port=5672, username="guest", password="guest", vhost="/"):
        import pika  # noqa: F401 -- optional dependency
        self._pika = pika
        cred = pika.PlainCredentials(username, password)
        self.conn = pika.BlockingConnection(pika.ConnectionParameters(host, port, vhost, cred))
        self.ch = self.conn.channel()

    def names(self):
        return sorted(QUEUE_MAPPINGS)

    def count(self, name):
        """Ready messages, or None when the queue does not exist.  A passive declare of a missing
        queue makes the broker close the channel (404), so a fresh one is opened for the next call."""
        try:
            return self.ch.queue_declare(queue=name, durable=True, passive=True).method.message_count
        except Exception:  # noqa: BLE001 -- pika's ChannelClosedByBroker; the SDK is optional
            self.ch = self.conn.channel()
            return None

    def peek(self, name, limit):
        out, tags = [], []
        for _ in range(limit):
            m, _, body = self.ch.basic_get(name, auto_ack=False)
            if m is None:
                break
            tags.append(m.delivery_tag)
            out.append(json.loads(body))
        for t in tags:
            self.ch.basic_nack(t, requeue=True)
        return out

    def pop(self, name):
        m, _, body = self.ch.basic_get(name, auto_ack=True)
        return None if m is None else json.loads(body)

    def publish(self, routing_key, event):
        self.ch.basic_publish(EXCHANGE, routing_key, json.dumps(event).encode(),
                              self._pika.BasicProperties(content_type="application/json", delivery_mode=2))


class FailedQueueManager:
    def __init__(self, backend):
        self.b = backend

    def list_failed_queues(self) -> list[dict[str, Any]]:
        rows = [{"queue": n, "message_count": self.b.count(n), "target": QUEUE_MAPPINGS.get(n)} for n in self.b.names()]
        return [r for r in rows if r["message_count"] is not None]     # absent queues skipped, as the reference

    def inspect_messages(self, queue: str, limit: int = 10) -> list[dict]:
        return self.b.peek(queue, limit)

    def export_messages(self, queue: str, path: str, limit: int = 1000) -> int:
        msgs = self.b.peek(queue, limit)
        with open(path, "w", encoding="utf-8") as fh:
            json.dump({"queue": queue, "exported_at": datetime.now(timezone.utc).isoformat(), "message_count": len(msgs),
                       "messages": msgs}, fh, indent=2)
        return len(msgs)

    def _target(self, queue: str, event: dict, target: str | None) -> str:
        if target:
            return target
        if queue.endswith(".dlq"):
            return routing_key_for(event["event_type"])
        if queue in QUEUE_MAPPINGS:
            return QUEUE_MAPPINGS[queue]
        raise ValueError(f"Unknown failed queue: {queue}. Specify --target.")

    def requeue_messages(self, queue: str, target: str | None = None, limit: int | None = None,
                         dry_run: bool = False) -> int:
        n = self.b.count(queue) if limit is None else min(limit, self.b.count(queue))
        if dry_run:
            for ev in self.b.peek(queue, n):
                self._target(queue, ev, target)
            return n
        done = 0
        for _ in range(n):
            ev = self.b.pop(queue)
            if ev is None:
                break
            try:
                self.b.publish(self._target(queue, ev, target), ev)
            except Exception:
                self.b.publish(queue, ev)   # put it back rather than lose it
                raise
            done += 1
        return done

    def purge_messages(self, queue: str, limit: int | None = None, dry_run: bool = False) -> int:
        n = self.b.count(queue) if limit is None else min(limit, self.b.count(queue))
        if dry_run:
            return n
        for _ in range(n):
            self.b.pop(queue)
        return n


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Manage failed-event queues (RabbitMQ or the native cfc-broker)")
    ap.add_argument("--backend", choices=["rabbitmq", "cfcbroker"], default="rabbitmq")
    ap.add_argument("--host", default="localhost")
    ap.add_argument("--port", type=int, default=None, help="default 5672 (rabbitmq) / 5680 (cfcbroker)")
    ap.add_argument("--username", default="guest")
    ap.add_argument("--password", default="guest")
    sub = ap.add_subparsers(dest="cmd", required=True)
    sub.add_parser("list")
    p = sub.add_parser("inspect"); p.add_argument("queue"); p.add_argument("--limit", type=int, default=10)
    p = sub.add_parser("export"); p.add_argument("queue"); p.add_argument("--output", required=True)
    p.add_argument("--limit", type=int, default=1000)
    p = sub.add_parser("requeue"); p.add_argument("queue"); p.add_argument("--target")
    p.add_argument("--limit", type=int); p.add_argument("--dry-run", action="store_true")
    p = sub.add_parser("purge"); p.add_argument("queue"); p.add_argument("--limit", type=int)
    p.add_argument("--dry-run", action="store_true"); p.add_argument("--confirm", action="store_true")
    a = ap.parse_args(argv)
    if a.backend == "cfcbroker":
        from ..bus.cfcbroker import CfcBrokerFailedQueues
        m = FailedQueueManager(CfcBrokerFailedQueues(a.host, a.port or 5680))
    else:
        m = FailedQueueManager(RabbitMQFailedQueues(a.host, a.port or 5672, a.username, a.password))
    if a.cmd == "list":
        print(json.dumps(m.list_failed_queues(), indent=2))
    elif a.cmd == "inspect":
        print(json.dumps(m.inspect_messages(a.queue, a.limit), indent=2))
    elif a.cmd == "export":
        print(m.export_messages(a.queue, a.output, a.limit))
    elif a.cmd == "requeue":
        print(m.requeue_messages(a.queue, a.target, a.limit, a.dry_run))
    elif a.cmd == "purge":
        if not (a.confirm or a.dry_run):
            print("refusing to purge without --confirm", file=sys.stderr)
            return 2
        print(m.purge_messages(a.queue, a.limit, a.dry_run))
    return 0


if __name__ == "__main__":
    sys.exit(main())
