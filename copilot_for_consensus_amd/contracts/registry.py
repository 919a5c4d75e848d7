"""Schema provider: events, documents and service configuration schemas by name.

Counterpart of the reference's FileSchemaProvider / create_schema_provider
(adapters/copilot_schema_validation/copilot_schema_validation/file_schema_provider.py:18,48) and
the versioned registry (schema_registry.py:113-296).  Schemas are generated in memory; ``export``
writes them as files (``docs/schemas/...``) for external consumers.
"""
from __future__ import annotations

import json
from pathlib import Path

from . import documents, events
from .validator import SchemaRegistry, iter_errors


class SchemaProvider:
    def __init__(self):
        self.registry = SchemaRegistry()
        self.registry.add(events.envelope_schema(), "event-envelope.schema.json", "event-envelope")
        self._events = {}
        for t in events.EVENT_TYPES:
            sch = events.event_schema(t)
            self._events[t] = sch
            self.registry.add(sch, t)
        self._docs = {c: documents.document_schema(c) for c in documents.COLLECTIONS}
        for c, sch in self._docs.items():
            self.registry.add(sch, c)

    def get_event_schema(self, event_type: str) -> dict | None:
        return self._events.get(event_type)

    def get_document_schema(self, collection: str) -> dict | None:
        return self._docs.get(collection)

    def list_event_types(self) -> list[str]:
        return list(self._events)

    def validate_event(self, event: dict) -> list[str]:
        sch = self._events.get(event.get("event_type"))
        if sch is None:
            return [f"unknown event_type {event.get('event_type')!r}"]
        return iter_errors(event, sch, self.registry)

    def validate_document(self, collection: str, doc: dict) -> list[str]:
        sch = self._docs.get(collection)
        return [] if sch is None else iter_errors(doc, sch, self.registry)

    def export(self, root: str | Path) -> list[Path]:
        root = Path(root)
        out = []
        ev = root / "events"
        ev.mkdir(parents=True, exist_ok=True)
        p = ev / "event-envelope.schema.json"
        p.write_text(json.dumps(events.envelope_schema(), indent=2) + "\n")
        out.append(p)
        for t, sch in self._events.items():
            p = ev / f"{t}.schema.json"
            p.write_text(json.dumps(sch, indent=2) + "\n")
            out.append(p)
        dd = root / "documents" / "v1"
        dd.mkdir(parents=True, exist_ok=True)
        for c, sch in self._docs.items():
            p = dd / f"{c}.schema.json"
            p.write_text(json.dumps(sch, indent=2) + "\n")
            out.append(p)
        p = dd / "collections.config.json"
        p.write_text(json.dumps(documents.collections_config(), indent=2) + "\n")
        out.append(p)
        return out


_default: SchemaProvider | None = None


def default_provider() -> SchemaProvider:
    global _default
    if _default is None:
        _default = SchemaProvider()
    return _default


def create_schema_provider(kind: str = "generated", **_) -> SchemaProvider:
    """Factory kept for API parity (the reference also supports a Mongo-backed provider)."""
    return default_provider()
