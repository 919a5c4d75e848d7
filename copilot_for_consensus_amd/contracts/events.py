"""Event envelope + the 17 pipeline event types (wire-compatible with the reference).

The envelope ``{event_type, event_id (uuid4), timestamp (ISO-8601 UTC), version, data}`` and the
payload fields/constraints of every event match docs/schemas/events/*.schema.json of the
reference (Python side: adapters/copilot_schema_validation/copilot_schema_validation/
models.py:41-492).  Here the payload specs are declared once, in a compact table, and the JSON
Schemas are GENERATED from it (``event_schema``), so the validator, the typed event classes and
the schema files on disk can never drift apart.

Routing key = dotted lower-case event type ("JSONParsed" -> "json.parsed"), exchange
``copilot.events`` (infra/rabbitmq/definitions.json of the reference).
"""
from __future__ import annotations

import random
import re
import threading
import uuid
from datetime import datetime, timezone
from typing import Any

_TLS = threading.local()


def _event_uuid() -> str:
    """A version-4 (random) UUID for an event id from a per-thread PRNG seeded once from the OS:
    ``uuid.uuid4()`` reads os.urandom on every call, a syscall per event on the bus's hot path.
    Event ids need uniqueness, not secrecy (nothing authenticates with them)."""
    rng = getattr(_TLS, "rng", None)
    if rng is None:
        rng = _TLS.rng = random.Random(int.from_bytes(uuid.uuid4().bytes, "big") ^ threading.get_ident())
    return str(uuid.UUID(int=rng.getrandbits(128), version=4))


SCHEMA_BASE = "https://alan-jowett.github.io/CoPilot-For-Consensus/schemas/events/"
EXCHANGE = "copilot.events"
EVENT_VERSION = "1.0"

# ---------------------------------------------------------------------------- field DSL

HEX_ID = {"type": "string", "pattern": "^[0-9a-f]{16,64}$"}


def s(min_len: int | None = 1, **kw) -> dict:
    d = {"type": "string", **kw}
    if min_len is not None:
        d["minLength"] = min_len
    return d


def i(minimum: int | None = 0) -> dict:
    return {"type": "integer"} if minimum is None else {"type": "integer", "minimum": minimum}


def num(minimum: float | None = 0) -> dict:
    return {"type": "number"} if minimum is None else {"type": "number", "minimum": minimum}


def arr(items: dict, **kw) -> dict:
    return {"type": "array", "items": items, **kw}


def obj(props: dict | None = None, required: list[str] | None = None, closed: bool = False) -> dict:
    d: dict[str, Any] = {"type": "object"}
    if props is not None:
        d["properties"] = props
    if required:
        d["required"] = required
    if closed:
        d["additionalProperties"] = False
    return d


DT = s(None, format="date-time")
UUID = s(None, format="uuid")
BOOL = {"type": "boolean"}
ARCHIVE_ID = {**HEX_ID, "minLength": 16, "maxLength": 64}
SOURCE_TYPE = {"type": "string", "enum": ["rsync", "imap", "http", "local"]}

SELECTED_CHUNK = obj({"chunk_id": {"type": "string"}, "source": {"type": "string"}, "score": num(None),
                      "rank": i(0), "metadata": obj()}, ["chunk_id", "source", "score", "rank"], closed=True)
CONTEXT_SELECTION = obj({"selector_type": {"type": "string"}, "selector_version": {"type": "string"},
                         "selection_params": obj(), "total_candidates": i(0), "total_tokens": i(0)},
                        ["selector_type", "selector_version"], closed=True)
CITATION = obj({"message_id": s(1), "chunk_id": HEX_ID, "offset": i(0), "text": {"type": "string"}},
               ["message_id", "chunk_id", "offset"], closed=True)

IDS1 = arr(HEX_ID, minItems=1, uniqueItems=True)  # non-empty, duplicate-free id lists
IDS0 = arr(HEX_ID, minItems=0, uniqueItems=True)
COUNTS = {"type": "object", "additionalProperties": {"type": "integer", "minimum": 0}}  # collection -> n deleted

# event type -> (required fields, optional fields); every payload is additionalProperties:false
EVENT_SPECS: dict[str, tuple[dict, dict]] = {
    "ArchiveIngested": ({
        "archive_id": ARCHIVE_ID, "source_name": s(), "source_type": SOURCE_TYPE, "source_url": s(),
        "file_size_bytes": i(), "file_hash_sha256": s(), "ingestion_started_at": DT, "ingestion_completed_at": DT,
    }, {"file_path": s()}),
    "ArchiveIngestionFailed": ({
        "source_name": s(), "source_type": SOURCE_TYPE, "source_url": s(), "error_message": s(), "error_type": s(),
        "retry_count": i(), "ingestion_started_at": DT, "failed_at": DT,
    }, {}),
    "JSONParsed": ({
        "archive_id": ARCHIVE_ID, "message_count": i(), "message_doc_ids": IDS1, "thread_count": i(),
        "thread_ids": IDS0, "parsing_duration_seconds": num(),
    }, {}),
    "ParsingFailed": ({
        "archive_id": ARCHIVE_ID, "error_message": s(), "error_type": s(), "messages_parsed_before_failure": i(),
        "retry_count": i(), "failed_at": DT,
    }, {"file_path": s()}),
    "ChunksPrepared": ({
        "message_doc_ids": IDS1, "chunk_count": i(), "chunk_ids": IDS1, "chunks_ready": BOOL,
        "chunking_strategy": s(), "avg_chunk_size_tokens": i(),
    }, {}),
    "ChunkingFailed": ({
        "message_doc_ids": IDS1, "error_message": s(), "error_type": s(), "retry_count": i(), "failed_at": DT,
    }, {}),
    "EmbeddingsGenerated": ({
        "chunk_ids": IDS1, "embedding_count": i(), "embedding_model": s(), "embedding_backend": s(),
        "embedding_dimension": i(1), "vector_store_collection": s(), "vector_store_updated": BOOL,
        "avg_generation_time_ms": num(),
    }, {}),
    "EmbeddingGenerationFailed": ({
        "chunk_ids": arr(s(), minItems=1, uniqueItems=True), "error_message": s(), "error_type": s(), "embedding_backend": s(), "retry_count": i(),
        "failed_at": DT,
    }, {}),
    "SummarizationRequested": ({
        "thread_ids": IDS1, "top_k": i(1), "prompt_template": s(),
    }, {"selected_chunks": arr(SELECTED_CHUNK), "context_selection": CONTEXT_SELECTION}),
    "OrchestrationFailed": ({
        "thread_ids": IDS1, "error_type": s(), "error_message": s(), "retry_count": i(),
    }, {}),
    "SummaryComplete": ({
        "summary_id": HEX_ID, "thread_id": HEX_ID, "summary_markdown": s(), "citations": arr(CITATION, minItems=0, uniqueItems=False),
        "llm_backend": s(), "llm_model": s(), "tokens_prompt": i(), "tokens_completion": i(), "latency_ms": i(),
    }, {}),
    "SummarizationFailed": ({
        "thread_id": HEX_ID, "error_type": s(), "error_message": s(), "retry_count": i(),
    }, {}),
    "ReportPublished": ({
        "thread_id": HEX_ID, "report_id": s(), "format": s(), "notified": BOOL, "delivery_channels": arr(s(), minItems=0, uniqueItems=True),
        "summary_url": s(),
    }, {}),
    "ReportDeliveryFailed": ({
        "report_id": s(), "thread_id": HEX_ID, "delivery_channel": s(), "error_message": s(), "error_type": s(),
        "retry_count": i(),
    }, {}),
    "SourceDeletionRequested": ({
        "source_name": s(), "correlation_id": UUID, "requested_at": DT,
    }, {"archive_ids": arr(HEX_ID), "delete_mode": {"type": "string", "enum": ["hard"]},
        "reason": {"type": "string"}, "requested_by": {"type": "string"}}),
    "SourceCleanupProgress": ({
        "source_name": s(), "correlation_id": UUID, "service_name": s(),
        "status": {"type": "string", "enum": ["started", "in_progress", "completed", "failed"]},
    }, {"deletion_counts": COUNTS, "error_summary": {"type": "string"}, "completed_at": DT}),
    "SourceCleanupCompleted": ({
        "source_name": s(), "correlation_id": UUID, "completed_at": DT, "total_deletion_counts": COUNTS,
        "services_completed": arr({"type": "string"}), "services_failed": arr({"type": "string"}),
        "overall_status": {"type": "string", "enum": ["success", "partial_success", "failed"]},
    }, {}),
}

EVENT_TYPES = tuple(EVENT_SPECS)


def routing_key_for(event_type: str) -> str:
    """PascalCase event type -> dotted routing key ("JSONParsed" -> "json.parsed")."""
    k = re.sub(r"([A-Z]+)([A-Z][a-z])", r"\1.\2", event_type)
    k = re.sub(r"([a-z\d])([A-Z])", r"\1.\2", k)
    return k.lower()


ROUTING_KEYS = {t: routing_key_for(t) for t in EVENT_TYPES}
EVENT_FOR_ROUTING_KEY = {v: k for k, v in ROUTING_KEYS.items()}


def _kebab(event_type: str) -> str:
    return routing_key_for(event_type).replace(".", "-")


def envelope_schema() -> dict:
    return {
        "$schema": "https://json-schema.org/draft/2020-12/schema",
        "$id": SCHEMA_BASE + "event-envelope.schema.json",
        "title": "Event Envelope",
        "type": "object",
        "properties": {"event_type": s(), "event_id": UUID, "timestamp": DT, "version": s(), "data": obj()},
        "required": ["event_type", "event_id", "timestamp", "version", "data"],
        "additionalProperties": False,
    }


def event_schema(event_type: str) -> dict:
    req, opt = EVENT_SPECS[event_type]
    data = {"type": "object", "properties": {**req, **opt}, "required": list(req), "additionalProperties": False}
    return {
        "$schema": "https://json-schema.org/draft/2020-12/schema",
        "$id": SCHEMA_BASE + f"{_kebab(event_type)}.schema.json",
        "title": f"{event_type} Event",
        "allOf": [
            {"$ref": "./event-envelope.schema.json"},
            # envelope fields repeated so additionalProperties:false is correct under strict Draft
            # 2020-12 semantics (the reference instead strips it at validation time,
            # schema_validator.py _strip_allof_additional_properties)
            {"type": "object", "properties": {"event_type": {"const": event_type}, "event_id": UUID, "timestamp": DT,
                                              "version": s(), "data": data},
             "required": ["event_type", "event_id", "timestamp", "version", "data"], "additionalProperties": False},
        ],
    }


def utc_now_iso() -> str:
    return datetime.now(timezone.utc).isoformat().replace("+00:00", "Z")


class Event:
    """A pipeline event: envelope + payload.  ``Event.create("JSONParsed", archive_id=...)``."""

    __slots__ = ("event_type", "data", "event_id", "timestamp", "version")

    def __init__(self, event_type: str, data: dict | None = None, event_id: str | None = None,
                 timestamp: str | None = None, version: str = EVENT_VERSION):
        if event_type not in EVENT_SPECS:
            raise ValueError(f"unknown event type {event_type!r}")
        self.event_type = event_type
        self.data = dict(data or {})
        self.event_id = event_id or _event_uuid()
        self.timestamp = timestamp or utc_now_iso()
        self.version = version

    @classmethod
    def create(cls, event_type: str, **data) -> "Event":
        return cls(event_type, data)

    @property
    def routing_key(self) -> str:
        return ROUTING_KEYS[self.event_type]

    def to_dict(self) -> dict:
        return {"event_type": self.event_type, "event_id": self.event_id, "timestamp": self.timestamp,
                "version": self.version, "data": dict(self.data)}

    @classmethod
    def from_dict(cls, d: dict) -> "Event":
        return cls(d["event_type"], d.get("data", {}), d.get("event_id"), d.get("timestamp"),
                   d.get("version", EVENT_VERSION))

    def __repr__(self) -> str:
        return f"Event({self.event_type}, {self.event_id[:8]}, {sorted(self.data)})"

    def __eq__(self, other) -> bool:
        return isinstance(other, Event) and self.to_dict() == other.to_dict()
