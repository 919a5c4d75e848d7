"""Document collections (archives, messages, threads, chunks, summaries, sources) + indexes.

Field names, required sets, status enum and indexes follow the reference's
docs/schemas/documents/v1/*.schema.json and collections.config.json; like the events, the JSON
Schemas are generated from the compact specs below.

Reference: docs/schemas/documents/v1/*.schema.json and collections.config.json (read by
infra/init/mongo-init.js:8-50).
"""
from __future__ import annotations

from .events import BOOL, DT, arr, i, obj

SCHEMA_BASE = "https://alan-jowett.github.io/CoPilot-For-Consensus/schemas/documents/v1/"

ID16 = {"type": "string", "pattern": "^[A-Fa-f0-9]{16}$"}
STR = {"type": "string"}
ANY_STR = {"type": ["string", "null"]}
STATUS = {"type": "string", "enum": ["pending", "processing", "completed", "failed", "failed_max_retries"]}
RETRY_FIELDS = {"status": STATUS, "attemptCount": i(0), "lastAttemptTime": {"type": ["string", "null"]},
                "lastUpdated": STR, "workerId": {"type": ["string", "null"]}}

COLLECTION_SPECS: dict[str, dict] = {
    "archives": {
        "required": ["_id", "file_hash", "file_size_bytes", "source", "ingestion_date", "status"],
        "properties": {"_id": ID16, "file_hash": {"type": "string", "pattern": "^[A-Fa-f0-9]{64}$"},
                       "file_size_bytes": i(0), "source": STR, "source_url": STR, "format": STR, "ingestion_date": STR,
                       "message_count": i(0), "file_path": STR, **RETRY_FIELDS},
        "indexes": ["source", "ingestion_date", "status"],
    },
    "messages": {
        "required": ["_id", "message_id", "archive_id", "thread_id", "body_normalized", "created_at"],
        "properties": {"_id": ID16, "message_id": STR, "archive_id": ID16, "thread_id": ID16,
                       "in_reply_to": ANY_STR, "references": arr(STR), "subject": ANY_STR,
                       "from": {"type": ["object", "null"]}, "to": arr({}), "cc": arr({}), "date": ANY_STR,
                       "body_raw": STR, "body_normalized": STR, "body_html": STR, "headers": obj(),
                       "attachments": arr({}), "draft_mentions": arr(STR), "created_at": STR, **RETRY_FIELDS},
        "indexes": ["message_id", "archive_id", "thread_id", "date", "in_reply_to", "draft_mentions", "created_at"],
    },
    "threads": {
        "required": ["_id", "archive_id", "has_consensus", "created_at"],
        "properties": {"_id": ID16, "thread_id": ID16, "archive_id": ID16, "subject": STR, "participants": arr({}),
                       "message_count": i(0), "first_message_date": ANY_STR, "last_message_date": ANY_STR,
                       "draft_mentions": arr(STR), "has_consensus": BOOL, "consensus_type": ANY_STR,
                       "summary_id": ANY_STR, "created_at": STR, **RETRY_FIELDS},
        "indexes": ["archive_id", "first_message_date", "last_message_date", "draft_mentions", "has_consensus",
                    "summary_id", "created_at"],
    },
    "chunks": {
        "required": ["_id", "message_doc_id", "message_id", "thread_id", "chunk_index", "text", "created_at",
                     "embedding_generated"],
        "properties": {"_id": ID16, "message_doc_id": ID16, "message_id": STR, "thread_id": ID16, "archive_id": STR,
                       "chunk_index": i(0), "text": STR, "token_count": i(0),
                       "start_offset": {"type": ["integer", "null"]}, "end_offset": {"type": ["integer", "null"]},
                       "overlap_with_previous": BOOL, "metadata": obj(), "created_at": STR,
                       "embedding_generated": BOOL, **RETRY_FIELDS},
        "indexes": ["message_id", "thread_id", "created_at", "embedding_generated"],
    },
    "summaries": {
        "required": ["_id", "summary_type", "generated_at", "content_markdown"],
        "properties": {"_id": ID16, "thread_id": ID16,
                       "summary_type": {"type": "string", "enum": ["thread", "weekly", "consensus", "draft-focused"]},
                       "title": STR, "content_markdown": STR, "content_html": STR, "citations": arr({}),
                       "generated_by": STR, "generated_at": STR, "first_message_date": ANY_STR,
                       "last_message_date": ANY_STR, "metadata": obj()},
        "indexes": ["thread_id", "summary_type", "generated_at", "first_message_date"],
    },
    "sources": {
        "required": ["name", "source_type", "url"],
        "properties": {"_id": STR, "name": STR, "source_type": {"type": "string",
                                                                 "enum": ["local", "http", "rsync", "imap"]},
                       "url": STR, "port": {"type": ["integer", "null"]}, "username": ANY_STR, "password": ANY_STR,
                       "folder": ANY_STR, "enabled": BOOL, "schedule": ANY_STR, "created_at": ANY_STR,
                       "updated_at": ANY_STR, "last_run_at": ANY_STR,
                       "last_run_status": {"type": ["string", "null"], "enum": ["success", "failure", None]},
                       "last_error": ANY_STR, "next_run_at": ANY_STR, "files_processed": i(0), "files_skipped": i(0)},
        "indexes": ["name", "enabled", "source_type"],
        "unique": ["name"],
    },
}

COLLECTIONS = tuple(COLLECTION_SPECS)
del DT


def document_schema(collection: str) -> dict:
    spec = COLLECTION_SPECS[collection]
    return {
        "$schema": "https://json-schema.org/draft/2020-12/schema",
        "$id": SCHEMA_BASE + f"{collection}.schema.json",
        "title": collection,
        "type": "object",
        "properties": spec["properties"],
        "required": spec["required"],
        "additionalProperties": True,
    }


def collections_config() -> dict:
    return {"collections": [
        {"name": c, "schema": f"/schemas/documents/v1/{c}.schema.json",
         "indexes": [{"keys": {f: 1}, "options": {"name": f"{f}_idx", **({"unique": True}
                                                                         if f in spec.get("unique", ()) else {})}}
                     for f in spec["indexes"]]}
        for c, spec in COLLECTION_SPECS.items()]}
