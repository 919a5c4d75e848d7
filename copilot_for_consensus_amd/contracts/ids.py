"""Deterministic document ids -- bit-identical to the reference.

* archive   ``sha256(bytes)[:16]``  (identifier_generator.py:26-32; local_volume_archive_store.py:125)
* message   ``sha256_16("archive_id|message_id[|date][|sender_email][|subject]")``; absent optional
            parts are skipped, not emptied (identifier_generator.py:35-56)
* chunk     ``sha256_16("message_doc_id|chunk_index")`` (:59-65)
* thread    ``_id`` of the thread's root message (parsing/app/thread_builder.py:45-65)
* summary   ``sha256("thread_id:" + ",".join(sorted(chunk_ids)))`` full hex, used as the event
            ``summary_id`` (summarization/app/service.py:741-769, orchestrator mirror :481-503)
* report    ``sha256(summary_id)[:16]`` = ``summaries._id`` (reporting/app/service.py:212)
* content summary id ``sha256_16("thread_id|content|generated_at")`` (identifier_generator.py:68)
"""
from __future__ import annotations

import hashlib


def sha256_16(s: str) -> str:
    return hashlib.sha256(s.encode("utf-8")).hexdigest()[:16]


def archive_id_from_bytes(data: bytes) -> str:
    return hashlib.sha256(data).hexdigest()[:16]


def message_doc_id(archive_id: str, message_id: str, date: str | None = None, sender_email: str | None = None,
                   subject: str | None = None) -> str:
    parts = [archive_id or "", message_id or ""]
    parts += [p for p in (date, sender_email, subject) if p]
    return sha256_16("|".join(parts))


def chunk_id(message_doc_id_: str, chunk_index: int) -> str:
    return sha256_16(f"{message_doc_id_}|{chunk_index}")


def summary_id(thread_id: str, chunk_ids) -> str:
    return hashlib.sha256(f"{thread_id}:{','.join(sorted(chunk_ids))}".encode("utf-8")).hexdigest()


def report_id(summary_id_: str) -> str:
    return hashlib.sha256(summary_id_.encode("utf-8")).hexdigest()[:16]


def content_summary_id(thread_id: str, content_markdown: str, generated_at_iso: str) -> str:
    return sha256_16(f"{thread_id}|{content_markdown}|{generated_at_iso}")
