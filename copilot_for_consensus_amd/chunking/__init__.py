"""Chunking strategies (adapters/copilot_chunking/copilot_chunking/chunkers.py of the reference).

* TokenWindowChunker -- sliding window over WHITESPACE WORDS (the reference's "tokens",
  chunkers.py:169): chunk_size 384, overlap 50; windows shorter than min_chunk_size are dropped
  unless they are the tail; ids sha256_16(message_doc_id|chunk_index).
* FixedSizeChunker -- N messages (or N "\\n\\n" blocks) per chunk.
* SemanticChunker -- sentence-boundary packing up to target_chunk_size words.
Semantics (incl. the word-count quirk) are preserved for id/chunk parity with the reference.
"""
from __future__ import annotations

import dataclasses
import re
from abc import ABC, abstractmethod
from typing import Any

from ..contracts.ids import chunk_id


@dataclasses.dataclass
class Chunk:
    chunk_id: str
    text: str
    chunk_index: int
    token_count: int
    metadata: dict[str, Any]
    message_doc_id: str
    thread_id: str
    start_offset: int | None = None
    end_offset: int | None = None


@dataclasses.dataclass
class Thread:
    thread_id: str
    text: str
    metadata: dict[str, Any]
    message_doc_id: str | None = None
    message_id: str | None = None
    messages: list[dict[str, Any]] | None = None


class ThreadChunker(ABC):
    strategy = "base"

    @abstractmethod
    def chunk(self, thread: Thread) -> list[Chunk]: ...


def _require(thread: Thread, need_text: bool = True):
    if need_text and (not thread.text or not thread.text.strip()):
        raise ValueError("Thread text cannot be empty")
    if thread.message_doc_id is None:
        raise ValueError("Thread message_doc_id must be provided before chunking")


class TokenWindowChunker(ThreadChunker):
    strategy = "token_window"

    def __init__(self, chunk_size: int = 384, overlap: int = 50, min_chunk_size: int = 100, max_chunk_size: int = 512):
        if chunk_size <= 0:
            raise ValueError("chunk_size must be positive")
        # a negative overlap would skip the words between two windows
        if overlap < 0:
            raise ValueError(f"overlap must be >= 0, got {overlap}")
        self.chunk_size, self.overlap = int(chunk_size), int(overlap)
        # A full window always meets the minimum: with CHUNK_SIZE_TOKENS set below the default
        # minimum (100) the reference discards every full window and keeps only the tail
        # (chunkers.py:184), silently losing the text -- the minimum is clamped to the window.
        self.min_chunk_size = min(int(min_chunk_size), self.chunk_size)
        self.max_chunk_size = int(max_chunk_size)

    def chunk(self, thread: Thread) -> list[Chunk]:
        _require(thread)
        words = thread.text.split()
        n = len(words)
        out, start, idx = [], 0, 0
        while start < n:
            end = min(start + self.chunk_size, n)
            if end - start >= self.min_chunk_size or end == n:
                out.append(Chunk(chunk_id(thread.message_doc_id, idx), " ".join(words[start:end]), idx, end - start,
                                 dict(thread.metadata), thread.message_doc_id, thread.thread_id))
                idx += 1
            if end == n:
                break
            nxt = end - self.overlap
            start = nxt if nxt > start else end
        return out


class FixedSizeChunker(ThreadChunker):
    strategy = "fixed_size"

    def __init__(self, messages_per_chunk: int = 5):
        if messages_per_chunk < 1:
            raise ValueError("messages_per_chunk must be at least 1")
        self.messages_per_chunk = int(messages_per_chunk)

    def chunk(self, thread: Thread) -> list[Chunk]:
        _require(thread, need_text=False)
        k = self.messages_per_chunk
        out = []
        if thread.messages:
            msgs = thread.messages
            missing = [i for i, m in enumerate(msgs) if not m.get("message_doc_id")]
            if missing:
                raise ValueError(f"message_doc_id is required for each message ({len(missing)} missing)")
            for i in range(0, len(msgs), k):
                group = msgs[i:i + k]
                text = "\n\n".join(m.get("text", m.get("body", "")) for m in group)
                md = dict(thread.metadata)
                md["message_doc_ids"] = [m["message_doc_id"] for m in group]
                md["message_count"] = len(group)
                ci = i // k
                out.append(Chunk(chunk_id(thread.message_doc_id, ci), text, ci, len(text.split()), md,
                                 thread.message_doc_id, thread.thread_id))
            return out
        if not thread.text or not thread.text.strip():
            raise ValueError("Thread must have either messages or text")
        blocks = [b.strip() for b in thread.text.split("\n\n") if b.strip()]
        for i in range(0, len(blocks), k):
            text = "\n\n".join(blocks[i:i + k])
            ci = i // k
            out.append(Chunk(chunk_id(thread.message_doc_id, ci), text, ci, len(text.split()), dict(thread.metadata),
                             thread.message_doc_id, thread.thread_id))
        return out


class SemanticChunker(ThreadChunker):
    """Sentence-boundary chunking up to ``target_chunk_size`` words (reference chunkers.py:352).

    ``split_on_speaker`` (declared but "not yet implemented" in the reference, chunkers.py:361):
    when the thread carries its ``messages`` (each with ``from``), a chunk never spans two
    consecutive messages by different senders, and each chunk records its ``speaker``."""
    strategy = "semantic"
    _SENT = re.compile(r"(?<=[.!?])\s+")

    def __init__(self, target_chunk_size: int = 400, split_on_speaker: bool = False):
        if target_chunk_size <= 0:
            raise ValueError("target_chunk_size must be positive")
        self.target_chunk_size = int(target_chunk_size)
        self.split_on_speaker = bool(split_on_speaker)

    def _sentences(self, text: str) -> list[str]:
        return [s.strip() for s in self._SENT.split(text) if s.strip()]

    @staticmethod
    def _speaker(m: dict) -> str:
        f = m.get("from")
        if isinstance(f, dict):
            return str(f.get("email") or f.get("name") or "")
        return str(f or m.get("sender") or "")

    def chunk(self, thread: Thread) -> list[Chunk]:
        by_speaker = self.split_on_speaker and bool(thread.messages)
        if by_speaker:
            _require(thread, need_text=False)
            turns = [(self._speaker(m), m.get("text", m.get("body", ""))) for m in thread.messages]
        else:
            _require(thread)
            turns = [(None, thread.text)]
        out, cur, count, idx = [], [], 0, 0
        cur_speaker = None

        def flush():
            nonlocal cur, count, idx
            md = dict(thread.metadata)
            if by_speaker:
                md["speaker"] = cur_speaker
            out.append(Chunk(chunk_id(thread.message_doc_id, idx), " ".join(cur), idx, count, md,
                             thread.message_doc_id, thread.thread_id))
            idx += 1
            cur, count = [], 0

        for speaker, text in turns:
            if cur and by_speaker and speaker != cur_speaker:
                flush()
            cur_speaker = speaker
            for s in self._sentences(text or ""):
                n = len(s.split())
                if cur and count + n > self.target_chunk_size:
                    flush()
                cur.append(s)
                count += n
        if cur:
            flush()
        if not out and by_speaker:
            raise ValueError("Thread messages contain no text")
        return out


def create_chunker(cfg=None, **overrides) -> ThreadChunker:
    name = str(getattr(cfg, "driver_name", cfg) or "token_window").strip().lower()
    kw = {k: v for k, v in dict(getattr(cfg, "driver_config", {}) or {}).items() if v is not None}
    kw.update(overrides)
    if name == "token_window":
        return TokenWindowChunker(**{k: kw[k] for k in ("chunk_size", "overlap", "min_chunk_size", "max_chunk_size")
                                     if k in kw})
    if name == "fixed_size":
        return FixedSizeChunker(**{k: kw[k] for k in ("messages_per_chunk",) if k in kw})
    if name == "semantic":
        return SemanticChunker(**{k: kw[k] for k in ("target_chunk_size", "split_on_speaker") if k in kw})
    raise ValueError(f"unknown chunker {name!r}")
