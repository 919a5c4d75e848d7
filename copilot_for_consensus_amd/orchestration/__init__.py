"""Orchestration: context candidates, context selection, prompt construction.

Mirrors the reference orchestrator (orchestrator/app/context_sources.py:40, context_selectors.py:20-181,
service.py:411-676) and the summarizer's template substitution (summarization/app/service.py:450):

* candidates come from the thread's chunks; when a query vector is available (the thread centroid
  of its chunk embeddings -- the reference leaves query vectors unimplemented,
  context_sources.py:57-64) they are scored by the HIP index, otherwise they get the neutral 0.5;
* TopKRelevanceSelector: score desc, chunk id asc, stop at top_k or when the 1.3 x words token
  estimate would exceed the budget (context_selectors.py:17,72,95-107);
* TopKCohesiveSelector: relevance top-k re-ordered by (message order, chunk index) so excerpts
  read in thread order;
* the prompt = system + user template; placeholders {thread_id} {message_count} {date_range}
  {participants} {draft_mentions} {email_chunks} only.
"""
from __future__ import annotations

import dataclasses
from pathlib import Path
from string import Formatter
from typing import Any, Callable

TOKEN_ESTIMATION_MULTIPLIER = 1.3
PROMPT_DIR = Path(__file__).resolve().parent / "prompts"
ALLOWED_PLACEHOLDERS = {"thread_id", "message_count", "date_range", "participants", "draft_mentions", "email_chunks"}


def estimate_tokens(text: str) -> int:
    return int(len(text.split()) * TOKEN_ESTIMATION_MULTIPLIER)


def load_prompts(system_path: str | None = None, user_path: str | None = None) -> tuple[str, str]:
    sp = Path(system_path) if system_path and Path(system_path).exists() else PROMPT_DIR / "system.txt"
    up = Path(user_path) if user_path and Path(user_path).exists() else PROMPT_DIR / "user.txt"
    return sp.read_text(encoding="utf-8"), up.read_text(encoding="utf-8")


def prompt_template(system_path: str | None = None, user_path: str | None = None) -> str:
    s, u = load_prompts(system_path, user_path)
    return f"{s.rstrip()}\n\n{u}"


@dataclasses.dataclass
class SelectedChunk:
    chunk_id: str
    source: str
    score: float
    rank: int
    metadata: dict[str, Any]

    def to_dict(self) -> dict:
        return {"chunk_id": self.chunk_id, "source": self.source, "score": float(self.score), "rank": self.rank,
                "metadata": self.metadata}


@dataclasses.dataclass
class ContextSelection:
    selected_chunks: list[SelectedChunk]
    selector_type: str
    selector_version: str
    selection_params: dict[str, Any]
    total_candidates: int
    total_tokens: int

    def metadata(self) -> dict:
        return {"selector_type": self.selector_type, "selector_version": self.selector_version,
                "selection_params": self.selection_params, "total_candidates": self.total_candidates,
                "total_tokens": self.total_tokens}


class TopKRelevanceSelector:
    VERSION = "1.0.0"
    selector_type = "top_k_relevance"

    def __init__(self, token_estimator: Callable[[str], int] | None = None):
        self.token_estimator = token_estimator or estimate_tokens

    def _rank(self, candidates):
        return sorted(candidates, key=lambda c: (-float(c.get("similarity_score", 0.0)), str(c.get("_id") or "")))

    def select(self, thread_id: str, candidates: list[dict], top_k: int,
               context_window_tokens: int | None = None) -> ContextSelection:
        params = {"top_k": top_k, "context_window_tokens": context_window_tokens}
        out, total = [], 0
        for c in self._rank(candidates)[:top_k]:
            cid = c.get("_id")
            if not cid:
                continue
            if context_window_tokens is not None:
                n = self.token_estimator(c.get("text", ""))
                if total + n > context_window_tokens:
                    break
                total += n
            out.append(SelectedChunk(str(cid), c.get("source_type", "thread_chunks"), float(c.get("similarity_score", 0.0)),
                                     len(out), {"message_id": c.get("message_id", ""),
                                                "message_doc_id": c.get("message_doc_id", ""),
                                                "offset": c.get("offset", 0),
                                                "thread_id": c.get("thread_id", thread_id)}))
        return ContextSelection(out, self.selector_type, self.VERSION, params, len(candidates), total)


class TopKCohesiveSelector(TopKRelevanceSelector):
    selector_type = "top_k_cohesive"

    def select(self, thread_id, candidates, top_k, context_window_tokens=None):
        sel = super().select(thread_id, candidates, top_k, context_window_tokens)
        by_id = {str(c.get("_id")): c for c in candidates}
        sel.selected_chunks.sort(key=lambda s: (str(by_id[s.chunk_id].get("date") or ""),
                                                by_id[s.chunk_id].get("chunk_index", 0)))
        for r, s in enumerate(sel.selected_chunks):
            s.rank = r
        sel.selector_type = self.selector_type
        return sel


def create_context_selector(strategy: str = "top_k_relevance"):
    strategy = str(strategy).strip().lower()
    if strategy in ("top_k_relevance", "topk", "relevance"):
        return TopKRelevanceSelector()
    if strategy in ("top_k_cohesive", "cohesive"):
        return TopKCohesiveSelector()
    raise ValueError(f"unknown chunk selection strategy {strategy!r}")


def build_context(chunks: list[dict], messages_by_id: dict[str, dict] | None = None) -> dict:
    """Context dict for prompt substitution: excerpts + per-chunk sender/date/draft metadata."""
    messages_by_id = messages_by_id or {}
    enriched = []
    for c in chunks:
        m = messages_by_id.get(c.get("message_doc_id"), {})
        e = dict(c)
        e.setdefault("from", m.get("from"))
        e.setdefault("date", m.get("date"))
        e.setdefault("draft_mentions", m.get("draft_mentions", []))
        enriched.append(e)
    return {"messages": [c.get("text", "") for c in enriched if c.get("text")], "chunks": enriched}


def substitute_prompt(template: str, thread_id: str, context: dict) -> str:
    chunks = context.get("chunks", [])
    messages = context.get("messages", [])
    parts = set()
    for c in chunks:
        s = c.get("from")
        if isinstance(s, dict) and s.get("email"):
            parts.add(f"{s.get('name') or s.get('email')} <{s.get('email')}>")
        elif isinstance(s, str) and s:
            parts.add(s)
    drafts = set()
    for c in chunks:
        if isinstance(c.get("draft_mentions"), list):
            drafts.update(c["draft_mentions"])
    dates = sorted(c["date"] for c in chunks if c.get("date"))
    found = {f for _, f, _, _ in Formatter().parse(template) if f}
    bad = found - ALLOWED_PLACEHOLDERS
    if bad:
        raise ValueError(f"Prompt template contains unexpected placeholders: {sorted(bad)}")
    return template.format(
        thread_id=thread_id,
        message_count=len(messages),
        date_range=f"{dates[0]} to {dates[-1]}" if dates else "Unknown",
        participants=", ".join(sorted(parts)) if parts else "Multiple participants",
        draft_mentions="\n".join(sorted(drafts)) if drafts else "No specific drafts mentioned",
        email_chunks="\n\n".join(f"Message {i + 1}:\n{m}" for i, m in enumerate(messages)) or "(No messages available)",
    )


def format_citations(chunks: list[dict], limit: int = 12) -> list[dict]:
    return [{"message_id": c.get("message_id", "") or "unknown", "chunk_id": c["_id"], "offset": int(c.get("offset", 0)),
             "text": c.get("text", "")} for c in chunks[:limit] if c.get("_id")]
