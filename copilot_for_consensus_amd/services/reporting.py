"""Reporting service: SummaryComplete -> summaries doc + thread link + webhook + ReportPublished, and
the read API (reference reporting/app/service.py:192-1187, reporting/main.py:73-474).

Read API (same paths / parameters): /api/reports (filters thread_id, limit<=100, skip,
message_start_date/end_date, source, min/max_participants, min/max_messages, sort_by, sort_order),
/api/reports/search (semantic topic search: embed topic -> index top (limit*3) -> group by
thread, max score -> threads >= min_score), /api/reports/{id}, /api/threads/{id}/summary,
/api/sources, /api/threads[/{id}], /api/messages[/{doc_id}], /api/chunks[/{id}].
"""
from __future__ import annotations

import json
import urllib.request
from datetime import datetime, timezone

from ..contracts import ids as cids
from ..retry import DocumentNotFoundError
from ..storage.document_store import DocumentAlreadyExistsError, DocumentNotFoundError as StoreNotFound
from .base import BaseService


class ReportingService(BaseService):
    name = "reporting"

    def __init__(self, publisher, subscriber, document_store, vector_store=None, embedding_provider=None,
                 notify_enabled: bool = False, notify_webhook_url: str = "", webhook_summary_max_length: int = 500,
                 **kw):
        super().__init__(publisher, subscriber, document_store, **kw)
        self.vectors, self.embedder = vector_store, embedding_provider
        self.notify_enabled, self.webhook_url = notify_enabled, notify_webhook_url
        self.webhook_max = webhook_summary_max_length
        self.stats.update(reports_stored=0, notifications_sent=0)

    def subscriptions(self):
        return {"SummaryComplete": lambda ev: self.process_summary(ev["data"], ev)}

    # ------------------------------------------------------------------ write path
    def process_summary(self, data: dict, event: dict | None = None) -> str:
        tid = data.get("thread_id")
        if not tid:
            raise ValueError("SummaryComplete event missing required 'thread_id'")
        sid = data.get("summary_id")
        rid = cids.report_id(sid) if sid else cids.sha256_16(f"{tid}|{data.get('summary_markdown', '')}")
        thread = self.store.get_document("threads", tid)
        if thread is None:
            raise DocumentNotFoundError(f"thread {tid} not found for denormalisation")
        now = datetime.now(timezone.utc).isoformat()
        cites = data.get("citations", [])
        doc = {"_id": rid, "summary_id": rid, "thread_id": tid, "summary_type": "thread",
               "title": f"Summary for {tid}", "content_markdown": data.get("summary_markdown", ""),
               "first_message_date": thread.get("first_message_date"),
               "last_message_date": thread.get("last_message_date"),
               "citations": [{"chunk_id": c.get("chunk_id", ""), "message_id": c.get("message_id", ""),
                              "quote": c.get("text", ""), "relevance_score": c.get("relevance_score", 1.0)}
                             for c in cites],
               "generated_by": data.get("llm_backend", ""), "generated_at": now,
               "metadata": {"llm_model": data.get("llm_model", ""), "tokens_prompt": data.get("tokens_prompt", 0),
                            "tokens_completion": data.get("tokens_completion", 0),
                            "latency_ms": data.get("latency_ms", 0),
                            "event_timestamp": (event or {}).get("timestamp", now), "original_summary_id": sid,
                            "original_citations": cites}}
        existing = self.store.get_document("summaries", rid)
        if existing is None:
            try:
                self.store.insert_document("summaries", doc)
                self.stats["reports_stored"] += 1
            except DocumentAlreadyExistsError:
                pass
        elif existing.get("first_message_date") is None and doc["first_message_date"] is not None:
            self.store.update_document("summaries", rid, {"first_message_date": doc["first_message_date"],
                                                          "last_message_date": doc["last_message_date"]})
        try:
            self.store.update_document("threads", tid, {"summary_id": rid})
        except StoreNotFound as e:
            raise DocumentNotFoundError(str(e)) from e
        notified, channels = False, []
        if self.notify_enabled and self.webhook_url:
            try:
                self._webhook(rid, tid, doc["content_markdown"])
                notified = True
                channels.append("webhook")
                self.stats["notifications_sent"] += 1
                self.metrics.increment("reporting_delivery_total", tags={"channel": "webhook", "status": "success"})
            except Exception as e:
                self.metrics.increment("reporting_delivery_total", tags={"channel": "webhook", "status": "failure"})
                self.publish("ReportDeliveryFailed", report_id=rid, thread_id=tid, delivery_channel="webhook",
                             error_message=str(e) or type(e).__name__, error_type=type(e).__name__, retry_count=0)
        self.publish("ReportPublished", thread_id=tid, report_id=rid, format="markdown", notified=notified,
                     delivery_channels=channels or ["api"], summary_url=f"/api/reports/{rid}")
        return rid

    def _webhook(self, rid, tid, markdown):
        body = json.dumps({"report_id": rid, "thread_id": tid, "summary": markdown[:self.webhook_max]}).encode()
        req = urllib.request.Request(self.webhook_url, data=body, headers={"Content-Type": "application/json"})
        urllib.request.urlopen(req, timeout=10).read()

    # ------------------------------------------------------------------ read path
    def _thread_filter_ok(self, t, start, end, min_p, max_p, min_m, max_m, source, archives):
        """Reference filter semantics (reporting/app/service.py:660-699, 1066-1107): date filters keep
        threads whose [first, last] message range overlaps [start, end] inclusively and skip threads
        without both dates; participant / message counts inclusive; source via the thread's archive."""
        if t is None:
            return False
        if start is not None or end is not None:
            first, last = t.get("first_message_date"), t.get("last_message_date")
            if not first or not last:
                return False
            if end is not None and first > end:
                return False
            if start is not None and last < start:
                return False
        n_p = len(t.get("participants") or [])
        if (min_p is not None and n_p < min_p) or (max_p is not None and n_p > max_p):
            return False
        n_m = t.get("message_count", 0)
        if (min_m is not None and n_m < min_m) or (max_m is not None and n_m > max_m):
            return False
        if source:
            a = self._archive(t.get("archive_id"), archives)
            if not a or a.get("source") != source:
                return False
        return True

    def _archive(self, archive_id, cache: dict):
        if not archive_id:
            return None
        if archive_id not in cache:
            cache[archive_id] = self.store.get_document("archives", archive_id)
        return cache[archive_id]

    @staticmethod
    def _sort_missing_last(docs: list[dict], path: tuple[str, ...], order: str) -> list[dict]:
        """Missing / empty values go last in either direction (reference service.py:722-741)."""
        def val(d):
            for k in path:
                d = d.get(k) if isinstance(d, dict) else None
            return d
        present = [d for d in docs if val(d)]
        missing = [d for d in docs if not val(d)]
        present.sort(key=lambda d: str(val(d)), reverse=order == "desc")
        return present + missing

    def get_reports(self, thread_id=None, limit=10, skip=0, message_start_date=None, message_end_date=None,
                    source=None, min_participants=None, max_participants=None, min_messages=None,
                    max_messages=None, sort_by="generated_at", sort_order="desc") -> list[dict]:
        """Summaries enriched with ``thread_metadata`` / ``archive_metadata`` (reports whose thread is
        gone are skipped), thread-level filters, sort by ``generated_at`` or ``thread_start_date``."""
        flt = {"thread_id": thread_id} if thread_id else {}
        docs = self.store.query_documents("summaries", flt, limit=1 << 30)
        tids = list({d.get("thread_id") for d in docs if d.get("thread_id")})
        threads = {t["_id"]: t for t in self.store.query_documents("threads", {"_id": {"$in": tids}},
                                                                    limit=len(tids) or 1)} if tids else {}
        archives: dict = {}
        out = []
        for d in docs:
            t = threads.get(d.get("thread_id"))
            if t is None or not self._thread_filter_ok(t, message_start_date, message_end_date, min_participants,
                                                       max_participants, min_messages, max_messages, source,
                                                       archives):
                continue
            parts = t.get("participants") or []
            d["thread_metadata"] = {"subject": t.get("subject", ""), "participants": parts,
                                    "participant_count": len(parts), "message_count": t.get("message_count", 0),
                                    "first_message_date": t.get("first_message_date"),
                                    "last_message_date": t.get("last_message_date")}
            a = self._archive(t.get("archive_id"), archives)
            if a:
                d["archive_metadata"] = {"source": a.get("source", ""), "source_url": a.get("source_url", ""),
                                         "ingestion_date": a.get("ingestion_date")}
            out.append(d)
        path = ("thread_metadata", "first_message_date") if sort_by == "thread_start_date" else ("generated_at",)
        out = self._sort_missing_last(out, path, sort_order)
        return out[skip:skip + limit]

    def search_reports_by_topic(self, topic: str, limit: int = 10, min_score: float = 0.5) -> list[dict]:
        if self.vectors is None or self.embedder is None:
            raise RuntimeError("semantic search needs a vector store and an embedding provider")
        vec = self.embedder.embed(topic)
        hits = self.vectors.query(vec, top_k=limit * 3)
        best: dict[str, dict] = {}
        for h in hits:
            tid = (h.metadata or {}).get("thread_id")
            if not tid:
                continue
            b = best.setdefault(tid, {"max": h.score, "sum": 0.0, "n": 0, "chunks": []})
            b["max"] = max(b["max"], h.score)
            b["sum"] += h.score
            b["n"] += 1
            b["chunks"].append(h.id)
        ranked = sorted(((tid, b) for tid, b in best.items() if b["max"] >= min_score),
                        key=lambda x: (-x[1]["max"], x[0]))[:limit]
        out = []
        for tid, b in ranked:
            summ = self.store.query_documents("summaries", {"thread_id": tid}, limit=1, sort_by="generated_at")
            thread = self.store.get_document("threads", tid)
            if not summ:
                continue
            r = dict(summ[0])
            r["relevance_score"] = b["max"]
            r["avg_score"] = b["sum"] / b["n"]
            r["matching_chunks"] = len(b["chunks"])
            if thread:
                r["thread_subject"] = thread.get("subject")
                r["thread_message_count"] = thread.get("message_count")
                r["thread_participants"] = thread.get("participants")
                arch = self.store.get_document("archives", thread.get("archive_id", ""))
                if arch:
                    r["archive_source"] = arch.get("source")
            out.append(r)
        return out

    def get_threads(self, limit=10, skip=0, archive_id=None, message_start_date=None, message_end_date=None,
                    source=None, min_participants=None, max_participants=None, min_messages=None, max_messages=None,
                    sort_by=None, sort_order="desc"):
        """Threads with the reference's filters, each enriched with ``archive_source``."""
        flt = {"archive_id": archive_id} if archive_id else {}
        docs = self.store.query_documents("threads", flt, limit=1 << 30)
        archives: dict = {}
        out = []
        for t in docs:
            if not self._thread_filter_ok(t, message_start_date, message_end_date, min_participants,
                                          max_participants, min_messages, max_messages, source, archives):
                continue
            a = self._archive(t.get("archive_id"), archives)
            t["archive_source"] = a.get("source") if a else None
            out.append(t)
        if sort_by:
            out = self._sort_missing_last(out, (sort_by,), sort_order)
        return out[skip:skip + limit]

    def get_sources(self) -> list[str]:
        return sorted({a.get("source") for a in self.store.query_documents("archives", {}, limit=1 << 30)
                       if a.get("source")})


def reporting_routes(app, service: ReportingService, auth=None):
    from fastapi import Depends, HTTPException, Query

    deps = [Depends(auth)] if auth else []

    @app.get("/api/reports", dependencies=deps)
    def reports(thread_id: str | None = None, limit: int = Query(10, ge=1, le=100), skip: int = Query(0, ge=0),
                message_start_date: str | None = None, message_end_date: str | None = None, source: str | None = None,
                min_participants: int | None = Query(None, ge=0), max_participants: int | None = Query(None, ge=0),
                min_messages: int | None = Query(None, ge=0), max_messages: int | None = Query(None, ge=0),
                sort_by: str = Query("generated_at", pattern="^(thread_start_date|generated_at)$"),
                sort_order: str = Query("desc", pattern="^(asc|desc)$")):
        r = service.get_reports(thread_id, limit, skip, message_start_date, message_end_date, source,
                                min_participants, max_participants, min_messages, max_messages, sort_by, sort_order)
        return {"reports": r, "count": len(r), "limit": limit, "skip": skip}

    @app.get("/api/reports/search", dependencies=deps)
    def search(topic: str, limit: int = Query(10, ge=1, le=50), min_score: float = Query(0.5, ge=0.0, le=1.0)):
        try:
            r = service.search_reports_by_topic(topic, limit, min_score)
        except ValueError as e:          # empty topic / search not configured (reporting/main.py:227-229)
            raise HTTPException(400, str(e))
        except RuntimeError as e:
            raise HTTPException(503, str(e))
        return {"topic": topic, "reports": r, "count": len(r), "min_score": min_score}

    @app.get("/api/reports/{report_id}", dependencies=deps)
    def report(report_id: str):
        d = service.store.get_document("summaries", report_id)
        if d is None:
            raise HTTPException(404, "Report not found")
        return d

    @app.get("/api/threads/{thread_id}/summary", dependencies=deps)
    def thread_summary(thread_id: str):
        r = service.store.query_documents("summaries", {"thread_id": thread_id}, limit=1, sort_by="generated_at")
        if not r:
            raise HTTPException(404, "Summary not found for thread")
        return r[0]

    @app.get("/api/sources", dependencies=deps)
    def sources():
        s = service.get_sources()
        return {"sources": s, "count": len(s)}

    @app.get("/api/threads", dependencies=deps)
    def threads(limit: int = Query(10, ge=1, le=100), skip: int = Query(0, ge=0), archive_id: str | None = None,
                message_start_date: str | None = None, message_end_date: str | None = None, source: str | None = None,
                min_participants: int | None = Query(None, ge=0), max_participants: int | None = Query(None, ge=0),
                min_messages: int | None = Query(None, ge=0), max_messages: int | None = Query(None, ge=0),
                sort_by: str | None = Query(None, pattern="^(first_message_date|last_message_date)$"),
                sort_order: str = Query("desc", pattern="^(asc|desc)$")):
        r = service.get_threads(limit, skip, archive_id, message_start_date, message_end_date, source,
                                min_participants, max_participants, min_messages, max_messages, sort_by, sort_order)
        return {"threads": r, "count": len(r), "limit": limit, "skip": skip}

    @app.get("/api/threads/{thread_id}", dependencies=deps)
    def thread(thread_id: str):
        d = service.store.get_document("threads", thread_id)
        if d is None:
            raise HTTPException(404, "Thread not found")
        return d

    @app.get("/api/messages", dependencies=deps)
    def messages(limit: int = Query(10, ge=1, le=100), skip: int = Query(0, ge=0), thread_id: str | None = None,
                 message_id: str | None = None):
        flt = {k: v for k, v in (("thread_id", thread_id), ("message_id", message_id)) if v}
        r = service.store.query_documents("messages", flt, limit=limit, skip=skip, sort_by="date", sort_order="asc")
        return {"messages": r, "count": len(r), "limit": limit, "skip": skip}

    @app.get("/api/messages/{message_doc_id}", dependencies=deps)
    def message(message_doc_id: str):
        d = service.store.get_document("messages", message_doc_id)
        if d is None:
            raise HTTPException(404, "Message not found")
        return d

    @app.get("/api/chunks", dependencies=deps)
    def chunks(limit: int = Query(10, ge=1, le=100), skip: int = Query(0, ge=0), message_id: str | None = None,
               thread_id: str | None = None, message_doc_id: str | None = None):
        flt = {k: v for k, v in (("message_id", message_id), ("thread_id", thread_id),
                                 ("message_doc_id", message_doc_id)) if v}
        r = service.store.query_documents("chunks", flt, limit=limit, skip=skip, sort_by="chunk_index", sort_order="asc")
        return {"chunks": r, "count": len(r), "limit": limit, "skip": skip}

    @app.get("/api/chunks/{chunk_id}", dependencies=deps)
    def chunk(chunk_id: str):
        d = service.store.get_document("chunks", chunk_id)
        if d is None:
            raise HTTPException(404, "Chunk not found")
        return d
