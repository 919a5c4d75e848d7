"""Mailing-list archive parsing: mbox -> messages -> threads.

Behaviour follows the reference parsing service (parsing/app/parser.py:42-383, normalizer.py,
draft_detector.py, thread_builder.py): Message-ID required (angle brackets stripped), In-Reply-To /
References, RFC-2047 decoded Subject, Date -> ISO-8601 UTC 'Z', From/To/CC parsed to
{name, email}, text/plain preferred over text/html, normalisation (HTML strip, signature cut,
quoted-line removal, whitespace collapse), RFC/draft mention detection, threads rooted at the
message with no In-Reply-To (walk <= 100 hops, cycle-safe), thread ``_id`` = root message ``_id``.

MI355X-native difference: the mbox is split by the C++ runtime (``cfc_mbox_split``: one memchr
pass) instead of Python's ``mailbox`` module, and messages can be parsed by a process pool.
"""
from __future__ import annotations

import ctypes
import re
from concurrent.futures import ProcessPoolExecutor
from datetime import datetime, timezone
from email.header import decode_header
from email.message import Message
from email.parser import BytesParser
from email.policy import compat32
from email.utils import getaddresses, parseaddr, parsedate_to_datetime
from typing import Any

from ..contracts.ids import message_doc_id


class MessageParsingError(Exception):
    pass


class RequiredFieldMissingError(MessageParsingError):
    pass


# ------------------------------------------------------------------------------ mbox splitting

def split_mbox(data: bytes) -> list[bytes]:
    """Split an mbox buffer into raw messages (without their ``From `` separator line)."""
    offsets = None
    try:
        from ..ops._native import runtime
        lib = runtime()
        import numpy as np
        cap = max(16, data.count(b"\nFrom ") + 2)
        out = np.empty(cap, dtype=np.int64)
        n = lib.cfc_mbox_split(data, len(data), out.ctypes.data_as(ctypes.c_void_p), cap)
        offsets = out[:min(n, cap)].tolist()
    except Exception:
        offsets = None
    if offsets is None:
        offsets = ([0] if data.startswith(b"From ") else []) + [m.start() + 1 for m in re.finditer(rb"\nFrom ", data)]
    msgs = []
    for i, off in enumerate(offsets):
        end = offsets[i + 1] if i + 1 < len(offsets) else len(data)
        chunk = data[off:end]
        nl = chunk.find(b"\n")
        body = chunk[nl + 1:] if nl >= 0 else b""
        # the empty line in front of the next "From " line (or at end of file) belongs to the
        # separator, as Python's mailbox.mbox (the reference parser) reads it
        if body.endswith(b"\n\n") and not body.endswith(b"\r\n\r\n"):
            body = body[:-1]
        if body.strip():
            msgs.append(body)
    return msgs


# ------------------------------------------------------------------------------ normaliser

_WS_RUN = re.compile(r" [ \t]+|\t[ \t]*")   # = [ \t]+ -> " ", without rewriting every single space
_BLANK_RUN = re.compile(r"\n{3,}")


class TextNormalizer:
    SIGNATURE_DELIMITERS = ("\n-- \n", "\n--\n", "\n___\n", "\n___________\n",
                            "\n________________________________________\n")
    _HTML_MARKERS = ("<html", "<body", "<div", "<p>", "<br>", "<span", "<table")

    def __init__(self, strip_html=True, strip_signatures=True, strip_quoted=True):
        self.strip_html, self.strip_signatures, self.strip_quoted = strip_html, strip_signatures, strip_quoted

    def normalize(self, text: str) -> str:
        if not text:
            return ""
        if self.strip_html and any(m in text.lower() for m in self._HTML_MARKERS):
            text = self._remove_html(text)
        if self.strip_signatures:
            for d in self.SIGNATURE_DELIMITERS:
                if d in text:
                    text = text.split(d)[0]
                    break
        if self.strip_quoted:
            text = "\n".join(ln for ln in text.split("\n")
                             if not ln.strip() or not ln.strip().startswith((">", "|")))
        text = _WS_RUN.sub(" ", text)
        text = _BLANK_RUN.sub("\n\n", text)
        return text.strip()

    @staticmethod
    def _remove_html(text: str) -> str:
        text = re.sub(r"<style(?:\s[^>]*)?>.*?</style(?:\s[^>]*)?>", "", text, flags=re.DOTALL | re.IGNORECASE)
        text = re.sub(r"<script(?:\s[^>]*)?>.*?</script(?:\s[^>]*)?>", "", text, flags=re.DOTALL | re.IGNORECASE)
        text = re.sub(r"<[^>]+>", "", text)
        for a, b in (("&nbsp;", " "), ("&lt;", "<"), ("&gt;", ">"), ("&quot;", '"'), ("&#39;", "'"), ("&amp;", "&")):
            text = text.replace(a, b)
        return text


class DraftDetector:
    DEFAULT_PATTERN = r"(draft-[a-z0-9-]+-\d+)|(RFC\s*\d+)|(rfc\d+)"

    def __init__(self, pattern: str | None = None):
        self.regex = re.compile(pattern or self.DEFAULT_PATTERN, re.IGNORECASE)
        # the default pattern only matches where "draft-" or "rfc" occurs (any case): most bodies
        # mention neither, and one lower() + two substring scans are far cheaper than the
        # case-insensitive three-way alternation tried at every position
        self._prefilter = pattern is None

    def detect(self, text: str) -> list[str]:
        if not text:
            return []
        matches = self.regex.finditer(text)
        if self._prefilter:
            low = text.lower()
            if "rfc" not in low and "draft-" not in low:
                return []
            if len(low) == len(text):
                # the default pattern can only start where "draft-" or "rfc" does (any case): run it
                # at those positions only, left to right and non-overlapping as finditer would
                matches = self._anchored(text, low)
        out, seen = [], set()
        for m in matches:
            g = next(x for x in m.groups() if x)
            if g.lower().startswith("rfc"):
                g = "RFC " + re.search(r"\d+", g).group()
            if g not in seen:
                seen.add(g)
                out.append(g)
        return out

    def _anchored(self, text: str, low: str):
        starts = []
        for needle in ("draft-", "rfc"):
            i = low.find(needle)
            while i >= 0:
                starts.append(i)
                i = low.find(needle, i + 1)
        end = 0
        for i in sorted(starts):
            if i < end:
                continue
            m = self.regex.match(text, i)
            if m is not None and m.end() > m.start():
                yield m
                end = m.end()


# ------------------------------------------------------------------------------ message parser

PRESERVED_HEADERS = ("X-Mailer", "User-Agent", "Content-Type", "Content-Transfer-Encoding", "MIME-Version",
                     "X-Priority", "Importance")


def _decode(value) -> str:
    if not value:
        return ""
    try:
        parts = []
        for content, enc in decode_header(str(value)):
            parts.append(content.decode(enc or "utf-8", errors="replace") if isinstance(content, bytes) else content)
        return " ".join(parts)
    except Exception:
        return str(value)


def _iso_date(value) -> str | None:
    if not value:
        return None
    try:
        return parsedate_to_datetime(value).astimezone(timezone.utc).isoformat().replace("+00:00", "Z")
    except Exception:
        return None


def _addr(value) -> dict | None:
    if not value:
        return None
    name, email = parseaddr(_decode(value))
    return {"name": name or "", "email": email} if email else None


def _addrs(value) -> list[dict]:
    if not value:
        return []
    return [{"name": n or "", "email": e} for n, e in getaddresses([_decode(value)]) if e]


def _payload_text(part: Message) -> str:
    payload = part.get_payload(decode=True)
    if isinstance(payload, bytes):
        return payload.decode(part.get_content_charset() or "utf-8", errors="replace")
    return ""


def extract_body(msg: Message) -> str:
    if msg.is_multipart():
        for ctype in ("text/plain", "text/html"):
            for part in msg.walk():
                if part.get_content_type() == ctype:
                    try:
                        body = _payload_text(part)
                    except Exception:
                        body = ""
                    if body:
                        return body
        return ""
    try:
        payload = msg.get_payload(decode=True)
        if isinstance(payload, bytes):
            return payload.decode(msg.get_content_charset() or "utf-8", errors="replace")
        return str(msg.get_payload())
    except Exception:
        return str(msg.get_payload())


class MessageParser:
    def __init__(self, normalizer: TextNormalizer | None = None, draft_detector: DraftDetector | None = None):
        self.normalizer = normalizer or TextNormalizer()
        self.draft_detector = draft_detector or DraftDetector()
        self._bp = BytesParser(policy=compat32)

    def parse_message(self, msg: Message, archive_id: str) -> dict[str, Any]:
        mid = (msg.get("Message-ID") or "").strip().strip("<>")
        if not mid:
            raise RequiredFieldMissingError("Message-ID")
        irt = (msg.get("In-Reply-To") or "").strip().strip("<>") or None
        refs = [r.strip("<>") for r in (msg.get("References") or "").split() if r]
        body_raw = extract_body(msg)
        body_norm = self.normalizer.normalize(body_raw)
        parsed = {
            "message_id": mid,
            "archive_id": archive_id,
            "thread_id": irt or mid,
            "in_reply_to": irt,
            "references": refs,
            "subject": _decode(msg.get("Subject", "")),
            "from": _addr(msg.get("From", "")),
            "to": _addrs(msg.get("To", "")),
            "cc": _addrs(msg.get("CC", "")),
            "date": _iso_date(msg.get("Date")),
            "body_raw": body_raw,
            "body_normalized": body_norm,
            "headers": {h.lower(): _decode(msg.get(h)) for h in PRESERVED_HEADERS if msg.get(h)},
            "draft_mentions": self.draft_detector.detect(body_norm),
            "created_at": datetime.now(timezone.utc).isoformat().replace("+00:00", "Z"),
        }
        parsed["_id"] = message_doc_id(archive_id, mid, parsed["date"], (parsed["from"] or {}).get("email"),
                                       parsed["subject"])
        return parsed

    def parse_bytes(self, raw: bytes, archive_id: str) -> dict[str, Any]:
        return self.parse_message(self._bp.parsebytes(raw), archive_id)

    def parse_mbox_bytes(self, data: bytes, archive_id: str, workers: int = 0) -> tuple[list[dict], list[str]]:
        """Parse every message; returns (messages, errors).  ``workers`` > 1 uses a process pool."""
        raws = split_mbox(data)
        if workers > 1 and len(raws) > 256:
            with ProcessPoolExecutor(workers) as ex:
                results = list(ex.map(_parse_one, [(r, archive_id) for r in raws], chunksize=64))
        else:
            results = [_parse_one((r, archive_id), self) for r in raws]
        msgs, errs = [], []
        for i, (m, e) in enumerate(results):
            if m is not None:
                msgs.append(m)
            else:
                errs.append(f"Message {i}: {e}")
        if not msgs and errs:
            raise MessageParsingError(f"Failed to parse any messages. Errors: {'; '.join(errs[:5])}")
        return msgs, errs

    def parse_mbox(self, path: str, archive_id: str, workers: int = 0) -> list[dict]:
        with open(path, "rb") as f:
            return self.parse_mbox_bytes(f.read(), archive_id, workers)[0]


_WORKER_PARSER: MessageParser | None = None


def _parse_one(args, parser: MessageParser | None = None):
    global _WORKER_PARSER
    raw, archive_id = args
    if parser is None:
        if _WORKER_PARSER is None:
            _WORKER_PARSER = MessageParser()
        parser = _WORKER_PARSER
    try:
        return parser.parse_bytes(raw, archive_id), None
    except Exception as e:  # collect, do not abort the archive
        return None, str(e)


# ------------------------------------------------------------------------------ threads

def clean_subject(subject: str) -> str:
    if not subject:
        return ""
    prev = None
    while prev != subject:
        prev = subject
        subject = re.sub(r"^(Re:|RE:|Fwd:|FWD:|FW:)\s*", "", subject, flags=re.IGNORECASE)
        subject = re.sub(r"^\[.*?\]\s*", "", subject).strip()
    return subject


class ThreadBuilder:
    def __init__(self, max_depth: int = 100):
        self.max_depth = max_depth

    def _root(self, mid: str, by_id: dict, roots: set) -> str:
        if mid in roots:
            return mid
        seen, cur = set(), mid
        for _ in range(self.max_depth):
            if cur in seen:
                return mid  # cycle
            seen.add(cur)
            m = by_id.get(cur)
            if m is None:
                return cur
            parent = m.get("in_reply_to")
            if not parent:
                roots.add(cur)
                return cur
            cur = parent
        return cur

    def build_threads(self, messages: list[dict]) -> list[dict]:
        if not messages:
            return []
        by_id = {m["message_id"]: m for m in messages}
        roots = {m["message_id"] for m in messages if not m.get("in_reply_to")}
        for m in messages:
            r = self._root(m["message_id"], by_id, roots)
            root_msg = by_id.get(r)
            if root_msg is None:
                root_msg = m  # parent outside the parsed set
            if "_id" not in root_msg:
                raise KeyError("messages need '_id' before threading")
            m["thread_id"] = root_msg["_id"]
        now = datetime.now(timezone.utc).isoformat().replace("+00:00", "Z")
        threads: dict[str, dict] = {}
        for m in messages:
            tid = m["thread_id"]
            t = threads.get(tid)
            if t is None:
                t = threads[tid] = {"_id": tid, "thread_id": tid, "archive_id": m["archive_id"],
                                    "subject": clean_subject(m.get("subject", "")), "participants": [],
                                    "_emails": set(), "message_count": 0, "first_message_date": m.get("date"),
                                    "last_message_date": m.get("date"), "draft_mentions": {}, "created_at": now}
            t["message_count"] += 1
            fr = m.get("from")
            if fr and fr.get("email") and fr["email"] not in t["_emails"]:
                t["_emails"].add(fr["email"])
                t["participants"].append(fr)
            d = m.get("date")
            if d:
                if not t["first_message_date"] or d < t["first_message_date"]:
                    t["first_message_date"] = d
                if not t["last_message_date"] or d > t["last_message_date"]:
                    t["last_message_date"] = d
            for dm in m.get("draft_mentions", []):
                t["draft_mentions"][dm] = None
        out = []
        for t in threads.values():
            del t["_emails"]
            t["draft_mentions"] = list(t["draft_mentions"])
            t.update(has_consensus=False, consensus_type=None, summary_id=None)
            out.append(t)
        return out
