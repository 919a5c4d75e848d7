"""Log template mining (Drain) for incident triage.

Parity target: scripts/log_mining/ of the reference (normalize_message mining.py:107 -- <TS>,
<GUID>, <IP>, <URL>, <HEX>, <NUM> masking; per-template counts, reservoir samples, shortest /
longest sample, rare-template and first-seen anomaly lists; JSON report; plain / docker-compose /
JSON-lines inputs; group-by service).  The reference depends on the ``drain3`` package; the Drain
fixed-depth parse tree is implemented here directly (He et al., ICWS'17): leaf groups keyed by
token count and the first ``depth-3`` tokens (digits-bearing tokens route to a wildcard branch),
similarity = fraction of positions with equal tokens, clusters merge by turning differing positions
into ``<*>``.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import random
import re
import sys
from datetime import datetime, timezone
from pathlib import Path
from typing import Iterable, Iterator

_TS = re.compile(r"\b\d{4}-\d{2}-\d{2}[T ]\d{2}:\d{2}:\d{2}(?:[.,]\d+)?(?:Z|[+-]\d{2}:?\d{2})?\b")
_GUID = re.compile(r"\b[0-9a-fA-F]{8}-[0-9a-fA-F]{4}-[0-9a-fA-F]{4}-[0-9a-fA-F]{4}-[0-9a-fA-F]{12}\b")
_IP = re.compile(r"\b(?:\d{1,3}\.){3}\d{1,3}\b")
_URL = re.compile(r"\bhttps?://\S+\b")
_HEX = re.compile(r"\b0x[0-9a-fA-F]+\b")
_INT = re.compile(r"\b\d+\b")
WILD = "<*>"


def normalize_message(text: str) -> str:
    for rx, tok in ((_TS, "<TS>"), (_GUID, "<GUID>"), (_IP, "<IP>"), (_URL, "<URL>"), (_HEX, "<HEX>"),
                    (_INT, "<NUM>")):
        text = rx.sub(tok, text)
    return " ".join(text.split())


@dataclasses.dataclass
class Cluster:
    cid: int
    tokens: list[str]

    @property
    def template(self) -> str:
        return " ".join(self.tokens)


class Drain:
    def __init__(self, depth: int = 4, sim_th: float = 0.4, max_children: int = 100):
        self.depth, self.sim_th, self.max_children = max(3, depth), sim_th, max_children
        self.root: dict = {}
        self.clusters: list[Cluster] = []

    @staticmethod
    def _has_digit(t: str) -> bool:
        return any(c.isdigit() for c in t)

    def _leaf(self, tokens: list[str]) -> list[Cluster]:
        node = self.root.setdefault(len(tokens), {})
        for t in tokens[:self.depth - 3]:  # depth counts root + length layer + leaf (drain3 convention)
            key = WILD if self._has_digit(t) else t
            if key not in node:
                key = key if len(node) < self.max_children else WILD
            node = node.setdefault(key, {})
        return node.setdefault("__clusters__", [])

    @staticmethod
    def _sim(a: list[str], b: list[str]) -> tuple[float, int]:
        eq = wild = 0
        for x, y in zip(a, b):
            if x == WILD:
                wild += 1
            elif x == y:
                eq += 1
        return eq / max(1, len(a)), wild

    def add(self, message: str) -> Cluster:
        tokens = message.split() or [""]
        group = self._leaf(tokens)
        best, best_key = None, (-1.0, -1)
        for c in group:
            s = self._sim(c.tokens, tokens)
            if s > best_key:
                best, best_key = c, s
        if best is not None and best_key[0] >= self.sim_th:
            best.tokens = [x if x == y else WILD for x, y in zip(best.tokens, tokens)]
            return best
        c = Cluster(len(self.clusters) + 1, list(tokens))
        self.clusters.append(c)
        group.append(c)
        return c


@dataclasses.dataclass
class Record:
    raw: str
    message: str
    service: str | None = None


def parse_line(line: str, fmt: str = "auto") -> Record | None:
    line = line.rstrip("\n")
    if not line.strip():
        return None
    if fmt in ("auto", "jsonl") and line.lstrip().startswith("{"):
        try:
            obj = json.loads(line)
            msg = obj.get("message") or obj.get("msg") or obj.get("log") or ""
            extra = " ".join(f"{k}={obj[k]}" for k in ("error", "event_type") if k in obj)
            return Record(line, f"{msg} {extra}".strip(), obj.get("service") or obj.get("logger") or obj.get("name"))
        except json.JSONDecodeError:
            if fmt == "jsonl":
                return None
    if fmt in ("auto", "docker") and " | " in line:
        svc, _, msg = line.partition(" | ")
        return Record(line, msg, re.sub(r"[-_]\d+$", "", svc.strip()))
    return Record(line, line)


def mine(lines: Iterable[str], fmt: str = "auto", group_by_service: bool = False, samples: int = 3,
         rare_threshold: int = 2, seed: int = 0, **drain_kw) -> dict:
    rng = random.Random(seed)
    miners: dict[str | None, Drain] = {}
    stats: dict[tuple, dict] = {}
    total = parsed = 0
    for line in lines:
        total += 1
        rec = parse_line(line, fmt)
        if rec is None:
            continue
        text = normalize_message(rec.message)
        if not text:
            continue
        parsed += 1
        svc = rec.service if group_by_service else None
        c = miners.setdefault(svc, Drain(**drain_kw)).add(text)
        st = stats.get((svc, c.cid))
        if st is None:
            st = stats[(svc, c.cid)] = {"service": svc, "template_id": str(c.cid), "count": 0, "samples": [],
                                        "first_seen_line": total, "first_seen_raw": rec.raw,
                                        "shortest_sample": rec.raw, "longest_sample": rec.raw, "_c": c}
        st["count"] += 1
        if len(st["samples"]) < samples:              # reservoir sampling of raw lines
            st["samples"].append(rec.raw)
        else:
            j = rng.randrange(st["count"])
            if j < samples:
                st["samples"][j] = rec.raw
        if len(rec.raw) < len(st["shortest_sample"]):
            st["shortest_sample"] = rec.raw
        if len(rec.raw) > len(st["longest_sample"]):
            st["longest_sample"] = rec.raw
    templates = []
    for st in stats.values():
        c = st.pop("_c")
        st["template"] = c.template
        st["placeholders"] = c.template.count(WILD)
        templates.append(st)
    templates.sort(key=lambda t: (-t["count"], t["first_seen_line"]))
    return {"meta": {"created_utc": datetime.now(timezone.utc).isoformat(), "lines_total": total,
                     "lines_parsed": parsed, "templates_total": len(templates),
                     "services": sorted({t["service"] for t in templates if t["service"]})},
            "templates": templates,
            "anomalies": {"rare_templates": [t for t in templates if t["count"] <= rare_threshold],
                          "first_seen": sorted(templates, key=lambda t: t["first_seen_line"])[:20]}}


def _lines(path: str | None) -> Iterator[str]:
    if path in (None, "-"):
        yield from sys.stdin
    else:
        with open(path, encoding="utf-8", errors="replace") as fh:
            yield from fh


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Mine log templates (Drain)")
    ap.add_argument("input", nargs="?", default="-")
    ap.add_argument("--format", default="auto", choices=["auto", "plain", "docker", "jsonl"])
    ap.add_argument("--group-by-service", action="store_true")
    ap.add_argument("--output", default="-")
    ap.add_argument("--sim-th", type=float, default=0.4)
    ap.add_argument("--depth", type=int, default=4)
    a = ap.parse_args(argv)
    rep = mine(_lines(a.input), a.format, a.group_by_service, sim_th=a.sim_th, depth=a.depth)
    text = json.dumps(rep, indent=2)
    if a.output == "-":
        print(text)
    else:
        Path(a.output).parent.mkdir(parents=True, exist_ok=True)
        Path(a.output).write_text(text, encoding="utf-8")
    return 0


if __name__ == "__main__":
    sys.exit(main())
