"""Consensus detection over a discussion thread.

Parity target: adapters/copilot_consensus/copilot_consensus/consensus.py of the reference
(levels :33, ConsensusSignal :45, HeuristicConsensusDetector :90 with its decision ladder
stagnation -> dissent -> (strong) consensus -> weak -> none :167-272, Mock :290, factory :399) and
thread.py (Message / Thread with message/reply/participant counts).

Differences by design:
  * patterns are compiled once per process (count = patterns matched per message, summed);
  * ``MLConsensusDetector`` is implemented instead of raising NotImplementedError: it embeds every
    message in ONE batched encoder call (the HIP encoder on the GPU) and scores it against
    agreement / dissent prototype sentences -- cosine to the nearest prototype of each class,
    thresholded, replaces the keyword match; the same ladder then decides the level.  A prototype
    file (``model_path``, JSON ``{"agreement": [...], "dissent": [...]}``) overrides the built-ins.

Reference: adapters/copilot_consensus/copilot_consensus/consensus.py:68 (ConsensusDetector), :90
(heuristic), :290 (mock), :351-393 (ML detector, NotImplementedError there).
"""
from __future__ import annotations

import dataclasses
import enum
import json
import re
from datetime import datetime, timezone
from typing import Any, Sequence


class ConsensusLevel(enum.Enum):
    STRONG_CONSENSUS = "strong_consensus"
    CONSENSUS = "consensus"
    WEAK_CONSENSUS = "weak_consensus"
    NO_CONSENSUS = "no_consensus"
    DISSENT = "dissent"
    STAGNATION = "stagnation"

    @classmethod
    def parse(cls, v) -> "ConsensusLevel":
        if isinstance(v, cls):
            return v
        key = str(v).strip().lower().replace("-", "_").replace(" ", "_")
        for lv in cls:
            if lv.value == key:
                return lv
        raise ValueError(f"Invalid consensus level: {v}")


@dataclasses.dataclass
class ConsensusSignal:
    level: ConsensusLevel
    confidence: float
    signals: list[str] = dataclasses.field(default_factory=list)
    explanation: str = ""
    metadata: dict[str, Any] = dataclasses.field(default_factory=dict)

    def __post_init__(self):
        if not 0.0 <= self.confidence <= 1.0:
            raise ValueError(f"Confidence must be between 0.0 and 1.0, got {self.confidence}")

    def to_dict(self) -> dict:
        return {"level": self.level.value, "confidence": self.confidence, "signals": list(self.signals),
                "explanation": self.explanation, "metadata": dict(self.metadata)}


@dataclasses.dataclass
class Message:
    message_id: str
    author: str
    subject: str
    content: str
    timestamp: datetime
    in_reply_to: str | None = None
    metadata: dict[str, Any] = dataclasses.field(default_factory=dict)


@dataclasses.dataclass
class Thread:
    thread_id: str
    subject: str
    messages: list[Message] = dataclasses.field(default_factory=list)
    started_at: datetime | None = None
    last_activity_at: datetime | None = None
    metadata: dict[str, Any] = dataclasses.field(default_factory=dict)

    def __post_init__(self):
        if self.messages:
            stamps = [m.timestamp for m in self.messages]
            self.started_at = self.started_at or min(stamps)
            self.last_activity_at = self.last_activity_at or max(stamps)

    @property
    def message_count(self) -> int:
        return len(self.messages)

    @property
    def reply_count(self) -> int:
        return max(0, len(self.messages) - 1)

    @property
    def participant_count(self) -> int:
        return len({m.author for m in self.messages})

    @classmethod
    def from_documents(cls, thread_doc: dict, message_docs: Sequence[dict]) -> "Thread":
        """Build from the pipeline's ``threads`` / ``messages`` documents."""
        msgs = []
        for d in message_docs:
            ts = d.get("date") or d.get("created_at")
            if isinstance(ts, str):
                try:
                    ts = datetime.fromisoformat(ts.replace("Z", "+00:00"))
                except ValueError:
                    ts = None
            frm = d.get("from") or {}
            author = frm.get("email") or frm.get("name") if isinstance(frm, dict) else str(frm)
            msgs.append(Message(d.get("message_id") or d.get("_id", ""), author or "", d.get("subject", ""),
                                d.get("body_normalized", "") or "", ts or datetime.now(timezone.utc),
                                d.get("in_reply_to")))
        return cls(thread_doc.get("_id") or thread_doc.get("thread_id", ""), thread_doc.get("subject", ""), msgs)


class ConsensusDetector:
    def detect(self, thread: Thread) -> ConsensusSignal:
        raise NotImplementedError

    def detect_batch(self, threads: Sequence[Thread]) -> list[ConsensusSignal]:
        return [self.detect(t) for t in threads]


AGREEMENT_PATTERNS = (r"\+1\b", r"\bLGTM\b", r"\bI agree\b", r"\bagree with\b", r"\bsounds good\b",
                      r"\bmakes sense\b", r"\bsupport this\b", r"\bapprove\b", r"\bconcur\b")
DISSENT_PATTERNS = (r"\bdisagree\b", r"\boppose\b", r"\bconcern\b", r"\bproblem with\b", r"\bissue with\b",
                    r"\bnot sure\b", r"\bwait\b", r"\bhold on\b", r"-1\b")


def _literal(p: str) -> str:
    """The lowercased literal every match of a word-boundary pattern contains ('+1', 'lgtm', ...)."""
    return p.replace(r"\b", "").replace("\\", "").lower()


def _compile(patterns):
    return tuple((_literal(p), re.compile(p, re.IGNORECASE)) for p in patterns)


class _Ladder:
    """The shared decision ladder: stagnation -> dissent -> consensus tiers -> weak -> none."""

    def __init__(self, agreement_threshold: int = 3, min_participants: int = 2, stagnation_days: int = 7):
        self.agreement_threshold = int(agreement_threshold)
        self.min_participants = int(min_participants)
        self.stagnation_days = int(stagnation_days)

    def decide(self, thread: Thread, agree: int, dissent: int, meta: dict | None = None) -> ConsensusSignal:
        meta = dict(meta or {})
        meta.update(message_count=thread.message_count, reply_count=thread.reply_count,
                    participant_count=thread.participant_count, agreement_signals=agree, dissent_signals=dissent)
        if thread.last_activity_at is not None:
            last = thread.last_activity_at
            last = last.replace(tzinfo=timezone.utc) if last.tzinfo is None else last.astimezone(timezone.utc)
            idle = (datetime.now(timezone.utc) - last).days
            meta["days_since_activity"] = idle
            if idle > self.stagnation_days:
                return ConsensusSignal(ConsensusLevel.STAGNATION, 0.8, [f"No activity for {idle} days"],
                                       f"Thread has been inactive for {idle} days", meta)
        if dissent > 0:
            return ConsensusSignal(ConsensusLevel.DISSENT, min(0.9, 0.5 + 0.1 * dissent),
                                   [f"Found {dissent} dissent signal(s)"],
                                   f"Thread shows dissent with {dissent} opposing view(s)", meta)
        parts = thread.participant_count
        if agree >= self.agreement_threshold and parts >= self.min_participants:
            sig = [f"Found {agree} agreement signal(s)", f"{parts} participant(s) engaged"]
            if agree >= 2 * self.agreement_threshold:
                return ConsensusSignal(ConsensusLevel.STRONG_CONSENSUS, min(0.95, 0.7 + 0.05 * agree), sig,
                                       f"Strong consensus with {agree} agreement signals from {parts} participants",
                                       meta)
            return ConsensusSignal(ConsensusLevel.CONSENSUS, min(0.85, 0.6 + 0.05 * agree), sig,
                                   f"Consensus detected with {agree} agreement signals from {parts} participants", meta)
        replies = thread.reply_count
        if agree > 0 or replies >= 2:
            return ConsensusSignal(ConsensusLevel.WEAK_CONSENSUS, 0.5,
                                   [f"Limited agreement ({agree} signal(s))", f"{replies} reply/replies"],
                                   f"Weak consensus with limited engagement ({replies} replies, {agree} agreements)",
                                   meta)
        return ConsensusSignal(ConsensusLevel.NO_CONSENSUS, 0.7, ["Insufficient activity or agreement signals"],
                               "No clear consensus detected in thread", meta)


class HeuristicConsensusDetector(ConsensusDetector, _Ladder):
    _AGREE = _compile(AGREEMENT_PATTERNS)
    _DISSENT = _compile(DISSENT_PATTERNS)

    @staticmethod
    def _count(pats, text: str) -> int:
        # patterns matched per message (not occurrences), summed over messages -- reference semantics.
        # ASCII text: a pattern whose literal is not a substring of the lowercased text cannot match,
        # so the regex runs only for the few present (the orchestrator scans every message of every
        # thread it requests; 18 IGNORECASE searches per message were most of its CPU time)
        if text.isascii():
            low = text.lower()
            return sum(1 for lit, rx in pats if lit in low and rx.search(text))
        return sum(1 for _, rx in pats if rx.search(text))

    def count_patterns(self, thread: Thread) -> tuple[int, int]:
        a = d = 0
        for m in thread.messages:
            a += self._count(self._AGREE, m.content)
            d += self._count(self._DISSENT, m.content)
        return a, d

    def detect(self, thread: Thread) -> ConsensusSignal:
        a, d = self.count_patterns(thread)
        return self.decide(thread, a, d)


class MockConsensusDetector(ConsensusDetector):
    def __init__(self, level="consensus", confidence: float = 0.8):
        self.level = ConsensusLevel.parse(level)
        self.confidence = float(confidence)

    def detect(self, thread: Thread) -> ConsensusSignal:
        return ConsensusSignal(self.level, self.confidence, ["mock_signal"], f"Mock detection: {self.level.value}",
                               {"mock": True, "thread_id": thread.thread_id})


DEFAULT_PROTOTYPES = {
    "agreement": ["I agree with this proposal.", "+1, looks good to me.", "LGTM, ship it.",
                  "This makes sense and I support adopting it.", "Sounds good, no objections from me.",
                  "I concur with the previous message."],
    "dissent": ["I disagree with this change.", "I have serious concerns about this approach.",
                "I oppose adopting this draft.", "There is a problem with this proposal.",
                "Hold on, I am not sure this is right.", "-1, this breaks existing deployments."],
}


class MLConsensusDetector(ConsensusDetector, _Ladder):
    """Embedding-prototype classifier: one batched encoder call per thread batch (see module doc)."""

    def __init__(self, model_path: str | None = None, embedding_provider=None, agree_threshold: float = 0.6,
                 dissent_threshold: float = 0.6, **ladder):
        _Ladder.__init__(self, **ladder)
        self.model_path = model_path
        protos = DEFAULT_PROTOTYPES
        if model_path:
            with open(model_path, encoding="utf-8") as fh:
                protos = json.load(fh)
        if embedding_provider is None:
            from ..embedding import create_embedding_provider
            embedding_provider = create_embedding_provider("hip")
        self.embedder = embedding_provider
        self.agree_threshold, self.dissent_threshold = agree_threshold, dissent_threshold
        self._protos = {k: self._embed(v) for k, v in protos.items()}

    def _embed(self, texts):
        import torch
        if hasattr(self.embedder, "embed_tensor"):
            x = self.embedder.embed_tensor(list(texts)).float()
        else:
            x = torch.tensor([self.embedder.embed(t) for t in texts], dtype=torch.float32)
        return torch.nn.functional.normalize(x, dim=-1)

    def detect_batch(self, threads: Sequence[Thread]) -> list[ConsensusSignal]:
        texts = [m.content or " " for t in threads for m in t.messages]
        out = []
        if not texts:
            return [self.decide(t, 0, 0, {"detector": "ml"}) for t in threads]
        E = self._embed(texts)
        agree = (E @ self._protos["agreement"].to(E.device).T).max(dim=1).values
        diss = (E @ self._protos["dissent"].to(E.device).T).max(dim=1).values
        is_agree = ((agree >= self.agree_threshold) & (agree > diss)).cpu()
        is_diss = ((diss >= self.dissent_threshold) & (diss >= agree)).cpu()
        off = 0
        for t in threads:
            n = len(t.messages)
            a, d = int(is_agree[off:off + n].sum()), int(is_diss[off:off + n].sum())
            out.append(self.decide(t, a, d, {"detector": "ml"}))
            off += n
        return out

    def detect(self, thread: Thread) -> ConsensusSignal:
        return self.detect_batch([thread])[0]


def create_consensus_detector(cfg=None, **overrides) -> ConsensusDetector:
    name = str(getattr(cfg, "driver_name", cfg) or "heuristic").strip().lower()
    kw = {k: v for k, v in dict(getattr(cfg, "driver_config", {}) or {}).items() if v is not None}
    kw.update(overrides)
    if name == "heuristic":
        return HeuristicConsensusDetector(**{k: kw[k] for k in ("agreement_threshold", "min_participants",
                                                                "stagnation_days") if k in kw})
    if name == "mock":
        return MockConsensusDetector(kw.get("level", "consensus"), kw.get("confidence", 0.8))
    if name == "ml":
        return MLConsensusDetector(**kw)
    raise ValueError(f"Unknown consensus_detector driver: {name!r}")
