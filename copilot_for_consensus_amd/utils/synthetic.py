"""Deterministic synthetic mailing-list archives (.mbox) -- the benchmark's data source.

There is no network, so no real IETF archive can be fetched.  The generator produces threads that
exercise every parser path of the reference (tests/fixtures/mailbox_sample/test-archive.mbox is a
10-message example of the shape): Message-ID / In-Reply-To / References chains, RFC-2047-free
ASCII headers, dates, To/CC lists, quoted reply lines, signatures, RFC and draft mentions.
Bodies use a Zipf-distributed vocabulary of 300k words (a core of technical English plus
syllable-built pseudo-words), so a BPE vocabulary trained on it yields a realistic ~1.3 tokens
per word (measured 1.36) and the orchestrator's 1.3x-words budget behaves as with real mail.

Message shape modelled on the reference fixture tests/fixtures/mailbox_sample/test-archive.mbox
(mbox with RFC 5322 headers, In-Reply-To threading).
"""
from __future__ import annotations

import random
from datetime import datetime, timedelta, timezone
from email.utils import format_datetime

CORE_WORDS = (
    "the of and to in a is that for it as with be on this are by we not or but from at have an will which "
    "can should would there their about more if protocol draft working group consensus proposal document "
    "section text change support agree disagree objection issue comment review implementation security "
    "considerations registry iana extension header field message server client request response option "
    "mechanism requirement normative informative reference update errata version deployment interoperability "
    "specification algorithm key certificate transport layer stream connection congestion latency packet "
    "routing address network encryption authentication authorization privacy tracker milestone charter chair "
    "editor author revision adoption call last meeting minutes interim session slides discussion thread list "
    "question answer clarify suggest propose believe think consider note point concern approach alternative "
    "backward compatibility migration performance overhead complexity testing vectors compliance profile"
).split()

SYLLABLES = ("ka", "ri", "to", "men", "sul", "va", "ne", "qu", "tra", "lo", "pi", "zer", "dan", "fe", "mo", "ix",
             "bre", "cal", "dor", "en", "gra", "hul", "ist", "jo", "kel", "lum", "nar", "ost", "pel", "rin", "sta",
             "ther", "ur", "vel", "wes", "yo", "zan", "ble", "cor", "dis", "ent", "for", "gen", "hab", "ic", "jun")

FIRST = ("Alice", "Bob", "Carol", "Dave", "Erin", "Frank", "Grace", "Heidi", "Ivan", "Judy", "Mallory", "Niaj",
         "Olivia", "Peggy", "Rupert", "Sybil", "Trent", "Uma", "Victor", "Walter", "Xena", "Yuri", "Zoe", "Quinn")
LAST = ("Smith", "Jones", "Garcia", "Chen", "Kumar", "Nakamura", "Okafor", "Rossi", "Schmidt", "Dubois", "Silva",
        "Novak", "Haddad", "Larsen", "Moreau", "Ivanova", "Kowalski", "Tanaka", "Fischer", "Bianchi")
DOMAINS = ("example.com", "example.org", "ietf.example", "vendor.example", "univ.example.edu")
TOPICS = ("transport parameters", "key update", "congestion control", "header compression", "error codes",
          "version negotiation", "privacy considerations", "registry policy", "extension framework",
          "path validation", "address migration", "flow control limits", "datagram support", "rate limiting")


_VOCAB_CACHE: dict = {}


def _vocabulary(vocab_size: int, zipf_s: float):
    key = (vocab_size, zipf_s)
    if key not in _VOCAB_CACHE:
        vr = random.Random(12345)  # the vocabulary is fixed across archive seeds
        words = list(CORE_WORDS)
        seen = set(words)
        while len(words) < vocab_size:
            w = "".join(vr.choice(SYLLABLES) for _ in range(vr.choice((1, 2, 2, 3, 3, 4))))
            if w not in seen:
                seen.add(w)
                words.append(w)
        weights = [1.0 / (r + 1) ** zipf_s for r in range(len(words))]
        tot = sum(weights)
        acc, cum = 0.0, []
        for x in weights:
            acc += x / tot
            cum.append(acc)
        people = [(f"{f} {l}", f"{f.lower()}.{l.lower()}@{vr.choice(DOMAINS)}") for f in FIRST for l in LAST]
        _VOCAB_CACHE[key] = (words, cum, people)
    return _VOCAB_CACHE[key]


class SyntheticArchive:
    def __init__(self, seed: int = 0, vocab_size: int = 300000, zipf_s: float = 0.95):
        self.rng = random.Random(seed)
        self.words, self._cum, self.people = _vocabulary(vocab_size, zipf_s)
        self._msg_counter = 0

    def _word(self) -> str:
        import bisect
        return self.words[min(bisect.bisect_left(self._cum, self.rng.random()), len(self.words) - 1)]

    def sentence(self, n: int | None = None) -> str:
        n = n or self.rng.randint(8, 24)
        ws = [self._word() for _ in range(n)]
        r = self.rng.random()
        if r < 0.06:
            ws.insert(self.rng.randrange(len(ws)), f"RFC {self.rng.randint(700, 9700)}")
        elif r < 0.12:
            ws.insert(self.rng.randrange(len(ws)),
                      f"draft-ietf-{self.rng.choice(('quic', 'tls', 'httpbis', 'mls', 'ohai'))}-"
                      f"{self._word()}-{self.rng.randint(0, 19):02d}")
        s = " ".join(ws)
        return s[0].upper() + s[1:] + self.rng.choice((".", ".", ".", "?", "!"))

    def paragraph(self, words: int) -> str:
        out, n = [], 0
        while n < words:
            s = self.sentence()
            out.append(s)
            n += len(s.split())
        return " ".join(out)

    def body(self, words: int, quote: str | None) -> str:
        parts = []
        if quote:
            ql = quote.split(". ")[:3]
            parts.append("\n".join("> " + q for q in ql))
            parts.append("")
        remaining = words
        while remaining > 0:
            n = min(remaining, self.rng.randint(60, 160))
            parts.append(self.paragraph(n))
            parts.append("")
            remaining -= n
        parts.append("-- \n" + self.rng.choice(("Regards", "Thanks", "Best", "Cheers")))
        return "\n".join(parts)

    def thread(self, n_messages: int, words_per_message: tuple[int, int] = (300, 700), t0: datetime | None = None,
               list_name: str = "wg") -> list[bytes]:
        """One discussion thread as a list of RFC-822 messages (bytes, no mbox From_ line)."""
        t = t0 or datetime(2025, 1, 1, tzinfo=timezone.utc) + timedelta(minutes=self.rng.randint(0, 500000))
        topic = self.rng.choice(TOPICS)
        subject = f"[{list_name}] {topic.capitalize()} for {self._word()} {self._word()}"
        participants = self.rng.sample(self.people, k=min(len(self.people), self.rng.randint(3, 8)))
        msgs, ids, bodies = [], [], []
        for i in range(n_messages):
            self._msg_counter += 1
            mid = f"<{self._msg_counter}.{self.rng.getrandbits(48):012x}@{self.rng.choice(DOMAINS)}>"
            name, email = participants[i % len(participants)] if i else participants[0]
            parent = None if i == 0 else self.rng.randrange(max(0, i - 3), i)
            body = self.body(self.rng.randint(*words_per_message), bodies[parent] if parent is not None else None)
            hdr = [f"From: {name} <{email}>",
                   f"To: {list_name}@ietf.example",
                   f"Cc: {participants[(i + 1) % len(participants)][1]}",
                   f"Subject: {'Re: ' if i else ''}{subject}",
                   f"Date: {format_datetime(t)}",
                   f"Message-ID: {mid}"]
            if parent is not None:
                hdr.append(f"In-Reply-To: {ids[parent]}")
                hdr.append(f"References: {' '.join(ids[:parent + 1])}")
            hdr += ["MIME-Version: 1.0", "Content-Type: text/plain; charset=utf-8",
                    "Content-Transfer-Encoding: 8bit", "X-Mailer: synthetic-mua 1.0"]
            msgs.append(("\n".join(hdr) + "\n\n" + body + "\n").encode())
            ids.append(mid)
            bodies.append(body.split("\n\n")[-2] if "\n\n" in body else body)
            t += timedelta(minutes=self.rng.randint(5, 2000))
        return msgs

    def mbox(self, n_threads: int, messages_per_thread: tuple[int, int] = (5, 9), **kw) -> bytes:
        out = []
        for _ in range(n_threads):
            for m in self.thread(self.rng.randint(*messages_per_thread), **kw):
                out.append(b"From synthetic@example.com Thu Jan  1 00:00:00 2025\n")
                out.append(m.replace(b"\nFrom ", b"\n>From "))
                out.append(b"\n")
        return b"".join(out)

    def corpus(self, n_words: int) -> str:
        """Plain text drawn from the same distribution (tokenizer training)."""
        return "\n".join(self.paragraph(200) for _ in range(max(1, n_words // 200)))
