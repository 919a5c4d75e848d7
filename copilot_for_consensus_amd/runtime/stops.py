"""Stop strings evaluated on the device, inside the captured decode step.

llama.cpp stops generating as soon as the detokenized text contains one of the request's stop
strings (the reference passes ``["</s>", "\\n\\n\\n"]``, llamacpp_summarizer.py:111-113).  A stop
string is text, not a token: "\\n\\n\\n" can arrive as one token, as "\\n\\n" + "\\n", as ".\\n" +
"\\n\\n" + "The" ...  So each decode slot carries a short byte window (the last L-1 bytes of its
generated text, L = the longest stop) and every sampled token is matched against the stops as

    window + token bytes  ->  stop occurrence ending inside the token?

From the tokenizer's per-token byte strings (``token_bytes``) this module builds, once per stop
set, four device tables indexed by token id -- the first L bytes, the last L-1 bytes, the byte
length, and whether a stop lies entirely inside the token -- which the decode-advance kernels
(csrc/kernels/elementwise.hip: stop_feed) read.  A slot that matches is finished on the device, so
the engine stops decoding it (the continuous engine frees and refills it) instead of generating all
``max_new`` tokens and cutting the text afterwards.  :meth:`StopStringMatcher.feed` is the host
reference of the same automaton (the CPU path, the prefill's first token, and the tests).
"""
from __future__ import annotations

import copy

import numpy as np
import torch

MAX_STOP_BYTES = 32


class StopStringMatcher:
    def __init__(self, token_bytes, vocab_size: int, stops, strip_leading_space: bool = False):
        self.stops = [s.encode("utf-8") if isinstance(s, str) else bytes(s) for s in stops if s]
        if not self.stops:
            raise ValueError("no stop strings")
        L = max(len(s) for s in self.stops)
        if L > MAX_STOP_BYTES:
            raise ValueError(f"stop strings longer than {MAX_STOP_BYTES} bytes are not supported")
        self.L, self.H = L, max(1, L - 1)
        self.strip = bool(strip_leading_space)
        self.V = int(vocab_size)
        head = np.zeros((self.V, L), np.uint8)
        tail = np.zeros((self.V, self.H), np.uint8)
        lens = np.zeros(self.V, np.int32)
        contains = np.zeros(self.V, np.uint8)
        self._bytes = []
        for v in range(self.V):
            b = token_bytes(v)
            self._bytes.append(b)
            lens[v] = len(b)
            hb = b[:L]
            head[v, :len(hb)] = np.frombuffer(hb, np.uint8)
            tb = b[-self.H:] if b else b""
            tail[v, :len(tb)] = np.frombuffer(tb, np.uint8)
            # a stop entirely inside the token (checked on the token as it would appear mid-text)
            contains[v] = any(s in b for s in self.stops)
        self.tables = {"head": head, "tail": tail, "len": lens, "contains": contains}
        smat = np.zeros((len(self.stops), L), np.uint8)
        for i, s in enumerate(self.stops):
            smat[i, :len(s)] = np.frombuffer(s, np.uint8)
        self.stop_mat = smat
        self.stop_lens = np.asarray([len(s) for s in self.stops], np.int32)
        self._dev: dict = {}

    @classmethod
    def for_tokenizer(cls, tokenizer, stops) -> "StopStringMatcher | None":
        stops = [s for s in (stops or ()) if s]
        if not stops or not hasattr(tokenizer, "token_bytes"):
            return None
        return cls(tokenizer.token_bytes, tokenizer.vocab_size, stops,
                   getattr(tokenizer, "strips_leading_space", False))

    # ---------------------------------------------------------------- host reference
    def initial(self) -> tuple[bytes, bool]:
        """Per-slot state: (last H bytes of the generated text, nothing generated yet)."""
        return b"", True

    def feed(self, state: tuple[bytes, bool], tok: int) -> tuple[tuple[bytes, bool], bool]:
        win, fresh = state
        b = self._bytes[tok] if 0 <= tok < self.V else b""
        if fresh and self.strip and b[:1] == b" ":
            b = b[1:]
        hit = bool(self.tables["contains"][tok]) if 0 <= tok < self.V else False
        if not hit and b:
            text = win + b
            for s in self.stops:
                # an occurrence that ends inside the token's bytes
                start = max(0, len(win) - len(s) + 1)
                if text.find(s, start) >= 0:
                    hit = True
                    break
        text = win + b
        return (text[-self.H:] if len(text) > self.H else text, fresh and not b), hit

    def match_tokens(self, toks) -> int | None:
        """Index of the token that completes the first stop, or None (host reference)."""
        st = self.initial()
        for i, t in enumerate(toks):
            st, hit = self.feed(st, int(t))
            if hit:
                return i
        return None

    # ---------------------------------------------------------------- device side
    def device_tables(self, device) -> dict:
        key = str(device)
        if key not in self._dev:
            d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(device) for k, v in self.tables.items()}
            d["stops"] = torch.from_numpy(self.stop_mat).to(device)
            d["stop_lens"] = torch.from_numpy(self.stop_lens).to(device)
            self._dev[key] = d
        return self._dev[key]

    def new_state(self, B: int, device) -> "StopState":
        return StopState(self, B, device)


class StopState:
    """Per-slot device state of the matcher for one decode batch (static buffers a captured graph
    reads and writes): window bytes [B, H], window length [B] (-1 = nothing generated yet, so a
    SentencePiece leading space can be dropped as decode() does), and ``keep`` [B] = tokens to keep
    (the count through the stop-completing token; ``cap`` while the slot runs on)."""

    def __init__(self, m: StopStringMatcher, B: int, device, cap: int = 1 << 30):
        self.m = m
        self.tables = m.device_tables(device)
        self.win = torch.zeros(B, m.H, dtype=torch.uint8, device=device)
        self.wlen = torch.full((B,), -1, dtype=torch.int32, device=device)
        self.keep = torch.full((B,), cap, dtype=torch.int32, device=device)
        self.cap = cap

    def set_slots(self, idx, states, keep=None) -> None:
        """Install host-side states (after the prefill's first token) for slots ``idx``."""
        H = self.m.H
        win = np.zeros((len(idx), H), np.uint8)
        wl = np.zeros(len(idx), np.int32)
        for i, (w, fresh) in enumerate(states):
            win[i, :len(w)] = np.frombuffer(w, np.uint8)
            wl[i] = -1 if fresh else len(w)
        it = torch.as_tensor(list(idx), dtype=torch.long, device=self.win.device)
        self.win.index_copy_(0, it, torch.from_numpy(win).to(self.win.device))
        self.wlen.index_copy_(0, it, torch.from_numpy(wl).to(self.win.device))
        kp = torch.full((len(idx),), self.cap, dtype=torch.int32) if keep is None else \
            torch.as_tensor(keep, dtype=torch.int32)
        self.keep.index_copy_(0, it, kp.to(self.win.device))

    def view(self, W: int) -> "StopState":
        """The same state restricted to the first W slots (row views of the same buffers)."""
        v = copy.copy(self)
        v.win, v.wlen, v.keep = self.win[:W], self.wlen[:W], self.keep[:W]
        return v

    def kernel_args(self) -> dict:
        t = self.tables
        return dict(head=t["head"], tail=t["tail"], tlen=t["len"], contains=t["contains"], stops=t["stops"],
                    stop_lens=t["stop_lens"], n_str=len(self.m.stops), L=self.m.L, H=self.m.H,
                    strip=int(self.m.strip), win=self.win, wlen=self.wlen, keep=self.keep)

    def host_feed(self, b: int, tok: int) -> bool:
        """CPU path: advance slot b's state by one token; True when a stop completed."""
        w = int(self.wlen[b])
        st = (bytes(self.win[b, :max(w, 0)].tolist()), w < 0)
        st, hit = self.m.feed(st, tok)
        self.win[b].zero_()
        if st[0]:
            self.win[b, :len(st[0])] = torch.tensor(list(st[0]), dtype=torch.uint8)
        self.wlen[b] = -1 if st[1] else len(st[0])
        return hit
