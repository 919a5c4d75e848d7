"""Stop strings matched as tokens arrive (runtime/stops.py + the decode-advance kernels' stop_feed).

* the host automaton equals brute force (decode the prefix, look for a stop) on random token
  streams of a tokenizer whose tokens split "\\n\\n\\n" every possible way;
* LLMEngine.generate / ContinuousEngine finish a sequence at the token completing the stop, even
  when the stop spans tokens, and the kept tokens equal the unstopped generation cut there;
* on the GPU the same through the captured decode graph and the kernel's stop_feed.
"""
from __future__ import annotations

import random

import pytest
import torch

from copilot_for_consensus_amd.models.decoder import DecoderModel, DecoderWeights, get_config
from copilot_for_consensus_amd.runtime.continuous import ContinuousEngine
from copilot_for_consensus_amd.runtime.engine import LLMEngine
from copilot_for_consensus_amd.runtime.kv_cache import PagedKVCache
from copilot_for_consensus_amd.runtime.stops import StopStringMatcher

STOPS = ["</s>", "\n\n\n"]


class _ToyTok:
    """Byte tokens chosen so stops split across tokens: "\\n", "\\n\\n", ".\\n", "\\nThe", "</",
    "s>", "<", "/s", ">", a leading-space word, ... plus filler words."""
    VOCAB = [b"", b"", b"", b"\n", b"\n\n", b".\n", b"\nThe", b"</", b"s>", b"<", b"/s", b">", b" a", b"b",
             b"x\n\n\ny", b"\n\n\n", b"ok", b" </s", b"> end", b"\n\n\n\n"]

    vocab_size = len(VOCAB)
    strips_leading_space = True

    def token_bytes(self, i):
        return self.VOCAB[i]

    def text(self, ids, strip=True):
        b = b"".join(self.VOCAB[i] for i in ids)
        return b[1:] if strip and b[:1] == b" " else b


def _brute(tok, ids):
    """First i such that the text of ids[:i+1] contains a stop (it must end in token i)."""
    for i in range(len(ids)):
        t = tok.text(ids[:i + 1])
        if any(s.encode() in t for s in STOPS):
            return i
    return None


def test_host_matcher_equals_brute_force():
    tok = _ToyTok()
    m = StopStringMatcher(tok.token_bytes, tok.vocab_size, STOPS, strip_leading_space=True)
    rng = random.Random(0)
    hits = 0
    for _ in range(3000):
        ids = [rng.randrange(3, tok.vocab_size) for _ in range(rng.randrange(1, 12))]
        want = _brute(tok, ids)
        assert m.match_tokens(ids) == want, (ids, [tok.VOCAB[i] for i in ids])
        hits += want is not None
    assert hits > 300       # the streams really exercise the stops


def test_matcher_split_cases():
    tok = _ToyTok()
    m = StopStringMatcher(tok.token_bytes, tok.vocab_size, STOPS, strip_leading_space=True)
    ix = {b: i for i, b in enumerate(tok.VOCAB) if i >= 3}
    assert m.match_tokens([ix[b"\n"], ix[b"\n"], ix[b"\n"]]) == 2
    assert m.match_tokens([ix[b"ok"], ix[b"\n\n"], ix[b"\nThe"]]) == 2
    assert m.match_tokens([ix[b"<"], ix[b"/s"], ix[b">"]]) == 2
    assert m.match_tokens([ix[b"</"], ix[b"s>"]]) == 1
    assert m.match_tokens([ix[b"x\n\n\ny"]]) == 0           # the stop inside one token
    assert m.match_tokens([ix[b"\n"], ix[b"ok"], ix[b"\n\n"]]) is None
    # " </s" as the FIRST token loses its leading space (SentencePiece decode), "> end" completes it
    assert m.match_tokens([ix[b" </s"], ix[b"> end"]]) == 1


def _model(device, seed=5):
    cfg = get_config("tiny")
    model = DecoderModel(DecoderWeights.random(cfg, device, seed=seed))
    kv = PagedKVCache(cfg.layers, 96, cfg.kv_heads, cfg.head_dim, device)
    return model, kv


def _vocab_tok(vocab_size, seed=0):
    """A byte view of the tiny model's vocabulary: many "\\n" pieces so generations hit stops."""
    rng = random.Random(seed)
    pieces = [b"\n", b"\n\n", b".\n", b"</", b"s>", b"a", b" b", b"cd", b"<", b"/s>", b"e"]

    class T:
        strips_leading_space = False

        def __init__(self):
            self.vocab_size = vocab_size
            self.table = [b""] * 3 + [rng.choice(pieces) for _ in range(vocab_size - 3)]

        def token_bytes(self, i):
            return self.table[i]
    return T()


def _stop_checks(device, use_graph):
    model, kv = _model(device)
    tok = _vocab_tok(model.cfg.vocab_size)
    m = StopStringMatcher.for_tokenizer(tok, STOPS)
    eng = LLMEngine(model, kv, max_prefill_tokens=256, use_graph=use_graph)
    prompts = [[1] + list(range(10 + 7 * i, 40 + 7 * i)) for i in range(6)]
    full = eng.generate(prompts, 40, ignore_eos=True).tokens
    cut = [m.match_tokens(g) for g in full]
    assert sum(c is not None for c in cut) >= 2, cut     # the fixture really stops some rows
    res = eng.generate(prompts, 40, ignore_eos=True, stop_strings=m)
    for g, c, got in zip(full, cut, res.tokens):
        assert got == (g if c is None else g[:c + 1])
    # continuous batching: the stopped slot frees and the queue drains with the same outputs
    ce = ContinuousEngine(eng, max_slots=3, max_new_cap=40, max_prompt=128, steps_per_sync=4, stop_strings=m)
    reqs = [ce.submit(p, 40) for p in prompts]
    ce.run()
    ce.close()
    for g, c, r in zip(full, cut, reqs):
        assert r.tokens == (g if c is None else g[:c + 1])
    return res


def test_engine_stops_on_strings_cpu():
    _stop_checks("cpu", use_graph=False)


@pytest.mark.gpu
def test_engine_stops_on_strings_gpu_graph():
    """The kernel's stop_feed inside the captured decode graph (static and continuous engines)."""
    _stop_checks("cuda", use_graph=True)
