"""Continuous batching (runtime/continuous.py): requests of different lengths and token limits,
submitted while others are decoding, produce exactly what LLMEngine.generate produces for each
request alone (greedy), slots are recycled, and every KV block is returned."""
from __future__ import annotations

import pytest
import torch

from copilot_for_consensus_amd.models.decoder import DecoderModel, DecoderWeights, get_config
from copilot_for_consensus_amd.runtime.continuous import ContinuousEngine
from copilot_for_consensus_amd.runtime.engine import LLMEngine
from copilot_for_consensus_amd.runtime.kv_cache import PagedKVCache


def _setup(device, seed=3, blocks=96):
    cfg = get_config("tiny")
    model = DecoderModel(DecoderWeights.random(cfg, device, seed=seed))
    kv = PagedKVCache(cfg.layers, blocks, cfg.kv_heads, cfg.head_dim, device)
    return model, kv


def _requests():
    g = torch.Generator().manual_seed(0)
    out = []
    for i in range(11):
        n = int(torch.randint(3, 150, (1,), generator=g))
        out.append(([1] + torch.randint(3, 500, (n,), generator=g).tolist(), int(torch.randint(1, 20, (1,), generator=g))))
    return out


def _run_continuous(model, kv, reqs, slots, use_graph):
    eng = LLMEngine(model, kv, max_prefill_tokens=128, use_graph=use_graph)
    ce = ContinuousEngine(eng, max_slots=slots, max_new_cap=24, max_prompt=256, steps_per_sync=3)
    free0 = kv.pool.num_free()
    handles, finished = [], []
    # staggered arrivals: 4 requests up front, then one more every step
    for p, m in reqs[:4]:
        handles.append(ce.submit(p, m))
    for p, m in reqs[4:]:
        finished += ce.step()
        handles.append(ce.submit(p, m))
    finished += ce.run()
    assert sorted(r.rid for r in finished) == list(range(len(reqs)))
    ce.close()
    assert kv.pool.num_free() + (eng.prefix_cache.cached_blocks() if eng.prefix_cache else 0) == free0 + 1
    return eng, [h.tokens for h in handles], ce.stats


def test_continuous_equals_per_request_generate_cpu():
    model, kv = _setup("cpu")
    reqs = _requests()
    eng, got, stats = _run_continuous(model, kv, reqs, slots=4, use_graph=False)
    want = [eng.generate([p], m, ignore_eos=True).tokens[0] for p, m in reqs]
    assert got == want
    assert stats["admitted"] == len(reqs) and stats["finished"] == len(reqs)


def test_stop_ids_finish_a_slot_early_cpu():
    model, kv = _setup("cpu")
    eng = LLMEngine(model, kv, max_prefill_tokens=128, use_graph=False)
    p = [1, 5, 9, 11, 13]
    full = eng.generate([p], 12, ignore_eos=True).tokens[0]
    stop = full[5]
    ce = ContinuousEngine(eng, max_slots=2, max_new_cap=16, max_prompt=64, steps_per_sync=4, stop_ids=(stop,))
    r = ce.submit(p, 12)
    ce.run()
    assert r.tokens == full[:full.index(stop)]


@pytest.mark.gpu
def test_continuous_gpu_graph_matches_generate():
    model, kv = _setup("cuda")
    reqs = _requests()
    eng, got, _ = _run_continuous(model, kv, reqs, slots=4, use_graph=True)
    want = [eng.generate([p], m, ignore_eos=True).tokens[0] for p, m in reqs]
    # different batch compositions can pick different GEMM kernels: allow rare bf16 near-tie flips
    agree = sum(a == b for x, y in zip(got, want) for a, b in zip(x, y))
    assert [len(x) for x in got] == [len(x) for x in want]
    assert agree >= 0.95 * sum(len(x) for x in want), (got, want)


def test_failed_admission_returns_blocks_and_requeues(monkeypatch):
    model, kv = _setup("cpu")
    eng = LLMEngine(model, kv, max_prefill_tokens=128, use_graph=False)
    ce = ContinuousEngine(eng, max_slots=2, max_new_cap=8, max_prompt=64, steps_per_sync=2)
    free0 = kv.pool.num_free()
    ce.submit([1, 2, 3, 4], 4)

    def boom(*a, **k):
        raise RuntimeError("HIP out of memory")
    monkeypatch.setattr(eng, "_prefill", boom)
    with pytest.raises(RuntimeError):
        ce.step()
    cached = eng.prefix_cache.cached_blocks() if eng.prefix_cache else 0
    assert kv.pool.num_free() + cached == free0 and len(ce.queue) == 1 and len(ce.free) == 2
    monkeypatch.undo()
    assert len(ce.run()) == 1


def test_admission_waits_for_kv_blocks_instead_of_failing():
    """With a KV cache too small for every queued request at once, admission takes what fits and
    the rest waits for finished slots to return their blocks (the LLM server's load case)."""
    import torch
    from copilot_for_consensus_amd.models.decoder import DecoderModel, DecoderWeights, get_config
    from copilot_for_consensus_amd.runtime.continuous import ContinuousEngine
    from copilot_for_consensus_amd.runtime.engine import LLMEngine
    from copilot_for_consensus_amd.runtime.kv_cache import PagedKVCache, blocks_needed
    cfg = get_config("tiny")
    model = DecoderModel(DecoderWeights.random(cfg, "cpu", seed=5))
    per = blocks_needed(60 + 8)
    kv = PagedKVCache(cfg.layers, 2 * per + 1 + 1, model.w.kv_heads, cfg.head_dim, "cpu")   # 2 requests + scratch
    eng = LLMEngine(model, kv, prefix_cache=False)
    ce = ContinuousEngine(eng, max_slots=4, max_new_cap=8, max_prompt=64, steps_per_sync=4)
    prompts = [[1] + [(3 * i + j) % 500 + 3 for j in range(59)] for i in range(5)]
    reqs = [ce.submit(p, 8) for p in prompts]
    done = ce.run()
    assert len(done) == 5 and all(len(r.tokens) == 8 for r in reqs)
    want = eng.generate([prompts[4]], 8, temperature=0.0, ignore_eos=True).tokens[0]
    assert reqs[4].tokens == want


def test_bulk_admission_fills_a_mostly_empty_batch_in_one_prefill():
    """A backlog larger than the admission token budget: with most slots free the budget is lifted
    and every free slot is filled by one admission (no staggered groups); with bulk admission off
    the budget splits it.  Outputs are the same either way."""
    model, kv = _setup("cpu", blocks=160)
    reqs = [([1] + [(7 * i + j) % 400 + 3 for j in range(90)], 6) for i in range(8)]
    out = {}
    for frac in (0.5, 0.0):
        eng = LLMEngine(model, kv, max_prefill_tokens=64, use_graph=False, prefix_cache=False)
        ce = ContinuousEngine(eng, max_slots=8, max_new_cap=8, max_prompt=128, steps_per_sync=2,
                              max_admit_tokens=200, bulk_admit_frac=frac)
        hs = [ce.submit(p, m) for p, m in reqs]
        ce.run()
        ce.close()
        out[frac] = ([h.tokens for h in hs], ce.stats["admissions"])
    assert out[0.5][1] == 1
    assert out[0.0][1] == 4          # 91-token prompts, 200-token budget: 2 per admission
    assert out[0.5][0] == out[0.0][0]


def _hip_summarizer(**kw):
    from copilot_for_consensus_amd.summarization import HipLLMSummarizer
    return HipLLMSummarizer(model="tiny", device="cpu", kv_cache_tokens=8192, ignore_eos=True, **kw)


def test_stop_continuous_fails_every_unfinished_thread_exactly_once():
    """Stopping the service engine with threads queued and running: every submitted thread gets
    its callback exactly once -- a summary or an error -- so none is dropped silently."""
    import collections
    import time

    from copilot_for_consensus_amd.summarization import Thread
    s = _hip_summarizer(max_new_tokens=300, max_batch=2)
    s.start_continuous(steps_per_sync=4, min_admit=1, max_wait_s=0.0)
    calls, errs = collections.Counter(), {}

    def cb(tid):
        def done(summary, err):
            calls[tid] += 1
            errs[tid] = err
        return done
    for i in range(6):
        s.submit(Thread(f"t{i}", ["m"], prompt="word " * 30), cb(f"t{i}"))
    time.sleep(0.3)
    s.stop_continuous()
    assert sorted(calls) == [f"t{i}" for i in range(6)] and set(calls.values()) == {1}, calls
    assert any(e is not None for e in errs.values())       # 2 slots x 300 tokens: not all could finish
    with pytest.raises(RuntimeError):        # a stopped engine refuses new threads (the bus redelivers)
        s.submit(Thread("late", ["m"]), cb("late"))


def test_raising_done_callback_is_not_called_twice():
    """A callback that raises (e.g. its publish failed after the summary was built) is logged, not
    re-invoked with an error -- a second call would publish SummarizationFailed for a thread whose
    SummaryComplete may already be out."""
    import time

    from copilot_for_consensus_amd.summarization import Thread
    s = _hip_summarizer(max_new_tokens=4, max_batch=2)
    s.start_continuous(steps_per_sync=2, min_admit=1, max_wait_s=0.0)
    seen = []

    def done(summary, err):
        seen.append((summary is not None, err))
        raise ConnectionError("bus down")
    s.submit(Thread("x", ["m"], prompt="word " * 10), done)
    deadline = time.time() + 60
    while not seen and time.time() < deadline:
        time.sleep(0.02)
    time.sleep(0.2)
    s.stop_continuous()
    assert seen == [(True, None)], seen


def test_decode_width_follows_the_occupied_slots_cpu():
    """A burst decodes only the first W slots (W the smallest width bucket holding every occupied
    slot; admission takes the lowest free slot): one request alone runs at width 1, tokens still
    equal generate(), and a freed low slot is refilled before a higher one."""
    model, kv = _setup("cpu")
    eng = LLMEngine(model, kv, max_prefill_tokens=128, use_graph=False)
    ce = ContinuousEngine(eng, max_slots=16, max_new_cap=24, max_prompt=256, steps_per_sync=4)
    assert ce.widths == [1, 2, 4, 8, 16]
    p = [1] + list(range(30, 90))
    r = ce.submit(p, 9)
    ce.run()
    assert ce.stats["width_steps"] == ce.stats["steps"]          # width 1 throughout
    assert r.tokens == eng.generate([p], 9, ignore_eos=True).tokens[0]
    a, b, c = ce.submit(p, 20), ce.submit([1, 7, 7, 3] * 9, 2), ce.submit([1] + list(range(5, 25)), 20)
    ce.step()                                      # b (2 tokens) finishes in this burst: slot 1 free
    assert (a.slot, c.slot) == (0, 2) and b.finished_s is not None and ce._width() == 4
    d = ce.submit([1, 9] * 12, 20)
    ce.step()
    assert d.slot == 1
    ce.run()
    ce.close()


@pytest.mark.parametrize("lpt", [True, False])
def test_admission_places_longest_prompt_in_lowest_slot(lpt):
    """One admission of several prompts: with the engine's longest-first setting the longest prompt
    takes the lowest free slot (the decode attention grid walks slots in order); either way every
    request's tokens equal its own generate()."""
    model, kv = _setup("cpu")
    eng = LLMEngine(model, kv, max_prefill_tokens=512, use_graph=False)
    eng.lpt = lpt
    reqs = [([1] + list(range(5, 5 + n)), 6) for n in (20, 90, 7, 140, 55)]
    ce = ContinuousEngine(eng, max_slots=8, max_new_cap=8, max_prompt=256, steps_per_sync=2, min_admit=5)
    hs = [ce.submit(p, m) for p, m in reqs]
    ce.step()                                            # one admission of all five
    assert all(h.slot is not None for h in hs)          # 6 tokens: none finished in a 2-step burst
    by_len = sorted(range(len(reqs)), key=lambda i: -len(reqs[i][0]))
    want = by_len if lpt else list(range(len(reqs)))
    assert [hs[i].slot for i in want] == list(range(len(reqs)))
    ce.run()
    ce.close()
    assert [h.tokens for h in hs] == [eng.generate([p], m, ignore_eos=True).tokens[0] for p, m in reqs]
