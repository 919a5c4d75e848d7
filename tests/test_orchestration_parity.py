"""Context selection, prompt substitution and citations against the reference's rules
(orchestrator/app/context_selectors.py:20-181: score desc / id asc, stop at top_k or at the first
chunk that would overflow the 1.3 x words budget, rank = position among the selected;
summarization/app/service.py:450-545 placeholders and fallbacks, :702-740 citations)."""
from __future__ import annotations

import pytest

from copilot_for_consensus_amd.contracts import ids as cids
from copilot_for_consensus_amd.orchestration import (TopKCohesiveSelector, TopKRelevanceSelector, build_context,
                                                     create_context_selector, estimate_tokens, format_citations,
                                                     prompt_template, substitute_prompt)


def _c(i, score, words=10, **kw):
    return {"_id": i, "similarity_score": score, "text": " ".join(["w"] * words), "message_id": f"<{i}@x>",
            "message_doc_id": f"m{i}", "thread_id": "t", **kw}


def test_topk_order_ties_and_metadata():
    cands = [_c("b", 0.9), _c("a", 0.9), _c("c", 0.95), _c("d", 0.1, offset=7)]
    sel = TopKRelevanceSelector().select("t", cands, top_k=3)
    assert [s.chunk_id for s in sel.selected_chunks] == ["c", "a", "b"]        # ties broken by id asc
    assert [s.rank for s in sel.selected_chunks] == [0, 1, 2]
    assert sel.metadata() == {"selector_type": "top_k_relevance", "selector_version": "1.0.0",
                              "selection_params": {"top_k": 3, "context_window_tokens": None},
                              "total_candidates": 4, "total_tokens": 0}
    d = TopKRelevanceSelector().select("t", cands, top_k=10).selected_chunks[-1].to_dict()
    assert d == {"chunk_id": "d", "source": "thread_chunks", "score": 0.1, "rank": 3,
                 "metadata": {"message_id": "<d@x>", "message_doc_id": "md", "offset": 7, "thread_id": "t"}}


def test_token_budget_stops_at_first_overflow():
    # 10 words -> 13 tokens each; a budget of 30 admits two; the third stops selection even though a
    # later, shorter chunk would fit (the reference breaks, it does not skip)
    cands = [_c("a", 0.9), _c("b", 0.8), _c("c", 0.7), _c("d", 0.6, words=1)]
    sel = TopKRelevanceSelector().select("t", cands, top_k=10, context_window_tokens=30)
    assert [s.chunk_id for s in sel.selected_chunks] == ["a", "b"] and sel.total_tokens == 26
    assert estimate_tokens("one two three") == 3
    assert TopKRelevanceSelector().select("t", [], 5).selected_chunks == []
    assert len(TopKRelevanceSelector().select("t", cands[:2], 5).selected_chunks) == 2      # fewer than k
    no_id = [{"similarity_score": 1.0, "text": "x"}, _c("z", 0.5)]
    sel = TopKRelevanceSelector().select("t", no_id, 5)
    assert [s.chunk_id for s in sel.selected_chunks] == ["z"] and sel.selected_chunks[0].rank == 0


def test_cohesive_and_factory():
    cands = [_c("a", 0.9, date="2025-01-03", chunk_index=0), _c("b", 0.8, date="2025-01-01", chunk_index=1),
             _c("c", 0.7, date="2025-01-01", chunk_index=0)]
    sel = create_context_selector("top_k_cohesive").select("t", cands, top_k=3)
    assert isinstance(create_context_selector("top_k_cohesive"), TopKCohesiveSelector)
    assert [s.chunk_id for s in sel.selected_chunks] == ["c", "b", "a"] and sel.selector_type == "top_k_cohesive"
    assert [s.rank for s in sel.selected_chunks] == [0, 1, 2]
    with pytest.raises(ValueError):
        create_context_selector("nope")


def test_prompt_substitution_fallbacks_and_errors():
    tpl = prompt_template()
    empty = substitute_prompt(tpl, "tid", {"messages": [], "chunks": []})
    for s in ("Thread: tid", "Messages in context: 0", "Period covered: Unknown", "Multiple participants",
              "No specific drafts mentioned", "(No messages available)"):
        assert s in empty
    chunks = [{"text": "hello", "from": {"name": "Ann", "email": "ann@x"}, "date": "2025-01-02",
               "draft_mentions": ["draft-ietf-quic-00"]},
              {"text": "world", "from": "bob@x", "date": "2025-01-01", "draft_mentions": "RFC 9000"},   # not a list
              {"text": "!", "from": None},                                                            # no sender
              {"text": "?", "from": {"email": "cy@x"}}]
    out = substitute_prompt("{thread_id}|{message_count}|{date_range}|{participants}|{draft_mentions}|"
                            "{email_chunks}", "t9", build_context(chunks))
    tid, n, dr, parts, drafts, body = out.split("|")
    assert (tid, n, dr) == ("t9", "4", "2025-01-01 to 2025-01-02")
    assert parts == "Ann <ann@x>, bob@x, cy@x <cy@x>"
    assert drafts == "draft-ietf-quic-00"
    assert body.startswith("Message 1:\nhello\n\nMessage 2:\nworld")
    with pytest.raises(ValueError, match="unexpected placeholders"):
        substitute_prompt("{thread_id} {secret}", "t", {"messages": [], "chunks": []})


def test_citations_and_ids():
    chunks = [{"_id": f"c{i}", "message_id": f"<{i}@x>", "text": "x" * 5000, "offset": i} for i in range(20)]
    cites = format_citations(chunks, limit=12)
    assert len(cites) == 12 and cites[3] == {"message_id": "<3@x>", "chunk_id": "c3", "offset": 3, "text": "x" * 5000}
    assert format_citations([{"text": "no id"}, {"_id": "k"}]) == [{"message_id": "unknown", "chunk_id": "k",
                                                                   "offset": 0, "text": ""}]
    sid = cids.summary_id("t", ["b", "a"])
    assert sid == cids.summary_id("t", ["a", "b"]) and len(sid) == 64                 # order-insensitive
    assert cids.summary_id("t", []) != cids.summary_id("u", [])
    assert cids.report_id(sid) == cids.sha256_16(sid)
