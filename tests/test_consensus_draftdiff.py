"""Consensus detectors and draft-diff providers (reference adapters copilot_consensus /
copilot_draft_diff test behaviour: ladder outcomes, mock driver parsing, predefined mock diffs)."""
from datetime import datetime, timedelta, timezone

import pytest

from copilot_for_consensus_amd.consensus import (ConsensusLevel, ConsensusSignal, HeuristicConsensusDetector,
                                                 Message, MLConsensusDetector, MockConsensusDetector, Thread,
                                                 create_consensus_detector)
from copilot_for_consensus_amd.draft_diff import (DatatrackerDiffProvider, DraftDiff, LocalDiffProvider,
                                                  MockDiffProvider, create_draft_diff_provider)

NOW = datetime.now(timezone.utc)


def _t(*bodies, authors=None, age_days=0):
    authors = authors or [f"u{i}@x" for i in range(len(bodies))]
    ts = NOW - timedelta(days=age_days)
    return Thread("t1", "subj", [Message(str(i), a, "subj", b, ts) for i, (a, b) in enumerate(zip(authors, bodies))])


def test_signal_confidence_range():
    with pytest.raises(ValueError):
        ConsensusSignal(ConsensusLevel.CONSENSUS, 1.5)


def test_heuristic_ladder():
    d = HeuristicConsensusDetector(agreement_threshold=3, min_participants=2, stagnation_days=7)
    assert d.detect(_t("proposal", "+1", "LGTM", "I agree")).level == ConsensusLevel.CONSENSUS
    strong = d.detect(_t("p", "+1 LGTM", "I agree, makes sense", "sounds good, I approve", "concur"))
    assert strong.level == ConsensusLevel.STRONG_CONSENSUS and strong.confidence <= 0.95
    diss = d.detect(_t("p", "+1", "I disagree"))
    assert diss.level == ConsensusLevel.DISSENT and diss.confidence == pytest.approx(0.6)
    assert d.detect(_t("p", "ok", "fine")).level == ConsensusLevel.WEAK_CONSENSUS
    assert d.detect(_t("p")).level == ConsensusLevel.NO_CONSENSUS
    assert d.detect(_t("p", "+1", age_days=30)).level == ConsensusLevel.STAGNATION
    # consensus needs enough distinct participants
    assert d.detect(_t("+1", "LGTM", "I agree", authors=["a", "a", "a"])).level == ConsensusLevel.WEAK_CONSENSUS


def test_pattern_count_is_patterns_per_message():
    d = HeuristicConsensusDetector()
    a, _ = d.count_patterns(_t("+1 +1 +1"))
    assert a == 1
    a, _ = d.count_patterns(_t("I agree with this"))   # "I agree" and "agree with" both match
    assert a == 2


def test_mock_and_factory():
    m = MockConsensusDetector("Strong-Consensus", 0.9)
    s = m.detect(_t("x"))
    assert s.level == ConsensusLevel.STRONG_CONSENSUS and s.metadata["thread_id"] == "t1"
    with pytest.raises(ValueError):
        MockConsensusDetector("bogus")
    assert isinstance(create_consensus_detector("heuristic"), HeuristicConsensusDetector)
    assert isinstance(create_consensus_detector("mock"), MockConsensusDetector)
    with pytest.raises(ValueError):
        create_consensus_detector("nope")


def test_ml_detector_with_prototype_embeddings():
    from copilot_for_consensus_amd.embedding import MockEmbeddingProvider

    # hash embeddings: identical text -> identical vector, so a message equal to a prototype scores 1.0
    det = MLConsensusDetector(embedding_provider=MockEmbeddingProvider(dimension=64), agree_threshold=0.99,
                              dissent_threshold=0.99)
    t = _t("Proposal text", "I agree with this proposal.", "LGTM, ship it.", "+1, looks good to me.")
    assert det.detect(t).level == ConsensusLevel.CONSENSUS
    t2 = _t("Proposal text", "I disagree with this change.")
    assert det.detect_batch([t, t2])[1].level == ConsensusLevel.DISSENT


def test_thread_from_documents():
    t = Thread.from_documents({"_id": "abc", "subject": "s"},
                              [{"_id": "m1", "from": {"email": "a@x"}, "body_normalized": "+1",
                                "date": "2025-01-01T00:00:00Z"}])
    assert t.thread_id == "abc" and t.messages[0].author == "a@x" and t.participant_count == 1


def test_mock_diff_provider():
    p = MockDiffProvider(default_format="markdown")
    d = p.getdiff("draft-ietf-foo", "01", "02")
    assert d.source == "mock" and "```diff" in d.content and d.url == "mock://draft-ietf-foo/01..02"
    pre = DraftDiff("draft-x", "00", "01", "text", "custom", "mock")
    p.add_mock_diff("draft-x", "00", "01", pre)
    assert p.getdiff("draft-x", "00", "01") is pre
    with pytest.raises(ValueError):
        p.getdiff("", "01", "02")


def test_datatracker_provider_with_injected_fetch():
    texts = {"00": "Intro\nold line\nEnd\n", "01": "Intro\nnew line\nEnd\nAppendix\n"}
    seen = []

    def fetch(url):
        seen.append(url)
        return texts[url[-6:-4]]

    p = DatatrackerDiffProvider("https://dt.example", "text", fetch=fetch)
    d = p.getdiff("draft-ietf-quic-transport", "00", "01")
    assert "-old line" in d.content and "+new line" in d.content and "+Appendix" in d.content
    assert d.metadata["lines_added"] == 2 and d.metadata["lines_removed"] == 1
    assert seen[0] == "https://dt.example/archive/id/draft-ietf-quic-transport-00.txt"
    p.getdiff("draft-ietf-quic-transport", "00", "01")
    assert len(seen) == 2          # cached
    html = DatatrackerDiffProvider(diff_format="html", fetch=fetch).getdiff("draft-ietf-quic-transport", "00", "01")
    assert "<table" in html.content
    with pytest.raises(ValueError):
        p.getdiff("not a draft", "00", "01")


def test_local_diff_provider(tmp_path):
    (tmp_path / "draft-a-b-00.txt").write_text("x\n")
    (tmp_path / "draft-a-b-01.txt").write_text("y\n")
    d = create_draft_diff_provider("local", root=str(tmp_path)).getdiff("draft-a-b", "00", "01")
    assert d.source == "local" and "-x" in d.content and "+y" in d.content


def test_register_custom_draft_diff_provider():
    from copilot_for_consensus_amd.draft_diff import (DraftDiff, DraftDiffProvider, create_draft_diff_provider,
                                                      register_draft_diff_provider)

    class Echo(DraftDiffProvider):
        def __init__(self, prefix="x"):
            self.prefix = prefix

        def getdiff(self, draft_name, version_a, version_b):
            return DraftDiff(draft_name, version_a, version_b, "text", f"{self.prefix}:{draft_name}", "echo")

    register_draft_diff_provider("Echo", Echo)
    p = create_draft_diff_provider("echo", prefix="p")
    assert isinstance(p, Echo) and p.getdiff("draft-a", "00", "01").content == "p:draft-a"
    with pytest.raises(TypeError):
        register_draft_diff_provider("bad", dict)
    with pytest.raises(ValueError):
        register_draft_diff_provider(" ", Echo)


def test_literal_prefilter_counts_exactly_what_the_regexes_match():
    """The ASCII literal prefilter in front of the pattern regexes never changes a count (mixed case,
    word boundaries, +1 / -1, non-ASCII text falling back to the regexes)."""
    import random
    import re

    from copilot_for_consensus_amd.consensus import AGREEMENT_PATTERNS, DISSENT_PATTERNS
    words = ["+1", "-1", "LGTM", "lgtm!", "I Agree", "agreed", "disagree", "Oppose", "concerned", "wait",
             "waiting", "hold on", "not sure", "sounds GOOD", "makes sense", "approve", "Concur", "x+1y",
             "issue with", "problem with", "support this", "İ agree", "naïve", "", "\n", "---1"]
    rng = random.Random(5)
    naive = [re.compile(p, re.IGNORECASE) for p in AGREEMENT_PATTERNS + DISSENT_PATTERNS]
    fast = HeuristicConsensusDetector._AGREE + HeuristicConsensusDetector._DISSENT
    for _ in range(400):
        text = " ".join(rng.choice(words) for _ in range(rng.randint(0, 12)))
        want = sum(1 for rx in naive if rx.search(text))
        assert HeuristicConsensusDetector._count(fast, text) == want, text
