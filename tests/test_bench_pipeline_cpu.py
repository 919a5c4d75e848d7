"""The benchmark's step loop (incl. the overlapped prepare of the next batch) on CPU, tiny models."""
from copilot_for_consensus_amd.pipeline.bench_pipeline import BenchPipeline


def test_run_steps_overlap_matches_sequential():
    outs = []
    for overlap in (False, True):
        p = BenchPipeline(model="tiny", encoder="tiny", device="cpu", threads_per_step=2, max_new_tokens=3,
                          prefill_tokens=4096, seed=5, index_prefill=0)
        p.prepare_sources([0, 1, 2])
        res = p.run_steps([0, 1, 2], overlap=overlap)
        assert [r.threads for r in res] == [2, 2, 2]
        assert all(r.generated_tokens == 6 for r in res)
        outs.append([r.prompt_tokens for r in res])
    assert outs[0] == outs[1]
