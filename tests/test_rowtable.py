"""The HBM index's host row table (vectorstore/rowtable.py): ids and metadata as numpy columns and
byte heaps -- upsert, lookup, delete, regroup permutation, hash collisions, .npy persistence, and
a 1M-row bulk build without a Python object per row."""
import time

import numpy as np
import pytest

from copilot_for_consensus_amd.vectorstore import HipFlatIndex, HipIVFIndex
from copilot_for_consensus_amd.vectorstore import rowtable as RT


def test_upsert_find_delete_permute_roundtrip(tmp_path):
    t = RT.RowTable(4)
    rows = t.upsert(["a", "bb", "ccc"], [{"thread_id": "t1"}, None, {"k": [1, 2]}])
    assert rows.tolist() == [0, 1, 2] and t.n == 3
    assert t.upsert(["bb"], [{"x": 1}]).tolist() == [1] and t.n == 3     # upsert keeps the row
    assert t.meta_at(1) == {"x": 1} and t.meta_at(0) == {"thread_id": "t1"} and t.id_at(2) == "ccc"
    t.kill(0)
    assert t.find("a") == -1 and t.id_at(0) is None
    t.permute(np.array([2, 1]))
    assert t.n == 2 and t.find("ccc") == 0 and t.find("bb") == 1 and t.meta_at(0) == {"k": [1, 2]}
    t.save(tmp_path)
    u = RT.RowTable.load(tmp_path)
    assert u.ids() == ["ccc", "bb"] and u.meta_at(1) == {"x": 1} and u.find("bb") == 1
    # many inserts merge the recent dict into the sorted lookup and stay findable
    ids = [f"id{i}" for i in range(200_000)]
    t.upsert(ids[:10])
    t.append_bulk(ids[10:])
    assert t.find("id123456") == t.n - (200_000 - 123456) and t.find("nope") == -1


def test_hash_collisions_never_return_a_wrong_row(monkeypatch):
    monkeypatch.setattr(RT, "_hash", lambda b: 7)       # every id collides
    t = RT.RowTable()
    t.upsert(["x", "y", "z"])
    t.rebuild()
    t.upsert(["w"])
    assert [t.find(k) for k in ("x", "y", "z", "w", "q")] == [0, 1, 2, 3, -1]
    t.kill(1)
    assert t.find("y") == -1 and t.find("z") == 2


def test_index_keeps_ids_and_metadata_through_ivf_regroup_and_save(tmp_path):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((3000, 32)).astype(np.float32)
    ids = [f"c{i:05d}" for i in range(3000)]
    idx = HipIVFIndex(32, nlist=16, nprobe=16, device="cpu")
    idx.add_bulk(ids[:2000], X[:2000], [{"thread_id": f"t{i // 10}"} for i in range(2000)])
    idx.add_embeddings(ids[2000:], X[2000:], [{"thread_id": f"t{i // 10}"} for i in range(2000, 3000)])
    idx.train(iters=4)
    hit = idx.query(X[1234], top_k=1)[0]
    assert hit.id == "c01234" and hit.metadata == {"thread_id": "t123"}
    idx.delete("c00007")
    assert not idx.has("c00007") and idx.count() == 2999
    idx.save(tmp_path)
    back = HipFlatIndex.load(tmp_path, device="cpu")
    assert back.count() == 2999 and back.get("c02999").metadata == {"thread_id": "t299"}
    assert back.query(X[42], top_k=1)[0].id == "c00042"


def test_bulk_build_of_a_million_ids_is_compact_and_fast():
    n = 1_000_000
    ids = [f"{i:016x}" for i in range(n)]
    t0 = time.perf_counter()
    t = RT.RowTable(n)
    t.append_bulk(ids)
    dt = time.perf_counter() - t0
    col_bytes = sum(a.nbytes for a in t._cols.values()) + t._ids.buf.nbytes
    assert col_bytes < 64 * n            # ~45 B per row (no Python object per row)
    assert t.find(ids[777_777]) == 777_777
    assert dt < 30, dt
    t.permute(np.arange(n - 1, -1, -1))
    assert t.find(ids[0]) == n - 1 and t.id_at(0) == ids[-1]


def test_table_saved_under_one_hash_loads_under_the_other(tmp_path, monkeypatch):
    """xxhash is optional (blake2b fallback): a table saved with either hash finds its ids after a
    load under the other one (the hash column is recomputed)."""
    import copilot_for_consensus_amd.vectorstore.rowtable as RT
    t = RT.RowTable(4)
    t.upsert([f"id{i}" for i in range(50)], [{"i": i} for i in range(50)])
    t.save(tmp_path / "x")
    other = "blake2b_64" if RT.HASH_NAME == "xxh3_64" else "xxh3_64"
    if other == "xxh3_64":
        pytest.importorskip("xxhash")
    monkeypatch.setattr(RT, "HASH_NAME", other)
    if other == "blake2b_64":
        monkeypatch.setattr(RT, "xxhash", None)
    else:
        import xxhash
        monkeypatch.setattr(RT, "xxhash", xxhash)
    u = RT.RowTable.load(tmp_path / "x")
    assert [u.find(f"id{i}") for i in range(50)] == list(range(50))
    assert u.meta_at(7) == {"i": 7}
