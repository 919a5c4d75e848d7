"""Data maintenance tools (export/import, counts, CSV, backfill, archive verification, queue
drainage) and the static policy gates -- reference scripts/test_convert_ndjson_to_csv.py,
test_backfill_archive_source_type.py, test_check_mutable_defaults.py,
test_check_no_runtime_env_vars.py, tests/test_data_migration_{export,import}.py,
tests/test_queue_drainage.py."""
from __future__ import annotations

import csv
import json
import threading
import time

import pytest

from copilot_for_consensus_amd.bus import InProcBroker, InProcPublisher, InProcSubscriber
from copilot_for_consensus_amd.storage.document_store import InMemoryDocumentStore
from copilot_for_consensus_amd.tools import data_ops, policy


def _store():
    s = InMemoryDocumentStore()
    s.connect()
    s.insert_document("sources", {"_id": "s1", "name": "quic", "source_type": "rsync"})
    for i in range(3):
        s.insert_document("archives", {"_id": f"a{i}", "source": "quic" if i else "legacy", "file_hash": "h",
                                       "status": "completed"})
    s.insert_document("messages", {"_id": "m1", "archive_id": "a1", "meta": {"x": 1}, "to": ["p", "q"]})
    s.insert_document("user_roles", {"_id": "u1", "roles": ["admin"]})
    return s


def test_export_import_roundtrip(tmp_path):
    src = _store()
    counts = data_ops.export_store(src, tmp_path, source_desc="mongodb://<redacted>@x")
    assert counts["archives"] == 3 and counts["user_roles"] == 1 and counts["chunks"] == 0
    man = json.loads((tmp_path / "manifest.json").read_text())
    assert man["counts"] == counts and "auth" in man["databases"]
    lines = (tmp_path / "copilot" / "archives.ndjson").read_text().splitlines()
    assert [json.loads(x)["_id"] for x in lines] == ["a0", "a1", "a2"]

    dst = InMemoryDocumentStore()
    stats = data_ops.import_store(dst, tmp_path, batch_size=2)
    assert stats["archives"]["inserted"] == 3 and stats["user_roles"]["inserted"] == 1
    assert dst.get_document("messages", "m1") == src.get_document("messages", "m1")

    # upsert replaces whole documents; merge patches fields and keeps local-only ones
    dst.update_document("archives", "a0", {"$set": {"status": "failed", "local": 1}})
    st = data_ops.import_store(dst, tmp_path, collections=["archives"], mode="upsert")
    assert st["archives"]["replaced"] == 3
    assert dst.get_document("archives", "a0") == src.get_document("archives", "a0")
    dst.update_document("archives", "a0", {"$set": {"status": "failed", "local": 1}})
    data_ops.import_store(dst, tmp_path, collections=["archives"], mode="merge")
    a0 = dst.get_document("archives", "a0")
    assert a0["status"] == "completed" and a0["local"] == 1
    with pytest.raises(ValueError):
        data_ops.import_store(dst, tmp_path, mode="clobber")


def test_import_reports_bad_json_line(tmp_path):
    (tmp_path / "copilot").mkdir()
    (tmp_path / "copilot" / "sources.ndjson").write_text('{"_id": "a"}\n{oops\n')
    with pytest.raises(ValueError, match="sources.ndjson:2"):
        data_ops.import_store(InMemoryDocumentStore(), tmp_path)


def test_counts_table_and_json():
    rows = data_ops.data_counts(_store(), collections=["archives", "messages"])
    assert rows == [{"name": "archives", "kind": "collection", "count": 3},
                    {"name": "messages", "kind": "collection", "count": 1}]
    table = data_ops.format_table(rows)
    assert table.splitlines()[0].split() == ["name", "kind", "count"] and "archives" in table


def test_ndjson_to_csv(tmp_path):
    src = tmp_path / "m.ndjson"
    src.write_text('{"_id": "1", "meta": {"a": 1, "b": {"c": 2}}, "tags": ["x"]}\n\n{"_id": "2", "extra": true}\n')
    n = data_ops.ndjson_to_csv(src, tmp_path / "m.csv")
    assert n == 2
    rows = list(csv.DictReader(open(tmp_path / "m.csv")))
    assert set(rows[0]) == {"_id", "meta.a", "meta.b.c", "tags", "extra"}
    assert rows[0]["meta.b.c"] == "2" and json.loads(rows[0]["tags"]) == ["x"] and rows[1]["extra"] == "True"
    data_ops.ndjson_to_csv(src, tmp_path / "f.csv", fields=["_id"])
    assert list(csv.reader(open(tmp_path / "f.csv")))[0] == ["_id"]


def test_backfill_source_type():
    s = _store()
    dry = data_ops.backfill_archive_source_type(s, dry_run=True)
    assert dry == {"total_found": 3, "updated": 0, "errors": 0}
    assert data_ops.backfill_archive_source_type(s, limit=1)["updated"] == 1
    res = data_ops.backfill_archive_source_type(s)
    assert res["updated"] == 2
    assert s.get_document("archives", "a0")["source_type"] == "local"   # unknown source -> default
    assert s.get_document("archives", "a1")["source_type"] == "rsync"   # source's own type
    assert data_ops.backfill_archive_source_type(s)["total_found"] == 0


def test_verify_archives():
    s = _store()
    assert data_ops.verify_archives(s)["ok"]
    s.insert_document("messages", {"_id": "m9", "archive_id": "gone"})
    s.insert_document("archives", {"_id": "a9", "status": "pending"})
    res = data_ops.verify_archives(s)
    assert not res["ok"] and res["messages_without_archive"] == 1 and res["missing_required_fields"] == ["a9"]
    assert res["status"] == {"completed": 3, "pending": 1}


def test_queue_drainage_checks():
    ok = data_ops.check_queue_drainage([{"name": "json.parsed", "messages": 0, "consumers": 1},
                                        {"name": "json.parsed.failed", "messages": 4, "consumers": 0}])
    assert ok["ok"], ok
    bad = data_ops.check_queue_drainage([{"name": "a", "messages": 3, "consumers": 1},
                                         {"name": "b", "messages": 0, "consumers": 0},
                                         {"name": "b.v1", "messages": 0, "consumers": 1}])
    assert bad["undrained"] == ["a"] and bad["without_consumers"] == ["b"] and "b" in bad["duplicates"]


def test_inproc_broker_drains_and_counts_consumers():
    broker = InProcBroker()
    sub = InProcSubscriber(broker=broker, queue_name="chunking")
    seen = []
    sub.subscribe("JSONParsed", lambda e: seen.append(e))
    pub = InProcPublisher(broker=broker)
    for _ in range(5):
        pub.publish("copilot.events", "json.parsed", {"event_type": "JSONParsed", "data": {}})
    stats = {q["name"]: q for q in data_ops.broker_queue_stats(broker)}
    assert stats["chunking"]["messages"] == 5 and stats["chunking"]["consumers"] == 0
    t = threading.Thread(target=sub.start_consuming, daemon=True)
    t.start()
    assert data_ops.wait_for_drainage(broker, timeout_s=10)
    deadline = time.monotonic() + 5
    while broker.consumer_counts()["chunking"] != 1 and time.monotonic() < deadline:
        time.sleep(0.01)
    assert broker.consumer_counts()["chunking"] == 1
    sub.stop_consuming()
    t.join(5)
    assert broker.consumer_counts()["chunking"] == 0 and len(seen) == 5


def test_cli_counts_and_export(tmp_path, capsys):
    src = _store()
    data_ops.export_store(src, tmp_path / "snap")
    assert data_ops.main(["--snapshot", str(tmp_path / "snap"), "counts", "--format", "json"]) == 0
    rows = json.loads(capsys.readouterr().out)
    assert {r["name"]: r["count"] for r in rows}["archives"] == 3
    assert data_ops.main(["--snapshot", str(tmp_path / "snap"), "verify-archives"]) == 0


# ------------------------------------------------------------------ policy gates
def test_policy_checks_detect_violations(tmp_path):
    bad = tmp_path / "bad.py"
    bad.write_text("import os\n\ndef f(a=[], *, b={}):\n    return os.environ.get('SECRET_THING'), os.getenv(a)\n"
                   "x = lambda q=set(): q\n")
    found = policy.check_mutable_defaults([bad])
    assert len(found) == 3 and {f.rule for f in found} == {"mutable-default"}
    env = policy.check_runtime_env_vars([bad], root=tmp_path)
    assert [f.detail.split()[0] for f in env] == ["SECRET_THING", "environment"]
    ok = tmp_path / "ok.py"
    ok.write_text('"""doc"""\nimport os\n\ndef g(a=(), b=None):\n    return os.environ.get("CFC_TP"), os.environ["RANK"]\n')
    assert policy.check_mutable_defaults([ok]) == [] and policy.check_runtime_env_vars([ok], root=tmp_path) == []
    assert policy.check_module_docstrings([bad]) and policy.check_module_docstrings([ok]) == []


def test_package_passes_policy_gates():
    found = policy.run_all()
    assert found == [], "\n".join(map(str, found))
