"""Ingestion service layer (reference ingestion/tests/test_service.py, test_scheduler.py,
test_cascade_delete.py, test_upload_api.py): source CRUD rules, SHA-256 dedupe across service
instances sharing a store, published event format, failure events, per-source isolation in
ingest-all, the scheduler lifecycle, manual trigger re-ingestion, cascade delete, uploads and
their filename rules, and the ingestion health payload."""
from __future__ import annotations

import os
import shutil
import time

import pytest

from copilot_for_consensus_amd.archive import InMemoryArchiveStore, LocalVolumeArchiveStore, SourceConfig
from copilot_for_consensus_amd.bus import NoopPublisher, ValidatingEventPublisher
from copilot_for_consensus_amd.contracts.ids import archive_id_from_bytes
from copilot_for_consensus_amd.services.ingestion import (MAX_UPLOAD_SIZE, IngestionScheduler, IngestionService,
                                                          sanitize_filename)
from copilot_for_consensus_amd.storage.document_store import DocumentNotFoundError, InMemoryDocumentStore

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "sample.mbox")


@pytest.fixture
def env(tmp_path):
    store = InMemoryDocumentStore()
    store.connect()
    pub = ValidatingEventPublisher(NoopPublisher())     # every published event is schema-checked
    svc = IngestionService(pub, store, InMemoryArchiveStore(), storage_path=str(tmp_path / "ing"), max_retries=0)
    src_dir = tmp_path / "src"
    src_dir.mkdir()
    shutil.copy(FIX, src_dir / "list.mbox")
    return svc, pub, store, src_dir


def _src(name, d, **kw):
    return {"name": name, "source_type": "local", "url": str(d), **kw}


# ------------------------------------------------------------------ sources
def test_create_list_get_sources(env):
    svc, _, _, d = env
    assert svc.list_sources() == []
    doc = svc.create_source(_src("b", d))
    svc.create_source(_src("a", d, enabled=False))
    assert doc["enabled"] is True and doc["files_processed"] == 0 and doc["created_at"]
    assert [s["name"] for s in svc.list_sources()] == ["a", "b"]            # sorted by name
    assert [s["name"] for s in svc.list_sources(enabled_only=True)] == ["b"]
    assert svc.get_source("b")["url"] == str(d)
    assert svc.get_source("missing") is None


@pytest.mark.parametrize("bad", [
    {"source_type": "local", "url": "/x"},                       # no name
    {"name": "n", "source_type": "local"},                       # no url
    {"name": "n", "source_type": "gopher", "url": "/x"},         # unknown type
    {"name": "../escape", "source_type": "local", "url": "/x"},  # path components in the name
    {"name": "a/b", "source_type": "local", "url": "/x"},
    {"name": "..", "source_type": "local", "url": "/x"},
])
def test_create_source_validation(env, bad):
    svc = env[0]
    with pytest.raises((ValueError, TypeError)):
        svc.create_source(bad)
    assert svc.list_sources() == []


def test_source_type_is_case_insensitive():
    assert SourceConfig.from_mapping({"name": "n", "source_type": "HTTP", "url": "http://x"}).source_type == "http"


def test_create_duplicate_source_rejected(env):
    svc, _, _, d = env
    svc.create_source(_src("wg", d))
    with pytest.raises(ValueError):
        svc.create_source(_src("wg", d))


def test_update_source(env):
    svc, _, _, d = env
    svc.create_source(_src("wg", d))
    before = svc.get_source("wg")
    time.sleep(0.002)
    after = svc.update_source("wg", {"enabled": False, "schedule": "daily"})
    assert after["enabled"] is False and after["schedule"] == "daily"
    assert after["created_at"] == before["created_at"] and after["updated_at"] >= before["updated_at"]
    with pytest.raises(ValueError):
        svc.update_source("wg", {"source_type": "gopher"})          # still validated as a whole
    with pytest.raises(DocumentNotFoundError):
        svc.update_source("ghost", {"enabled": True})


# ------------------------------------------------------------------ ingestion
def test_ingest_archive_records_and_publishes(env):
    svc, pub, store, d = env
    svc.create_source(_src("wg", d))
    ids = svc.ingest_archive(svc.get_source("wg"))
    data = open(FIX, "rb").read()
    assert ids == [archive_id_from_bytes(data)]
    rec = store.get_document("archives", ids[0])
    assert rec["status"] == "pending" and rec["source"] == "wg" and rec["file_size_bytes"] == len(data)
    assert len(rec["file_hash"]) == 64
    ev = pub.get_events("ArchiveIngested")[0]
    assert set(ev) == {"event_type", "event_id", "timestamp", "version", "data"}
    assert ev["data"]["archive_id"] == ids[0] and ev["data"]["file_hash_sha256"] == rec["file_hash"]
    assert ev["data"]["source_type"] == "local" and ev["data"]["file_size_bytes"] == len(data)
    assert ev["data"]["ingestion_started_at"] <= ev["data"]["ingestion_completed_at"]
    st = svc.get_source("wg")
    assert st["last_run_status"] == "success" and st["files_processed"] == 1 and st["last_error"] is None
    assert svc.stats["files_ingested"] == 1


def test_dedupe_within_and_across_service_instances(env, tmp_path):
    svc, pub, store, d = env
    svc.create_source(_src("wg", d))
    assert len(svc.ingest_archive(svc.get_source("wg"))) == 1
    assert svc.ingest_archive(svc.get_source("wg")) == []          # same bytes: skipped
    assert svc.stats["files_skipped"] == 1
    # a second service instance on the same document store sees the hash too
    pub2 = NoopPublisher()
    svc2 = IngestionService(pub2, store, InMemoryArchiveStore(), storage_path=str(tmp_path / "ing2"), max_retries=0)
    assert svc2.ingest_archive(svc.get_source("wg")) == []
    assert pub2.get_events("ArchiveIngested") == []
    assert len(pub.get_events("ArchiveIngested")) == 1


def test_identical_file_in_two_sources_ingested_once(env, tmp_path):
    svc, pub, _, d = env
    d2 = tmp_path / "src2"
    d2.mkdir()
    shutil.copy(FIX, d2 / "copy.mbox")
    svc.create_source(_src("a", d))
    svc.create_source(_src("b", d2))
    out = svc.ingest_all_enabled_sources()
    assert sorted(len(v) for v in out.values()) == [0, 1]
    assert len(pub.get_events("ArchiveIngested")) == 1


def test_fetch_failure_publishes_failure_event(env, tmp_path):
    svc, pub, _, _ = env
    svc.create_source(_src("gone", tmp_path / "does-not-exist"))
    assert svc.ingest_archive(svc.get_source("gone"), max_retries=1) == []
    ev = pub.get_events("ArchiveIngestionFailed")[0]["data"]
    assert ev["source_name"] == "gone" and ev["retry_count"] == 1 and ev["error_message"]
    st = svc.get_source("gone")
    assert st["last_run_status"] == "failure" and st["last_error"]
    assert svc.stats["files_failed"] == 1


def test_ingest_all_isolates_a_failing_source(env):
    svc, pub, store, d = env
    svc.create_source(_src("good", d))
    # a stored record that no longer validates (edited behind the API)
    store.insert_document("sources", {"_id": "broken", "name": "broken", "source_type": "gopher", "url": "x",
                                      "enabled": True})
    out = svc.ingest_all_enabled_sources()
    assert isinstance(out["broken"], ValueError)
    assert len(out["good"]) == 1 and len(pub.get_events("ArchiveIngested")) == 1


def test_disabled_sources_skipped_by_ingest_all(env):
    svc, pub, _, d = env
    svc.create_source(_src("off", d, enabled=False))
    assert svc.ingest_all_enabled_sources() == {}
    assert pub.get_events() == []


def test_publisher_failure_propagates(env):
    svc, _, _, d = env

    class Down(NoopPublisher):
        def publish(self, *a, **k):
            raise ConnectionError("broker down")

    svc.publisher = Down()
    svc.create_source(_src("wg", d))
    with pytest.raises(ConnectionError):
        svc.ingest_archive(svc.get_source("wg"))
    # the archive record stays 'pending' for the start-up requeue to republish
    assert svc.store.query_documents("archives", {"status": "pending"})


def test_trigger_reingests_disabled_and_missing(env):
    svc, pub, _, d = env
    svc.create_source(_src("wg", d))
    ok, msg, ids = svc.trigger_ingestion("wg")
    assert ok and len(ids) == 1
    ok, msg, ids2 = svc.trigger_ingestion("wg")          # manual trigger bypasses the dedupe
    assert ok and ids2 == ids and "1 previous" in msg
    assert len(pub.get_events("ArchiveIngested")) == 2
    svc.update_source("wg", {"enabled": False})
    ok, msg, _ = svc.trigger_ingestion("wg")
    assert not ok and "disabled" in msg
    ok, msg, _ = svc.trigger_ingestion("ghost")
    assert not ok and "not found" in msg


def test_cascade_delete(env):
    svc, pub, store, d = env
    svc.create_source(_src("wg", d))
    ids = svc.ingest_archive(svc.get_source("wg"))
    out = svc.delete_source_cascade("wg")
    assert out["archives_deleted"] == 1 and out["correlation_id"]
    ev = pub.get_events("SourceDeletionRequested")[0]["data"]
    assert ev["source_name"] == "wg" and ev["archive_ids"] == ids and ev["correlation_id"] == out["correlation_id"]
    assert store.count_documents("archives") == 0 and not svc.archives.archive_exists(ids[0])
    assert svc.get_source("wg") is None
    with pytest.raises(DocumentNotFoundError):
        svc.delete_source_cascade("wg")


def test_delete_without_cascade_keeps_archives(env):
    svc, pub, store, d = env
    svc.create_source(_src("wg", d))
    ids = svc.ingest_archive(svc.get_source("wg"))
    out = svc.delete_source_cascade("wg", cascade=False)
    assert out["archives_deleted"] == 0
    assert pub.get_events("SourceDeletionRequested") == []
    assert store.get_document("archives", ids[0]) is not None and svc.archives.archive_exists(ids[0])


def test_local_volume_store_keeps_source_directories(env, tmp_path):
    svc, _, _, d = env
    svc.archives = LocalVolumeArchiveStore(archive_base_path=str(tmp_path / "archives"))
    svc.create_source(_src("wg", d))
    aid = svc.ingest_archive(svc.get_source("wg"))[0]
    assert (tmp_path / "archives" / "wg" / f"{aid}.mbox").read_bytes() == open(FIX, "rb").read()


# ------------------------------------------------------------------ scheduler
def test_scheduler_lifecycle(env):
    svc, pub, _, d = env
    svc.create_source(_src("wg", d))
    sch = IngestionScheduler(svc, interval_seconds=3600)
    assert not sch.is_running and sch.stop() is False          # stop when not running: no-op
    assert sch.start() is True
    assert sch.start() is False                                # already running: not started twice
    deadline = time.time() + 5
    while sch.runs < 1 and time.time() < deadline:
        time.sleep(0.01)
    assert sch.runs == 1 and len(pub.get_events("ArchiveIngested")) == 1   # first run is immediate
    assert sch.stop() is True and not sch.is_running
    assert not sch._thread.is_alive()


def test_scheduler_survives_errors_and_repeats(env):
    svc = env[0]
    calls = []

    def boom():
        calls.append(1)
        raise RuntimeError("store down")

    svc.ingest_all_enabled_sources = boom
    sch = IngestionScheduler(svc, interval_seconds=0.01)
    sch.start()
    deadline = time.time() + 5
    while len(calls) < 3 and time.time() < deadline:
        time.sleep(0.01)
    sch.stop()
    assert len(calls) >= 3                                     # an error does not end the loop


# ------------------------------------------------------------------ uploads
def test_upload_rules(env):
    svc = env[0]
    data = open(FIX, "rb").read()
    r = svc.upload("list.mbox", data)
    assert r["filename"] == "list.mbox" and r["size_bytes"] == len(data) and r["suggested_source_type"] == "local"
    assert r["archive_id"] == archive_id_from_bytes(data) and len(r["sha256"]) == 64
    assert svc.upload("list.mbox", data)["filename"] == "list_1.mbox"          # never overwritten
    assert svc.upload("b.tar.gz", b"x")["filename"] == "b.tar.gz"
    assert svc.upload("b.tar.gz", b"y")["filename"] == "b_1.tar.gz"            # compound extension kept
    with pytest.raises(ValueError):
        svc.upload("evil.exe", b"MZ")
    with pytest.raises(ValueError):
        svc.upload("empty.mbox", b"")
    with pytest.raises(OverflowError):
        svc.upload("big.mbox", b"\0" * (MAX_UPLOAD_SIZE + 1))


@pytest.mark.parametrize("raw,want", [
    ("../../etc/passwd.mbox", "passwd.mbox"),
    ("C:\\\\Users\\\\x\\\\list.mbox", "list.mbox"),
    ("my list (v2).mbox", "my_list__v2_.mbox"),
    (".hidden.mbox", "hidden.mbox"),
    ("", "upload.mbox"),
])
def test_sanitize_filename(raw, want):
    assert sanitize_filename(raw) == want


# ------------------------------------------------------------------ health
def test_health_reports_scheduler_and_sources(env):
    from fastapi.testclient import TestClient

    from copilot_for_consensus_amd.services.base import create_app
    svc, _, _, d = env
    svc.create_source(_src("a", d))
    svc.create_source(_src("b", d, enabled=False))
    c = TestClient(create_app(svc))
    h = c.get("/health").json()
    assert h["scheduler_running"] is False and h["sources_configured"] == 2 and h["sources_enabled"] == 1
    svc.scheduler = IngestionScheduler(svc, interval_seconds=3600)
    svc.scheduler.start()
    try:
        assert c.get("/health").json()["scheduler_running"] is True
    finally:
        svc.scheduler.stop()


from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


@settings(max_examples=300, deadline=None)
@given(st.text(max_size=400))
def test_sanitize_filename_properties(raw):
    """Upload names (reference fuzzing/corpus/filenames): whatever arrives, the stored name has no
    path component, no leading dot, only [A-Za-z0-9._-], at most 255 characters, never empty."""
    import re
    name = sanitize_filename(raw)
    assert name and len(name) <= 255
    assert "/" not in name and "\\\\" not in name and not name.startswith(".")
    assert re.fullmatch(r"[A-Za-z0-9._-]+", name)


@settings(max_examples=200, deadline=None)
@given(st.text(max_size=60))
def test_source_names_never_escape_the_archive_directory(name):
    try:
        cfg = SourceConfig.from_mapping({"name": name, "source_type": "local", "url": "/x"})
    except (ValueError, TypeError):
        return
    assert "/" not in cfg.name and "\\\\" not in cfg.name and cfg.name.strip() not in (".", "..")
