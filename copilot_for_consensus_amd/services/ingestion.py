"""Ingestion service: sources CRUD, scheduled / triggered fetch, SHA-256 dedupe, archive store,
ArchiveIngested events, uploads and cascade delete (reference ingestion/app/service.py:165-1733,
api.py:149-325, scheduler.py:72).
"""
from __future__ import annotations

import io
import os
import re
import tarfile
import tempfile
import threading
import time
import uuid
import zipfile
from datetime import datetime, timezone
from pathlib import Path

try:  # route annotations are resolved against module globals (postponed evaluation)
    from fastapi import Request
except ImportError:  # pragma: no cover - services without the HTTP layer
    Request = None

from ..archive import SourceConfig, calculate_file_hash, create_fetcher
from ..contracts.events import utc_now_iso
from ..contracts.ids import archive_id_from_bytes
from ..storage.document_store import DocumentAlreadyExistsError, DocumentNotFoundError
from .base import BaseService

ALLOWED_EXTENSIONS = (".mbox", ".zip", ".tar", ".tar.gz", ".tgz")
MAX_UPLOAD_SIZE = 100 * 1024 * 1024


def sanitize_filename(name: str) -> str:
    name = os.path.basename(name.replace("\\", "/"))
    name = re.sub(r"[^A-Za-z0-9._-]", "_", name).lstrip(".")
    return name[:255] or "upload.mbox"


def allowed_extension(name: str) -> bool:
    return name.lower().endswith(ALLOWED_EXTENSIONS)


class IngestionService(BaseService):
    name = "ingestion"

    def __init__(self, publisher, document_store, archive_store, storage_path: str | None = None,
                 max_retries: int = 3, **kw):
        super().__init__(publisher, None, document_store, **kw)
        self.archives = archive_store
        path = None
        if storage_path:
            try:   # INGESTION_STORAGE_PATH (uploads + fetch scratch); a temp dir if it cannot be created
                Path(storage_path).mkdir(parents=True, exist_ok=True)
                path = Path(storage_path)
            except OSError:
                path = None
        self.storage_path = path or Path(tempfile.mkdtemp(prefix="cfc-ingest-"))
        self.max_retries = max_retries
        self.scheduler: "IngestionScheduler | None" = None   # set by the node when it runs threaded
        self.stats.update(files_ingested=0, files_skipped=0, files_failed=0)

    # ------------------------------------------------------------------ sources
    def list_sources(self, enabled_only: bool = False) -> list[dict]:
        flt = {"enabled": True} if enabled_only else {}
        return self.store.query_documents("sources", flt, limit=10000, sort_by="name", sort_order="asc")

    def get_source(self, name: str) -> dict | None:
        r = self.store.query_documents("sources", {"name": name}, limit=1)
        return r[0] if r else None

    def create_source(self, src: dict) -> dict:
        cfg = SourceConfig.from_mapping(src)  # validates type / name / url
        if self.get_source(cfg.name):
            raise ValueError(f"Source '{cfg.name}' already exists")
        now = utc_now_iso()
        doc = {**src, "_id": cfg.name, "name": cfg.name, "source_type": cfg.source_type, "url": cfg.url,
               "enabled": src.get("enabled", True), "created_at": now, "updated_at": now, "files_processed": 0,
               "files_skipped": 0}
        self.store.insert_document("sources", doc)
        return doc

    def update_source(self, name: str, src: dict) -> dict:
        cur = self.get_source(name)
        if cur is None:
            raise DocumentNotFoundError(name)
        SourceConfig.from_mapping({**cur, **src})
        patch = {**src, "updated_at": utc_now_iso()}
        patch.pop("_id", None)
        self.store.update_document("sources", cur["_id"], patch)
        return self.get_source(name)

    def delete_source_cascade(self, name: str, cascade: bool = True) -> dict:
        cur = self.get_source(name)
        if cur is None:
            raise DocumentNotFoundError(name)
        archives = self.store.query_documents("archives", {"source": name}, limit=1 << 30)
        corr = str(uuid.uuid4())
        if cascade:
            self.publish("SourceDeletionRequested", source_name=name, correlation_id=corr, requested_at=utc_now_iso(),
                         archive_ids=[a["_id"] for a in archives], delete_mode="hard", reason="source deleted")
            for a in archives:
                self.archives.delete_archive(a["_id"])
                self.store.delete_document("archives", a["_id"])
        self.store.delete_document("sources", cur["_id"])
        return {"source_name": name, "correlation_id": corr, "archives_deleted": len(archives) if cascade else 0}

    # ------------------------------------------------------------------ ingestion
    def _record(self, cfg: SourceConfig, content: bytes, file_path: str, started: str) -> str | None:
        sha = __import__("hashlib").sha256(content).hexdigest()
        if self.store.query_documents("archives", {"file_hash": sha}, limit=1):
            self.stats["files_skipped"] += 1
            self.metrics.increment("ingestion_files_skipped_total", tags={"source": cfg.name})
            return None  # dedupe: identical content already ingested
        aid = self.archives.store_archive(cfg.name, file_path, content)
        try:
            self.store.insert_document("archives", {"_id": aid, "file_hash": sha, "file_size_bytes": len(content),
                                                    "source": cfg.name, "source_url": cfg.url, "format": "mbox",
                                                    "ingestion_date": started, "file_path": file_path,
                                                    "status": "pending", "attemptCount": 0})
        except DocumentAlreadyExistsError:
            return None
        self.publish("ArchiveIngested", archive_id=aid, source_name=cfg.name, source_type=cfg.source_type,
                     source_url=cfg.url, file_size_bytes=len(content), file_hash_sha256=sha,
                     ingestion_started_at=started, ingestion_completed_at=utc_now_iso(), file_path=file_path)
        self.stats["files_ingested"] += 1
        self.metrics.increment("ingestion_files_total", tags={"source": cfg.name, "status": "success"})
        return aid

    def record_archive(self, source: SourceConfig, content: bytes, file_path: str) -> str | None:
        """Store one fetched archive and announce it (ArchiveIngested); None when identical content was
        already ingested.  The fetch-free entry point of the batched driver (pipeline/rag.py)."""
        return self._record(source, content, file_path, utc_now_iso())

    def ingest_archive(self, source: dict | SourceConfig, max_retries: int | None = None) -> list[str]:
        cfg = source if isinstance(source, SourceConfig) else SourceConfig.from_mapping(source)
        started = utc_now_iso()
        retries = self.max_retries if max_retries is None else max_retries
        last = None
        for attempt in range(retries + 1):
            out_dir = tempfile.mkdtemp(prefix="fetch-", dir=self.storage_path)
            ok, paths, err = create_fetcher(cfg).fetch(out_dir)
            if ok:
                ids = []
                for p in paths or []:
                    data = Path(p).read_bytes()
                    for name, content in self._expand(p, data):
                        aid = self._record(cfg, content, name, started)
                        if aid:
                            ids.append(aid)
                self._update_source_status(cfg.name, "success", None, len(ids))
                return ids
            last = err
            time.sleep(min(0.05 * (2 ** attempt), 2.0))
        self.stats["files_failed"] += 1
        self.publish("ArchiveIngestionFailed", source_name=cfg.name, source_type=cfg.source_type, source_url=cfg.url,
                     error_message=str(last) or "fetch failed", error_type="FetchError", retry_count=retries,
                     ingestion_started_at=started, failed_at=utc_now_iso())
        self._update_source_status(cfg.name, "failure", str(last), 0)
        return []

    @staticmethod
    def _expand(path: str, data: bytes):
        """Archives inside .zip / .tar(.gz) uploads are ingested member by member."""
        low = path.lower()
        if low.endswith(".zip"):
            with zipfile.ZipFile(io.BytesIO(data)) as z:
                for n in z.namelist():
                    if not n.endswith("/"):
                        yield n, z.read(n)
        elif low.endswith((".tar", ".tar.gz", ".tgz")):
            with tarfile.open(fileobj=io.BytesIO(data)) as t:
                for m in t.getmembers():
                    if m.isfile():
                        yield m.name, t.extractfile(m).read()
        else:
            yield path, data

    def _update_source_status(self, name, status, error, files):
        src = self.get_source(name)
        if src is None:
            return
        self.store.update_document("sources", src["_id"], {
            "last_run_at": utc_now_iso(), "last_run_status": status, "last_error": error,
            "files_processed": int(src.get("files_processed", 0)) + files})

    def trigger_ingestion(self, name: str) -> tuple[bool, str, list[str]]:
        src = self.get_source(name)
        if src is None:
            return False, f"Source '{name}' not found", []
        if not src.get("enabled", True):
            return False, f"Source '{name}' is disabled", []
        # a manual trigger re-ingests everything the source holds: its archive records are dropped
        # first so the checksum dedupe lets the files through again (reference service.py:1733-1772);
        # downstream stages are idempotent on the deterministic ids, so nothing is duplicated
        deleted = self.delete_archives_for_source(name)
        ids = self.ingest_archive(src)
        return True, f"Ingested {len(ids)} archive(s) ({deleted} previous record(s) reset)", ids

    def delete_archives_for_source(self, name: str) -> int:
        """Drop the source's ``archives`` records (not the stored bytes); returns how many."""
        return self.store.delete_many("archives", {"source": name})

    def ingest_all_enabled_sources(self) -> dict[str, list[str] | Exception]:
        """Ingest every enabled source; one source's failure (bad stored config, store error) is
        returned in its slot and does not stop the others (reference service.py:1044)."""
        out: dict[str, list[str] | Exception] = {}
        for s in self.list_sources(enabled_only=True):
            try:
                out[s["name"]] = self.ingest_archive(s)
            except Exception as e:  # noqa: BLE001 - isolated per source, reported
                self.stats["files_failed"] += 1
                self.log.error("source ingestion failed", source=s.get("name"), error=repr(e))
                self.errors.report(e, context={"source": s.get("name")})
                out[s["name"]] = e
        return out

    def upload(self, filename: str, content: bytes) -> dict:
        name = sanitize_filename(filename)
        if not allowed_extension(name):
            raise ValueError(f"Invalid file type. Allowed: {', '.join(ALLOWED_EXTENSIONS)}")
        if len(content) > MAX_UPLOAD_SIZE:
            raise OverflowError("File too large")
        if not content:
            raise ValueError("File is empty")
        d = self.storage_path / "uploads"
        d.mkdir(parents=True, exist_ok=True)
        p = d / name
        if p.exists():   # never overwrite an earlier upload: name_1.mbox, name_2.tar.gz, ...
            low = name.lower()
            ext = next((e for e in (".tar.gz", ".tgz", ".tar", ".zip", ".mbox") if low.endswith(e)), p.suffix)
            stem = name[:len(name) - len(ext)]
            n = 1
            while (d / f"{stem}_{n}{ext}").exists():
                n += 1
            name = f"{stem}_{n}{ext}"
            p = d / name
        p.write_bytes(content)
        return {"filename": name, "server_path": str(p), "size_bytes": len(content),
                "uploaded_at": datetime.now(timezone.utc).isoformat(), "suggested_source_type": "local",
                "sha256": calculate_file_hash(str(p)), "archive_id": archive_id_from_bytes(content)}


class IngestionScheduler:
    """Background loop ingesting every enabled source each ``interval_seconds`` (scheduler.py:72)."""

    def __init__(self, service: IngestionService, interval_seconds: float = 21600):
        self.service, self.interval = service, interval_seconds
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self.runs = 0

    @property
    def is_running(self) -> bool:
        return self._thread is not None and self._thread.is_alive()

    def start(self) -> bool:
        """Start the loop; False (and nothing started) if it is already running."""
        if self.is_running:
            return False
        self._stop.clear()

        def loop():
            while not self._stop.is_set():
                try:
                    self.service.ingest_all_enabled_sources()
                except Exception as e:
                    self.service.log.error("scheduled ingestion failed", error=repr(e))
                self.runs += 1
                self._stop.wait(self.interval)
        self._thread = threading.Thread(target=loop, name="ingestion-scheduler", daemon=True)
        self._thread.start()
        return True

    def stop(self, timeout: float | None = 5.0) -> bool:
        """Stop the loop and wait for it; False if it was not running."""
        if not self.is_running:
            return False
        self._stop.set()
        self._thread.join(timeout)
        return True


def ingestion_routes(app, service: IngestionService, auth=None):
    from fastapi import Depends, HTTPException, Request

    deps = [Depends(auth)] if auth else []

    @app.get("/api/sources", dependencies=deps)
    def list_sources(enabled_only: bool = False):
        s = service.list_sources(enabled_only)
        return {"sources": s, "count": len(s)}

    @app.get("/api/sources/{name}", dependencies=deps)
    def get_source(name: str):
        s = service.get_source(name)
        if s is None:
            raise HTTPException(404, f"Source '{name}' not found")
        return s

    @app.post("/api/sources", status_code=201, dependencies=deps)
    def create_source(body: dict):
        # required fields missing -> 422 like the reference's pydantic request model
        missing = [k for k in ("name", "source_type", "url") if not body.get(k)]
        if missing:
            raise HTTPException(422, [{"loc": ["body", k], "msg": "Field required", "type": "missing"}
                                      for k in missing])
        try:
            return {"source": service.create_source(body)}
        except (ValueError, TypeError) as e:
            raise HTTPException(400, str(e))

    @app.put("/api/sources/{name}", dependencies=deps)
    def update_source(name: str, body: dict):
        if body.get("name", name) != name:
            raise HTTPException(400, "Source name in URL must match name in request body")
        try:
            return {"source": service.update_source(name, body)}
        except DocumentNotFoundError:
            raise HTTPException(404, f"Source '{name}' not found")
        except (ValueError, TypeError) as e:
            raise HTTPException(400, str(e))

    @app.delete("/api/sources/{name}", dependencies=deps)
    def delete_source(name: str, cascade: bool = True):
        try:
            return service.delete_source_cascade(name, cascade)
        except DocumentNotFoundError:
            raise HTTPException(404, f"Source '{name}' not found")

    @app.post("/api/sources/{name}/trigger", dependencies=deps)
    def trigger(name: str):
        ok, msg, ids = service.trigger_ingestion(name)
        if not ok:
            raise HTTPException(400 if "disabled" in msg else 404, msg)
        return {"source_name": name, "status": "completed", "message": msg, "archive_ids": ids,
                "triggered_at": utc_now_iso()}

    @app.get("/api/sources/{name}/status", dependencies=deps)
    def status(name: str):
        s = service.get_source(name)
        if s is None:
            raise HTTPException(404, f"Source '{name}' not found")
        return {k: s.get(k) for k in ("name", "enabled", "last_run_at", "last_run_status", "last_error",
                                      "next_run_at", "files_processed", "files_skipped")}

    @app.post("/api/uploads", status_code=201, dependencies=deps)
    async def upload(request: Request, filename: str | None = None):
        """multipart/form-data (field ``file``) -- parsed with the stdlib (no python-multipart in
        this image) -- or a raw body with ``?filename=``."""
        body = await request.body()
        ctype = request.headers.get("content-type", "")
        name, data = filename, body
        if ctype.startswith("multipart/form-data"):
            name, data = parse_multipart_file(ctype, body)
        if not name:
            raise HTTPException(400, "Filename is required")
        try:
            return service.upload(name, data)
        except OverflowError:
            raise HTTPException(413, "File too large. Maximum size: 100MB")
        except ValueError as e:
            raise HTTPException(400, str(e))


def parse_multipart_file(content_type: str, body: bytes) -> tuple[str | None, bytes]:
    from email.parser import BytesParser
    from email.policy import HTTP
    msg = BytesParser(policy=HTTP).parsebytes(b"Content-Type: " + content_type.encode() + b"\r\n\r\n" + body)
    for part in msg.iter_parts():
        fn = part.get_filename()
        if fn is not None or part.get_param("name", header="content-disposition") == "file":
            return fn, part.get_payload(decode=True) or b""
    return None, b""
