"""Raw-archive storage and source fetchers.

ArchiveStore API = adapters/copilot_archive_store/copilot_archive_store/archive_store.py:59-148
(store_archive / get_archive / get_archive_by_hash / archive_exists / delete_archive /
list_archives), archive id = sha256(content)[:16] (local_volume_archive_store.py:125-126).
Fetchers = adapters/copilot_archive_fetcher (fetch(output_dir) -> (ok, paths, error)) for local,
http, rsync and imap sources.
"""
from __future__ import annotations

import dataclasses
import hashlib
import imaplib
import json
import os
import shutil
import subprocess
import threading
import urllib.request
from abc import ABC, abstractmethod
from datetime import datetime, timezone
from pathlib import Path
from typing import Any, Mapping

from ..contracts.ids import archive_id_from_bytes


class ArchiveStoreError(Exception):
    pass


class ArchiveStore(ABC):
    @abstractmethod
    def store_archive(self, source_name: str, file_path: str, content: bytes) -> str: ...

    @abstractmethod
    def get_archive(self, archive_id: str) -> bytes | None: ...

    @abstractmethod
    def get_archive_by_hash(self, content_hash: str) -> str | None: ...

    @abstractmethod
    def archive_exists(self, archive_id: str) -> bool: ...

    @abstractmethod
    def delete_archive(self, archive_id: str) -> bool: ...

    @abstractmethod
    def list_archives(self, source_name: str) -> list[dict[str, Any]]: ...


class InMemoryArchiveStore(ArchiveStore):
    def __init__(self, **_):
        self._lock = threading.Lock()
        self._data: dict[str, bytes] = {}
        self._meta: dict[str, dict] = {}

    def store_archive(self, source_name, file_path, content):
        aid = archive_id_from_bytes(content)
        with self._lock:
            self._data[aid] = bytes(content)
            self._meta[aid] = {"archive_id": aid, "source_name": source_name, "original_path": file_path,
                               "content_hash": hashlib.sha256(content).hexdigest(), "size_bytes": len(content),
                               "stored_at": datetime.now(timezone.utc).isoformat()}
        return aid

    def get_archive(self, archive_id):
        return self._data.get(archive_id)

    def get_archive_by_hash(self, content_hash):
        for aid, m in self._meta.items():
            if m["content_hash"] == content_hash:
                return aid
        return None

    def archive_exists(self, archive_id):
        return archive_id in self._data

    def delete_archive(self, archive_id):
        with self._lock:
            self._meta.pop(archive_id, None)
            return self._data.pop(archive_id, None) is not None

    def list_archives(self, source_name):
        return [dict(m) for m in self._meta.values() if m["source_name"] == source_name]


class LocalVolumeArchiveStore(ArchiveStore):
    """Files under ``<base>/<source>/<archive_id>.mbox`` + one JSON metadata sidecar per archive
    (``<base>/.meta/<archive_id>.json``, written atomically).  Several processes share the volume
    (the reference mounts one ``raw_archives`` volume into ingestion and parsing): an archive stored
    by one process is visible to the others on their next lookup, with no shared index file to race
    on."""

    def __init__(self, archive_base_path: str = "/data/raw_archives", **_):
        self.base = Path(archive_base_path)
        self.base.mkdir(parents=True, exist_ok=True)
        self._meta_dir = self.base / ".meta"
        self._meta_dir.mkdir(exist_ok=True)
        self._lock = threading.Lock()
        self._meta: dict[str, dict] = {}
        legacy = self.base / "metadata.json"          # single-index layout of earlier versions
        if legacy.exists():
            for aid, m in json.loads(legacy.read_text()).items():
                if not (self._meta_dir / f"{aid}.json").exists():
                    self._write_meta(aid, m)
        self._refresh()

    def _write_meta(self, aid: str, m: dict) -> None:
        tmp = self._meta_dir / f".{aid}.{os.getpid()}.tmp"
        tmp.write_text(json.dumps(m))
        os.replace(tmp, self._meta_dir / f"{aid}.json")
        self._meta[aid] = m

    def _read_meta(self, aid: str) -> dict | None:
        m = self._meta.get(aid)
        if m is None:
            try:
                m = json.loads((self._meta_dir / f"{aid}.json").read_text())
            except (OSError, ValueError):
                return None
            self._meta[aid] = m
        return m

    def _refresh(self) -> None:
        seen = {}
        for f in self._meta_dir.glob("*.json"):
            try:
                seen[f.stem] = json.loads(f.read_text())
            except (OSError, ValueError):
                continue
        self._meta = seen

    def store_archive(self, source_name, file_path, content):
        aid = archive_id_from_bytes(content)
        d = self.base / source_name
        d.mkdir(parents=True, exist_ok=True)
        p = d / f"{aid}.mbox"
        with self._lock:
            if not p.exists():
                tmp = p.with_suffix(f".{os.getpid()}.part")
                tmp.write_bytes(content)
                os.replace(tmp, p)
            self._write_meta(aid, {"archive_id": aid, "source_name": source_name, "file_path": str(p),
                                   "original_path": file_path, "content_hash": hashlib.sha256(content).hexdigest(),
                                   "size_bytes": len(content), "stored_at": datetime.now(timezone.utc).isoformat()})
        return aid

    def get_archive(self, archive_id):
        m = self._read_meta(archive_id)
        if not m:
            return None
        p = Path(m["file_path"])
        return p.read_bytes() if p.exists() else None

    def get_archive_by_hash(self, content_hash):
        self._refresh()
        for aid, m in self._meta.items():
            if m["content_hash"] == content_hash:
                return aid
        return None

    def archive_exists(self, archive_id):
        m = self._read_meta(archive_id)
        return bool(m) and Path(m["file_path"]).exists()

    def delete_archive(self, archive_id):
        with self._lock:
            m = self._read_meta(archive_id)
            self._meta.pop(archive_id, None)
            if not m:
                return False
            Path(m["file_path"]).unlink(missing_ok=True)
            (self._meta_dir / f"{archive_id}.json").unlink(missing_ok=True)
            return True

    def list_archives(self, source_name):
        self._refresh()
        return [dict(m) for m in self._meta.values() if m["source_name"] == source_name]


class DocumentStoreArchiveStore(ArchiveStore):
    """Archives kept in a DocumentStore collection (base64 content) -- the reference's MongoDB
    archive store is a stub (mongodb_archive_store.py:13); this one works on any DocumentStore."""

    def __init__(self, document_store=None, collection: str = "raw_archives", **_):
        from ..storage.document_store import InMemoryDocumentStore
        self.store = document_store or InMemoryDocumentStore()
        self.coll = collection

    def store_archive(self, source_name, file_path, content):
        import base64
        aid = hashlib.sha256(content).hexdigest()[:16]
        if self.store.get_document(self.coll, aid) is None:
            self.store.insert_document(self.coll, {"_id": aid, "archive_id": aid, "source_name": source_name,
                                                   "file_path": file_path, "original_path": file_path,
                                                   "file_hash": hashlib.sha256(content).hexdigest(),
                                                   "content_hash": hashlib.sha256(content).hexdigest(),
                                                   "size_bytes": len(content),
                                                   "stored_at": datetime.now(timezone.utc).isoformat(),
                                                   "content_b64": base64.b64encode(content).decode()})
        return aid

    def get_archive(self, archive_id):
        import base64
        d = self.store.get_document(self.coll, archive_id)
        return None if d is None else base64.b64decode(d["content_b64"])

    def get_archive_by_hash(self, content_hash):
        r = self.store.query_documents(self.coll, {"file_hash": content_hash}, limit=1)
        return r[0]["_id"] if r else None

    def archive_exists(self, archive_id):
        return self.store.get_document(self.coll, archive_id) is not None

    def delete_archive(self, archive_id):
        if self.store.get_document(self.coll, archive_id) is None:
            return False
        self.store.delete_document(self.coll, archive_id)
        return True

    def list_archives(self, source_name):
        return [{**{k: v for k, v in d.items() if k not in ("content_b64", "_id")}, "archive_id": d["_id"]}
                for d in self.store.query_documents(self.coll, {"source_name": source_name}, limit=1 << 30)]


def create_archive_store(cfg=None) -> ArchiveStore:
    name = str(getattr(cfg, "driver_name", cfg) or "local").strip().lower()
    kw = dict(getattr(cfg, "driver_config", {}) or {})
    if name == "local":
        return LocalVolumeArchiveStore(**{k: v for k, v in kw.items() if v is not None})
    if name == "inmemory":
        return InMemoryArchiveStore()
    if name == "azureblob":
        from ..cloud.azure import AzureBlobArchiveStore
        return AzureBlobArchiveStore(**{k: v for k, v in kw.items() if v is not None})
    if name in ("mongodb", "document_store"):
        return DocumentStoreArchiveStore(**kw)
    raise ValueError(f"unknown archive_store driver {name!r}")


# ------------------------------------------------------------------------------------ fetchers

SOURCE_TYPES = ("local", "http", "rsync", "imap")


@dataclasses.dataclass
class SourceConfig:
    name: str
    source_type: str
    url: str
    port: int | None = None
    username: str | None = None
    password: str | None = None
    folder: str | None = None
    enabled: bool = True
    schedule: str | None = None

    def __post_init__(self):
        self.source_type = str(self.source_type).lower()
        if self.source_type not in SOURCE_TYPES:
            raise ValueError(f"source_type must be one of {SOURCE_TYPES}, got {self.source_type!r}")
        if not self.name or not self.url:
            raise ValueError("source name and url are required")
        # the name becomes a directory under the archive store's base path: no path components
        if any(c in str(self.name) for c in "/\\\0") or str(self.name).strip() in (".", ".."):
            raise ValueError(f"invalid source name {self.name!r}: no path separators, '.' or '..'")

    @classmethod
    def from_mapping(cls, m: Mapping[str, Any]) -> "SourceConfig":
        fields = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in m.items() if k in fields})


class ArchiveFetcher(ABC):
    def __init__(self, source: SourceConfig):
        self.source = source

    @abstractmethod
    def fetch(self, output_dir: str) -> tuple[bool, list[str] | None, str | None]:
        """Download the source's archive files into output_dir -> (ok, paths, error)."""


ARCHIVE_SUFFIXES = (".mbox", ".txt", ".mail", ".eml")


class LocalFetcher(ArchiveFetcher):
    def fetch(self, output_dir):
        src = Path(self.source.url.removeprefix("file://"))
        out = Path(output_dir)
        out.mkdir(parents=True, exist_ok=True)
        try:
            if src.is_dir():
                files = [p for p in sorted(src.rglob("*")) if p.is_file()]
            elif src.is_file():
                files = [src]
            else:
                return False, None, f"path not found: {src}"
            paths = []
            for f in files:
                dst = out / f.name
                shutil.copyfile(f, dst)
                paths.append(str(dst))
            return True, paths, None
        except OSError as e:
            return False, None, str(e)


class HTTPFetcher(ArchiveFetcher):
    def __init__(self, source: SourceConfig, timeout: float = 60.0):
        super().__init__(source)
        self.timeout = timeout

    def fetch(self, output_dir):
        out = Path(output_dir)
        out.mkdir(parents=True, exist_ok=True)
        name = self.source.url.rstrip("/").rsplit("/", 1)[-1] or "archive.mbox"
        dst = out / name
        try:
            with urllib.request.urlopen(self.source.url, timeout=self.timeout) as r, open(dst, "wb") as f:
                shutil.copyfileobj(r, f, 1 << 20)
            return True, [str(dst)], None
        except Exception as e:  # network errors are reported, not raised
            return False, None, f"{type(e).__name__}: {e}"


class RsyncFetcher(ArchiveFetcher):
    def fetch(self, output_dir):
        Path(output_dir).mkdir(parents=True, exist_ok=True)
        if shutil.which("rsync") is None:
            return False, None, "rsync binary not available"
        cmd = ["rsync", "-az", "--timeout=300", self.source.url.rstrip("/") + "/", str(output_dir)]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            return False, None, res.stderr.strip()[-2000:]
        return True, [str(p) for p in sorted(Path(output_dir).rglob("*")) if p.is_file()], None


class IMAPFetcher(ArchiveFetcher):
    """Downloads every message of ``folder`` into one mbox file."""

    def fetch(self, output_dir):
        out = Path(output_dir)
        out.mkdir(parents=True, exist_ok=True)
        try:
            cls = imaplib.IMAP4_SSL if (self.source.port or 993) == 993 else imaplib.IMAP4
            with cls(self.source.url, self.source.port or 993) as m:
                if self.source.username:
                    m.login(self.source.username, self.source.password or "")
                m.select(self.source.folder or "INBOX", readonly=True)
                _, data = m.search(None, "ALL")
                dst = out / f"{self.source.name}.mbox"
                with open(dst, "wb") as f:
                    for num in data[0].split():
                        _, msg = m.fetch(num, "(RFC822)")
                        f.write(b"From imap@localhost Thu Jan  1 00:00:00 1970\n")
                        f.write(msg[0][1].replace(b"\nFrom ", b"\n>From "))
                        f.write(b"\n")
            return True, [str(dst)], None
        except Exception as e:
            return False, None, f"{type(e).__name__}: {e}"


def create_fetcher(source: SourceConfig | Mapping) -> ArchiveFetcher:
    if not isinstance(source, SourceConfig):
        source = SourceConfig.from_mapping(source)
    return {"local": LocalFetcher, "http": HTTPFetcher, "rsync": RsyncFetcher, "imap": IMAPFetcher}[
        source.source_type](source)


def calculate_file_hash(path: str, algorithm: str = "sha256") -> str:
    h = hashlib.new(algorithm)
    with open(path, "rb") as f:
        for block in iter(lambda: f.read(1 << 20), b""):
            h.update(block)
    return h.hexdigest()
