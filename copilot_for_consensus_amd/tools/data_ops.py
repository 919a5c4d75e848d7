"""Data-plane maintenance tools for the document store, vector store and bus.

Parity targets (reference ``scripts/``):
  * ``data-migration-export.py`` / ``data-migration-import.py`` -- NDJSON per collection plus a
    ``manifest.json``; import in ``upsert`` (replace) or ``merge`` (patch existing) mode, batched;
  * ``get_data_counts.py`` -- per-collection document counts (+ vector count), table or JSON;
  * ``convert_ndjson_to_csv.py`` -- flatten NDJSON records to CSV (dotted column names);
  * ``backfill_archive_source_type.py`` -- set ``source_type`` on legacy archives (``local``, or
    the type of the archive's source when it is known), ``--dry-run`` / ``--limit``;
  * ``verify_archives_collection.py`` -- archive status histogram and dangling references;
  * ``validate_queue_drainage.py`` -- every queue drained, no duplicate queues, every queue consumed.

The reference implements each of these separately against pymongo / the Cosmos SDK / the RabbitMQ
management API.  Here they are written once against the DocumentStore / VectorStore / broker
interfaces, so they run on the in-process node, Mongo or Cosmos alike.
"""
from __future__ import annotations

import argparse
import csv
import json
import sys
import time
from collections import Counter
from datetime import datetime, timezone
from pathlib import Path
from typing import Any, Iterable, Iterator

# database -> collections, as in the reference's DATABASE_COLLECTIONS (data-migration-export.py:46)
DATABASE_COLLECTIONS = {
    "copilot": ["sources", "archives", "messages", "threads", "chunks", "summaries", "reports"],
    "auth": ["user_roles"],
}
ALL_COLLECTIONS = [c for cs in DATABASE_COLLECTIONS.values() for c in cs]


def _json_default(o):
    if isinstance(o, datetime):
        return o.isoformat()
    if isinstance(o, (bytes, bytearray)):
        return o.hex()
    return str(o)


# ---------------------------------------------------------------------------- export / import
def export_store(store, out_dir: str | Path, collections: Iterable[str] | None = None,
                 source_desc: str = "document_store") -> dict[str, int]:
    """Write ``<out_dir>/<database>/<collection>.ndjson`` + ``manifest.json``; returns counts."""
    out = Path(out_dir)
    wanted = set(collections) if collections else None
    counts: dict[str, int] = {}
    for db, colls in DATABASE_COLLECTIONS.items():
        for c in colls:
            if wanted is not None and c not in wanted:
                continue
            docs = store.query_documents(c, {}, limit=None)
            (out / db).mkdir(parents=True, exist_ok=True)
            with open(out / db / f"{c}.ndjson", "w", encoding="utf-8") as fh:
                for d in sorted(docs, key=lambda d: str(d.get("_id"))):
                    fh.write(json.dumps(d, default=_json_default, sort_keys=True) + "\n")
            counts[c] = len(docs)
    manifest = {"exported_at": datetime.now(timezone.utc).isoformat(), "source": source_desc,
                "databases": {db: [c for c in cs if c in counts] for db, cs in DATABASE_COLLECTIONS.items()},
                "counts": counts, "format": "ndjson"}
    (out / "manifest.json").write_text(json.dumps(manifest, indent=2) + "\n")
    return counts


def iter_ndjson(path: str | Path) -> Iterator[dict]:
    with open(path, encoding="utf-8") as fh:
        for n, line in enumerate(fh, 1):
            line = line.strip()
            if not line:
                continue
            try:
                yield json.loads(line)
            except json.JSONDecodeError as e:
                raise ValueError(f"{path}:{n}: invalid JSON ({e.msg})") from e


def import_store(store, export_dir: str | Path, collections: Iterable[str] | None = None, mode: str = "upsert",
                 batch_size: int = 500) -> dict[str, dict[str, int]]:
    """Load an export into ``store``.  ``upsert`` replaces documents with the same ``_id``;
    ``merge`` patches existing documents field-by-field (new documents are inserted either way)."""
    if mode not in ("upsert", "merge"):
        raise ValueError(f"mode must be upsert|merge, got {mode!r}")
    root = Path(export_dir)
    manifest = json.loads((root / "manifest.json").read_text()) if (root / "manifest.json").exists() else {}
    dbs = manifest.get("databases") or DATABASE_COLLECTIONS
    wanted = set(collections) if collections else None
    stats: dict[str, dict[str, int]] = {}
    for db, colls in dbs.items():
        for c in colls:
            f = root / db / f"{c}.ndjson"
            if (wanted is not None and c not in wanted) or not f.exists():
                continue
            st = stats.setdefault(c, {"inserted": 0, "replaced": 0, "merged": 0, "failed": 0})
            batch: list[dict] = []

            def flush():
                ids = [d["_id"] for d in batch if "_id" in d]
                existing = {d["_id"] for d in store.query_documents(c, {"_id": {"$in": ids}}, limit=None)} if ids else set()
                for d in batch:
                    try:
                        if d.get("_id") in existing:
                            if mode == "merge":
                                store.update_document(c, d["_id"], {k: v for k, v in d.items() if k != "_id"})
                                st["merged"] += 1
                            else:
                                store.delete_document(c, d["_id"])
                                store.insert_document(c, d)
                                st["replaced"] += 1
                        else:
                            store.insert_document(c, d)
                            st["inserted"] += 1
                    except Exception:  # noqa: BLE001 -- one bad record must not stop the import
                        st["failed"] += 1
                batch.clear()

            for d in iter_ndjson(f):
                batch.append(d)
                if len(batch) >= batch_size:
                    flush()
            if batch:
                flush()
    return stats


# ---------------------------------------------------------------------------- counts
def data_counts(store, vector_store=None, collections: Iterable[str] | None = None) -> list[dict[str, Any]]:
    rows = [{"name": c, "kind": "collection", "count": store.count_documents(c)}
            for c in (collections or DATABASE_COLLECTIONS["copilot"])]
    if vector_store is not None:
        n = vector_store.count() if hasattr(vector_store, "count") else len(vector_store)
        rows.append({"name": getattr(vector_store, "collection_name", "embeddings"), "kind": "vectors", "count": int(n)})
    return rows


def format_table(rows: list[dict[str, Any]]) -> str:
    cols = ["name", "kind", "count"]
    w = {c: max(len(c), *(len(str(r[c])) for r in rows)) for c in cols} if rows else {c: len(c) for c in cols}
    line = lambda cells: "  ".join(str(v).ljust(w[c]) for c, v in zip(cols, cells))  # noqa: E731
    return "\n".join([line(cols), line(["-" * w[c] for c in cols])] + [line([r[c] for c in cols]) for r in rows])


# ---------------------------------------------------------------------------- ndjson -> csv
def _flatten(d: dict, prefix: str = "") -> dict[str, Any]:
    out: dict[str, Any] = {}
    for k, v in d.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict):
            out.update(_flatten(v, key + "."))
        elif isinstance(v, list):
            out[key] = json.dumps(v, default=_json_default)
        else:
            out[key] = v
    return out


def ndjson_to_csv(src: str | Path, dst: str | Path, fields: list[str] | None = None) -> int:
    rows = [_flatten(r) for r in iter_ndjson(src)]
    cols = fields or sorted({k for r in rows for k in r})
    with open(dst, "w", newline="", encoding="utf-8") as fh:
        w = csv.DictWriter(fh, fieldnames=cols, extrasaction="ignore")
        w.writeheader()
        for r in rows:
            w.writerow({c: r.get(c, "") for c in cols})
    return len(rows)


# ---------------------------------------------------------------------------- migrations / checks
def backfill_archive_source_type(store, dry_run: bool = False, limit: int | None = None,
                                 default: str = "local") -> dict[str, int]:
    todo = store.query_documents("archives", {"source_type": {"$exists": False}}, limit=limit)
    types = {s.get("name"): s.get("source_type") for s in store.query_documents("sources", {}, limit=None)}
    stats = {"total_found": len(todo), "updated": 0, "errors": 0}
    for a in todo:
        st = types.get(a.get("source")) or default
        if dry_run:
            continue
        try:
            store.update_document("archives", a["_id"], {"$set": {"source_type": st}})
            stats["updated"] += 1
        except Exception:  # noqa: BLE001
            stats["errors"] += 1
    return stats


def verify_archives(store) -> dict[str, Any]:
    archives = store.query_documents("archives", {}, limit=None)
    ids = {a["_id"] for a in archives}
    status = Counter(a.get("status", "<missing>") for a in archives)
    missing_fields = sorted(a["_id"] for a in archives
                            if any(f not in a for f in ("file_hash", "source", "status")))
    orphan_msgs = store.count_documents("messages", {"archive_id": {"$nin": sorted(ids)}}) if ids else \
        store.count_documents("messages")
    return {"archives": len(archives), "status": dict(status), "missing_required_fields": missing_fields,
            "messages_without_archive": orphan_msgs, "ok": not missing_fields and orphan_msgs == 0}


def check_queue_drainage(queues: list[dict[str, Any]], max_depth: int = 0) -> dict[str, Any]:
    """``queues``: [{name, messages, consumers}] (RabbitMQ management API shape)."""
    names = [q["name"] for q in queues]
    dup = sorted(n for n, k in Counter(names).items() if k > 1)
    # the reference also flags near-duplicates that differ only by a ".v1"-style suffix
    base = Counter(n.rsplit(".v", 1)[0] for n in set(names))
    dup += sorted(n for n, k in base.items() if k > 1 and n not in dup)
    undrained = sorted(q["name"] for q in queues if q.get("messages", 0) > max_depth and not q["name"].endswith(".failed"))
    unconsumed = sorted(q["name"] for q in queues if q.get("consumers", 0) == 0 and not q["name"].endswith(".failed"))
    return {"duplicates": dup, "undrained": undrained, "without_consumers": unconsumed,
            "ok": not dup and not undrained and not unconsumed}


def broker_queue_stats(broker) -> list[dict[str, Any]]:
    """Queue stats of the in-process broker in the management-API shape."""
    consumers = broker.consumer_counts()
    return [{"name": n, "messages": d, "consumers": consumers.get(n, 0)} for n, d in broker.queues().items()]


def wait_for_drainage(broker, timeout_s: float = 60.0, poll_s: float = 0.2) -> bool:
    end = time.monotonic() + timeout_s
    while time.monotonic() < end:
        if all(d == 0 for d in broker.queues().values()):
            return True
        time.sleep(poll_s)
    return False


# ---------------------------------------------------------------------------- CLI
def _store_from_args(a):
    from ..storage.document_store import create_document_store

    class _Cfg:
        driver_name = a.store
        driver_config = {k: v for k, v in (("host", a.host), ("port", a.port), ("database", a.database),
                                           ("username", a.username), ("password", a.password)) if v is not None}

    s = create_document_store(_Cfg)
    s.connect()
    if a.store == "inmemory" and a.snapshot:
        import_store(s, a.snapshot)
    return s


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="document-store maintenance (see module docstring)")
    ap.add_argument("--store", default="inmemory", choices=["inmemory", "mongodb", "azure_cosmosdb"])
    ap.add_argument("--snapshot", help="inmemory: load this export directory first")
    for k in ("host", "port", "database", "username", "password"):
        ap.add_argument(f"--{k}")
    sub = ap.add_subparsers(dest="cmd", required=True)
    e = sub.add_parser("export")
    e.add_argument("--output-dir", default=None)
    e.add_argument("--collections")
    i = sub.add_parser("import")
    i.add_argument("--export-dir", required=True)
    i.add_argument("--collections")
    i.add_argument("--mode", choices=["upsert", "merge"], default="upsert")
    i.add_argument("--batch-size", type=int, default=500)
    c = sub.add_parser("counts")
    c.add_argument("--format", choices=["table", "json"], default="table")
    v = sub.add_parser("ndjson-to-csv")
    v.add_argument("src")
    v.add_argument("dst")
    v.add_argument("--fields")
    b = sub.add_parser("backfill-source-type")
    b.add_argument("--dry-run", action="store_true")
    b.add_argument("--limit", type=int)
    sub.add_parser("verify-archives")
    a = ap.parse_args(argv)
    if a.cmd == "ndjson-to-csv":
        print(ndjson_to_csv(a.src, a.dst, a.fields.split(",") if a.fields else None))
        return 0
    store = _store_from_args(a)
    cols = a.collections.split(",") if getattr(a, "collections", None) else None
    if a.cmd == "export":
        out = a.output_dir or f"data-export-{datetime.now(timezone.utc).strftime('%Y%m%dT%H%M%SZ')}"
        print(json.dumps(export_store(store, out, cols, source_desc=a.store)))
    elif a.cmd == "import":
        print(json.dumps(import_store(store, a.export_dir, cols, a.mode, a.batch_size)))
    elif a.cmd == "counts":
        rows = data_counts(store)
        print(json.dumps(rows) if a.format == "json" else format_table(rows))
    elif a.cmd == "backfill-source-type":
        print(json.dumps(backfill_archive_source_type(store, a.dry_run, a.limit)))
    elif a.cmd == "verify-archives":
        res = verify_archives(store)
        print(json.dumps(res))
        return 0 if res["ok"] else 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
