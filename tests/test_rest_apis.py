"""REST surfaces of the services (reference ingestion/tests/test_api.py, reporting/tests/test_api.py,
auth/tests/test_main.py): source CRUD and error codes, uploads (multipart, raw, zip/tar archives),
report/thread filters, pagination and sorting, health/readiness/stats/config-schema routes, and the
auth service's login, token, JWKS and admin routes."""
from __future__ import annotations

import io
import os
import shutil
import tarfile
import zipfile

import pytest
from fastapi.testclient import TestClient

from copilot_for_consensus_amd.embedding import HipEncoderProvider
from copilot_for_consensus_amd.security.auth import AuthService, MockIdentityProvider, RoleStore
from copilot_for_consensus_amd.security.jwt import HMACSigner, JWTManager
from copilot_for_consensus_amd.services.auth import create_auth_app
from copilot_for_consensus_amd.services.base import create_app
from copilot_for_consensus_amd.services.ingestion import ingestion_routes
from copilot_for_consensus_amd.services.node import Node
from copilot_for_consensus_amd.services.reporting import reporting_routes
from copilot_for_consensus_amd.storage.document_store import InMemoryDocumentStore
from copilot_for_consensus_amd.summarization import MockSummarizer
from copilot_for_consensus_amd.vectorstore import HipFlatIndex

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "sample.mbox")
ENV = {"DOCUMENT_STORE_TYPE": "inmemory", "MESSAGE_BUS_TYPE": "inproc", "METRICS_TYPE": "prometheus",
       "LOG_TYPE": "silent", "ERROR_REPORTER_TYPE": "silent", "EMBEDDING_BACKEND_TYPE": "mock",
       "VECTOR_STORE_TYPE": "inmemory", "LLM_BACKEND_TYPE": "mock", "ARCHIVE_STORE_TYPE": "inmemory",
       "SECRET_PROVIDER_TYPE": "env"}


@pytest.fixture
def stack(tmp_path):
    emb = HipEncoderProvider(model_name="tiny", device="cpu")
    node = Node(env={**ENV, "INGESTION_STORAGE_PATH": str(tmp_path / "ing")}, embedding_provider=emb,
                vector_store=HipFlatIndex(emb.dimension, device="cpu"), summarizer=MockSummarizer(mock_latency_ms=0))
    node.start(threaded=False)
    ing_app = create_app(node.services["ingestion"])
    ingestion_routes(ing_app, node.services["ingestion"], None)
    rep_app = create_app(node.services["reporting"], extra_routes=reporting_routes)
    return node, TestClient(ing_app), TestClient(rep_app), tmp_path


def test_source_crud_and_errors(stack):
    node, ing, _, tmp = stack
    src = {"name": "wg", "source_type": "local", "url": str(tmp)}
    assert ing.post("/api/sources", json=src).status_code == 201
    assert ing.post("/api/sources", json=src).status_code == 400          # duplicate
    assert ing.post("/api/sources", json={"name": "x", "source_type": "gopher", "url": "u"}).status_code == 400
    assert ing.get("/api/sources/wg").json()["source_type"] == "local"
    assert ing.get("/api/sources/nope").status_code == 404
    assert ing.put("/api/sources/wg", json={**src, "name": "other"}).status_code == 400
    r = ing.put("/api/sources/wg", json={**src, "enabled": False})
    assert r.status_code == 200
    assert ing.post("/api/sources/wg/trigger").status_code == 400         # disabled
    assert ing.post("/api/sources/ghost/trigger").status_code == 404
    assert ing.get("/api/sources/wg/status").status_code == 200
    assert [s["name"] for s in ing.get("/api/sources").json()["sources"]] == ["wg"]
    assert ing.delete("/api/sources/wg").status_code in (200, 204)
    assert ing.delete("/api/sources/wg").status_code == 404


def test_uploads(stack):
    node, ing, _, tmp = stack
    data = open(FIX, "rb").read()
    r = ing.post("/api/uploads", files={"file": ("list.mbox", data, "application/mbox")})
    assert r.status_code == 201, r.text
    body = r.json()
    assert body["filename"] == "list.mbox" and body["size_bytes"] == len(data) and len(body["archive_id"]) == 16
    r = ing.post("/api/uploads?filename=raw.mbox", content=data, headers={"Content-Type": "application/octet-stream"})
    assert r.status_code == 201
    assert ing.post("/api/uploads", files={"file": ("evil.exe", b"MZ", "application/octet-stream")}).status_code == 400
    assert ing.post("/api/uploads", files={"file": ("empty.mbox", b"", "application/mbox")}).status_code == 400
    # path components are stripped from the uploaded name
    r = ing.post("/api/uploads", files={"file": ("../../etc/x.mbox", data, "application/mbox")})
    assert r.status_code == 201 and "/" not in r.json()["filename"] and ".." not in r.json()["filename"]


def _zip(data):
    b = io.BytesIO()
    with zipfile.ZipFile(b, "w") as z:
        z.writestr("a/list.mbox", data)
    return b.getvalue()


def _tgz(data):
    b = io.BytesIO()
    with tarfile.open(fileobj=b, mode="w:gz") as t:
        info = tarfile.TarInfo("list.mbox")
        info.size = len(data)
        t.addfile(info, io.BytesIO(data))
    return b.getvalue()


@pytest.mark.parametrize("name,pack", [("bundle.zip", _zip), ("bundle.tar.gz", _tgz)])
def test_archive_bundles_are_expanded(stack, name, pack):
    node, ing, rep, tmp = stack
    d = tmp / "bundle"
    d.mkdir()
    (d / name).write_bytes(pack(open(FIX, "rb").read()))
    assert ing.post("/api/sources", json={"name": "b", "source_type": "local", "url": str(d)}).status_code == 201
    r = ing.post("/api/sources/b/trigger")
    assert r.status_code == 200 and len(r.json()["archive_ids"]) == 1
    node.drain()
    assert node.store.count_documents("messages") == 10


def test_reporting_filters_pagination_sorting(stack):
    node, ing, rep, tmp = stack
    d = tmp / "src"
    d.mkdir()
    shutil.copy(FIX, d / "list.mbox")
    ing.post("/api/sources", json={"name": "wg", "source_type": "local", "url": str(d)})
    ing.post("/api/sources/wg/trigger")
    node.drain()
    all_r = rep.get("/api/reports", params={"limit": 100}).json()
    assert all_r["count"] == 2
    p1 = rep.get("/api/reports", params={"limit": 1}).json()["reports"]
    p2 = rep.get("/api/reports", params={"limit": 1, "skip": 1}).json()["reports"]
    assert len(p1) == len(p2) == 1 and p1[0]["_id"] != p2[0]["_id"]
    asc = [r["_id"] for r in rep.get("/api/reports", params={"sort_order": "asc", "limit": 10}).json()["reports"]]
    desc = [r["_id"] for r in rep.get("/api/reports", params={"sort_order": "desc", "limit": 10}).json()["reports"]]
    assert asc == list(reversed(desc))
    assert rep.get("/api/reports", params={"sort_order": "sideways"}).status_code == 422
    assert rep.get("/api/reports", params={"limit": 101}).status_code == 422
    assert rep.get("/api/reports", params={"min_participants": 99}).json()["count"] == 0
    assert rep.get("/api/reports", params={"message_start_date": "2999-01-01"}).json()["count"] == 0
    assert rep.get("/api/reports", params={"message_end_date": "2999-01-01"}).json()["count"] == 2
    tid = all_r["reports"][0]["thread_id"]
    assert rep.get("/api/reports", params={"thread_id": tid}).json()["count"] == 1
    assert rep.get("/api/reports/doesnotexist").status_code == 404
    assert rep.get("/api/threads/doesnotexist").status_code == 404
    assert rep.get("/api/threads/doesnotexist/summary").status_code == 404
    assert rep.get("/api/messages/doesnotexist").status_code == 404
    assert rep.get("/api/chunks/doesnotexist").status_code == 404
    th = rep.get("/api/threads", params={"limit": 10, "sort_by": "first_message_date", "sort_order": "asc"}).json()
    firsts = [t["first_message_date"] for t in th["threads"]]
    assert firsts == sorted(firsts) and all(t["archive_source"] == "wg" for t in th["threads"])
    # the reference accepts only these sort keys (reporting/main.py:152-156, 319-323)
    assert rep.get("/api/threads", params={"sort_by": "message_count"}).status_code == 422
    assert rep.get("/api/reports", params={"sort_by": "title"}).status_code == 422
    assert rep.get("/api/reports/search", params={"topic": "x", "limit": 51}).status_code == 422


def test_service_meta_routes(stack):
    _, ing, rep, _ = stack
    for c in (ing, rep):
        assert c.get("/health").json()["status"] == "healthy"
        assert c.get("/readyz").status_code == 200
        assert "events_processed" in c.get("/stats").json()
        sch = c.get("/.well-known/configuration-schema").json()
        assert "service_settings" in sch and "adapters" in sch


# ------------------------------------------------------------------ auth service
@pytest.fixture
def auth_client():
    store = InMemoryDocumentStore()
    svc = AuthService(JWTManager(HMACSigner("k")), RoleStore(store, first_user_auto_promotion=True),
                      {"mock": MockIdentityProvider()})
    return TestClient(create_auth_app(svc, token_exchange_secret="s3"))


def _login(c, code):
    start = c.get("/login", params={"provider": "mock"}).json()
    r = c.get("/callback", params={"code": code, "state": start["state"]})
    assert r.status_code == 200, r.text
    assert "auth_token" in r.cookies
    return r.json()["access_token"]


def test_auth_login_userinfo_admin(auth_client):
    c = auth_client
    assert c.get("/providers").json() == {"providers": ["mock"]}
    assert c.get("/login", params={"provider": "nope"}).status_code == 400
    assert c.get("/login", params={"provider": "mock", "redirect": True}, follow_redirects=False).status_code in (302, 307)
    admin = _login(c, "alice")                     # first user: auto-promoted admin
    user = _login(c, "bob")                        # pending, no roles
    h = lambda t: {"Authorization": f"Bearer {t}"}  # noqa: E731
    assert c.get("/userinfo", headers=h(admin)).json()["roles"] == ["admin", "reader"]
    assert c.get("/userinfo").json()["sub"] == "mock:bob"        # the callback's auth_token cookie
    c.cookies.clear()
    assert c.get("/userinfo").status_code == 401
    assert c.get("/admin/role-assignments/pending", headers=h(user)).status_code == 403
    pend = c.get("/admin/role-assignments/pending", headers=h(admin)).json()["pending"]
    assert [p["_id"] for p in pend] == ["mock:bob"]
    assert c.post("/admin/users/mock:bob/roles", json={"roles": ["reader"]}, headers=h(admin)).json()["roles"] == ["reader"]
    assert c.get("/admin/users/mock:bob/roles", headers=h(admin)).json()["status"] == "approved"
    assert c.get("/admin/users/ghost/roles", headers=h(admin)).status_code == 404
    assert c.get("/admin/users/search", params={"q": "bob"}, headers=h(admin)).json()["users"][0]["_id"] == "mock:bob"
    r = c.request("DELETE", "/admin/users/mock:bob/roles", json={"roles": ["reader"]}, headers=h(admin))
    assert r.json()["roles"] == []
    assert c.post("/admin/users/mock:bob/deny", headers=h(admin)).status_code == 409   # approved, not pending
    _login(c, "carol")
    assert c.post("/admin/users/mock:carol/deny", headers=h(admin)).json()["status"] == "denied"
    refreshed = c.get("/refresh", headers=h(admin)).json()["access_token"]
    assert c.get("/userinfo", headers=h(refreshed)).status_code == 200
    assert c.post("/logout").status_code == 200


def test_auth_token_exchange_and_jwks(auth_client):
    c = auth_client
    assert c.post("/token", json={"secret": "wrong"}).status_code == 401
    tok = c.post("/token", json={"secret": "s3", "subject": "parsing", "roles": ["processor"]}).json()["access_token"]
    assert c.get("/userinfo", headers={"Authorization": f"Bearer {tok}"}).json()["roles"] == ["processor"]
    assert c.get("/keys").json() == {"keys": []}          # HMAC signer publishes nothing
    assert c.get("/.well-known/public_key.pem").status_code == 404


def test_ingestion_api_reference_semantics(stack):
    """Reference ingestion/tests/test_api.py behaviours: duplicate source 400 'already exists',
    missing fields 422, uploads never overwrite each other, path parts stripped from names,
    compound extensions accepted, re-trigger re-ingests."""
    node, ing, _, tmp = stack
    assert ing.post("/api/sources", json={"name": "x"}).status_code == 422
    body = {"name": "dup", "source_type": "local", "url": str(tmp)}
    assert ing.post("/api/sources", json=body).status_code == 201
    r = ing.post("/api/sources", json=body)
    assert r.status_code == 400 and "already exists" in r.json()["detail"]
    data = open(FIX, "rb").read()
    u1 = ing.post("/api/uploads", params={"filename": "test.mbox"}, content=data).json()
    u2 = ing.post("/api/uploads", params={"filename": "test.mbox"}, content=data).json()
    assert u1["filename"] == "test.mbox" and u2["filename"] == "test_1.mbox"
    u3 = ing.post("/api/uploads", params={"filename": "../../etc/a.tar.gz"}, content=_tgz(data)).json()
    assert ".." not in u3["filename"] and "/" not in u3["filename"] and u3["filename"].endswith(".tar.gz")
    assert ing.post("/api/uploads", params={"filename": "x.exe"}, content=b"MZ").status_code == 400
    assert ing.post("/api/uploads", params={"filename": "e.mbox"}, content=b"").status_code == 400
    assert ing.post("/api/sources/nope/trigger").status_code == 404
