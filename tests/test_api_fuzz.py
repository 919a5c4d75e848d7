"""OpenAPI-driven property tests of the REST surfaces (the reference fuzzes its APIs with
Schemathesis, fuzzing/tests; that library is not installed here, so Hypothesis drives requests
built from each app's own OpenAPI document).  Every GET operation of the ingestion and reporting
services, with arbitrary values for its declared path / query parameters, must answer with a
non-5xx status -- bad input is a 4xx, never a crash."""
from __future__ import annotations

import os
import shutil
import string

import pytest
from fastapi.testclient import TestClient
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from copilot_for_consensus_amd.embedding import HipEncoderProvider
from copilot_for_consensus_amd.services.base import create_app
from copilot_for_consensus_amd.services.ingestion import ingestion_routes
from copilot_for_consensus_amd.services.node import Node
from copilot_for_consensus_amd.services.reporting import reporting_routes
from copilot_for_consensus_amd.summarization import MockSummarizer
from copilot_for_consensus_amd.vectorstore import HipFlatIndex

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "sample.mbox")
ENV = {"DOCUMENT_STORE_TYPE": "inmemory", "MESSAGE_BUS_TYPE": "inproc", "METRICS_TYPE": "prometheus",
       "LOG_TYPE": "silent", "ERROR_REPORTER_TYPE": "silent", "EMBEDDING_BACKEND_TYPE": "mock",
       "VECTOR_STORE_TYPE": "inmemory", "LLM_BACKEND_TYPE": "mock", "ARCHIVE_STORE_TYPE": "inmemory",
       "SECRET_PROVIDER_TYPE": "env"}


@pytest.fixture(scope="module")
def clients(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("fuzz")
    emb = HipEncoderProvider(model_name="tiny", device="cpu")
    node = Node(env={**ENV, "INGESTION_STORAGE_PATH": str(tmp / "ing")}, embedding_provider=emb,
                vector_store=HipFlatIndex(emb.dimension, device="cpu"), summarizer=MockSummarizer(mock_latency_ms=0))
    node.start(threaded=False)
    ing = create_app(node.services["ingestion"])
    ingestion_routes(ing, node.services["ingestion"], None)
    rep = create_app(node.services["reporting"], extra_routes=reporting_routes)
    ci, cr = TestClient(ing), TestClient(rep)
    d = tmp / "src"
    d.mkdir()
    shutil.copy(FIX, d / "list.mbox")
    ci.post("/api/sources", json={"name": "wg", "source_type": "local", "url": str(d)})
    ci.post("/api/sources/wg/trigger")
    node.drain()
    return {"ingestion": ci, "reporting": cr}


def _gets(client):
    spec = client.get("/openapi.json").json()
    for path, ops in sorted(spec["paths"].items()):
        if "get" in ops:
            yield path, ops["get"].get("parameters", [])


_text = st.text(alphabet=string.ascii_letters + string.digits + "-_.:%/ ", max_size=24)


def _value(schema):
    schema = schema or {}
    if "anyOf" in schema:
        return st.one_of([_value(s) for s in schema["anyOf"]])
    t = schema.get("type")
    if t == "integer":
        return st.integers(-10 ** 6, 10 ** 6)
    if t == "number":
        return st.floats(allow_nan=False, allow_infinity=False, width=32)
    if t == "boolean":
        return st.booleans()
    if "enum" in schema:
        return st.sampled_from(schema["enum"]) | _text
    return _text


def _requests(client):
    ops = list(_gets(client))

    @st.composite
    def req(draw):
        path, params = draw(st.sampled_from(ops))
        url, query = path, {}
        for p in params:
            v = draw(_value(p.get("schema")))
            if p["in"] == "path":
                url = url.replace("{" + p["name"] + "}", str(v).replace("/", "_") or "x")
            elif p["in"] == "query" and (p.get("required") or draw(st.booleans())):
                query[p["name"]] = v
        return url, query
    return req()


@pytest.mark.parametrize("service", ["ingestion", "reporting"])
def test_get_operations_never_5xx(clients, service):
    client = clients[service]
    assert len(list(_gets(client))) >= 4

    @settings(max_examples=150, deadline=None, suppress_health_check=list(HealthCheck))
    @given(_requests(client))
    def run(r):
        url, query = r
        resp = client.get(url, params=query)
        assert resp.status_code < 500, (url, query, resp.status_code, resp.text[:200])

    run()


_json_scalar = st.none() | st.booleans() | st.integers(-10 ** 9, 10 ** 9) | _text
_body = st.dictionaries(st.sampled_from(["name", "source_type", "url", "enabled", "port", "username", "folder",
                                         "schedule", "extra"]) | _text, _json_scalar | st.lists(_json_scalar, max_size=3),
                        max_size=8)


def test_source_writes_never_5xx(clients):
    c = clients["ingestion"]

    @settings(max_examples=150, deadline=None, suppress_health_check=list(HealthCheck))
    @given(_body, st.sampled_from(["post", "put"]), _text)
    def run(body, method, name):
        if method == "post":
            r = c.post("/api/sources", json=body)
        else:
            r = c.put(f"/api/sources/{name.replace('/', '_') or 'x'}", json=body)
        assert r.status_code < 500, (method, body, r.status_code, r.text[:200])
        if r.status_code in (200, 201) and method == "post":
            c.delete(f"/api/sources/{body.get('name')}")

    run()


def test_uploads_never_5xx(clients):
    c = clients["ingestion"]

    @settings(max_examples=80, deadline=None, suppress_health_check=list(HealthCheck))
    @given(st.binary(max_size=512), _text, st.sampled_from([".mbox", ".zip", ".tar.gz", ".tgz", ".tar", ".txt", ""]))
    def run(data, stem, ext):
        r = c.post("/api/uploads", files={"file": ((stem or "f") + ext, data, "application/octet-stream")})
        assert r.status_code < 500, (stem + ext, len(data), r.status_code, r.text[:200])

    run()
