"""Start-up validation (reference parsing/tests/test_startup_validation.py:115-165): a service
whose message bus publisher, subscriber or document store cannot connect exits with code 1
before serving, instead of starting half-wired."""
from __future__ import annotations

import pytest

from copilot_for_consensus_amd.services import main as svc_main
from copilot_for_consensus_amd.services import node as node_mod


class _Broken:
    def __init__(self, inner):
        self.inner = inner

    def connect(self):
        raise ConnectionError("connection refused")

    def __getattr__(self, k):
        return getattr(self.inner, k)


@pytest.fixture(autouse=True)
def _env(monkeypatch):
    for k, v in {"DOCUMENT_STORE_TYPE": "inmemory", "MESSAGE_BUS_TYPE": "inproc", "LOG_TYPE": "silent",
                 "EMBEDDING_BACKEND_TYPE": "mock", "VECTOR_STORE_TYPE": "inmemory", "LLM_BACKEND_TYPE": "mock",
                 "ARCHIVE_STORE_TYPE": "inmemory", "METRICS_TYPE": "noop", "ERROR_REPORTER_TYPE": "silent"}.items():
        monkeypatch.setenv(k, v)
    # never start a server in these tests
    monkeypatch.setattr("copilot_for_consensus_amd.services.base.run_service", lambda *a, **k: None)


@pytest.mark.parametrize("which", ["publisher", "subscriber"])
def test_service_exits_1_when_bus_cannot_connect(monkeypatch, which):
    real = node_mod.create_publisher if which == "publisher" else node_mod.create_subscriber
    monkeypatch.setattr(node_mod, f"create_{which}", lambda *a, **k: _Broken(real(*a, **k)))
    assert svc_main.main(["parsing"]) == 1


def test_service_exits_1_when_document_store_cannot_connect(monkeypatch):
    real = node_mod.create_document_store
    monkeypatch.setattr(node_mod, "create_document_store", lambda *a, **k: _Broken(real(*a, **k)))
    assert svc_main.main(["chunking"]) == 1


def test_healthy_start_connects_everything(monkeypatch):
    seen = []
    real = node_mod.create_publisher

    def pub(*a, **k):
        p = real(*a, **k)
        orig = p.connect
        p.connect = lambda: (seen.append("pub"), orig())[1]
        return p
    monkeypatch.setattr(node_mod, "create_publisher", pub)
    assert svc_main.main(["orchestrator"]) == 0
    assert seen == ["pub"]          # only the selected service's endpoints are connected
