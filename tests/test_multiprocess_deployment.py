"""The reference's compose topology as separate OS processes, talking only over TCP.

Infrastructure: the native broker (RabbitMQ's role), the document store server (MongoDB's role)
and the Qdrant-REST vector store (Qdrant's role).  Services: ingestion, parsing, chunking,
embedding, orchestrator, summarization and reporting, each one ``python -m
copilot_for_consensus_amd.services.main <service>`` process with its own uvicorn + consumer thread
(reference <service>/main.py).  The flow is the reference's docker-compose CI job
(.github/workflows/docker-compose-ci.yml:339-521): create a source and trigger it through the
ingestion REST API, then poll the reporting API until the reports exist.  Then the chunking
service is killed with SIGKILL, a second archive is uploaded while it is down (its events wait in
the broker's durable ``chunking`` queue), the service is restarted and the pipeline completes.
"""
from __future__ import annotations

import json
import os
import shutil
import signal
import socket
import subprocess
import sys
import time
import urllib.error
import urllib.parse
import urllib.request

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "fixtures", "sample.mbox")
SERVICES = ("ingestion", "parsing", "chunking", "embedding", "orchestrator", "summarization", "reporting")


_TAKEN: set[int] = set()


def _free_port() -> int:
    """A free port BELOW the kernel's ephemeral range: a port bind(0) hands out stays in that range,
    so another process's outgoing connection could take it before the service binds it (seen as
    "address already in use" when the services start one after another)."""
    import random
    try:
        lo = int(open("/proc/sys/net/ipv4/ip_local_port_range").read().split()[0])
    except (OSError, ValueError):
        lo = 32768
    rng = random.Random()
    for _ in range(1000):
        p = rng.randrange(max(1024, lo - 12000), lo)
        if p in _TAKEN:
            continue
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", p))
            except OSError:
                continue
        _TAKEN.add(p)
        return p
    raise RuntimeError("no free port below the ephemeral range")


def _http(method: str, url: str, body=None, headers=None, timeout=10):
    data = body if isinstance(body, (bytes, type(None))) else json.dumps(body).encode()
    h = {"Content-Type": "application/json"} if isinstance(body, (dict, list)) else {}
    h.update(headers or {})
    req = urllib.request.Request(url, data=data, method=method, headers=h)
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return r.status, json.loads(r.read() or b"null")
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode(errors="replace")


class Deployment:
    def __init__(self, tmp, overrides: dict | None = None):
        self.tmp = tmp
        self.procs: dict[str, subprocess.Popen] = {}
        self.ports = {n: _free_port() for n in ("broker", "docstore", "vectorstore", "llm", "auth", *SERVICES)}
        self.env = {**os.environ, "PYTHONPATH": ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""),
                    "MESSAGE_BUS_TYPE": "cfcbroker", "CFC_BROKER_HOST": "127.0.0.1",
                    "CFC_BROKER_PORT": str(self.ports["broker"]),
                    "DOCUMENT_STORE_TYPE": "cfcstore", "CFC_DOCSTORE_HOST": "127.0.0.1",
                    "CFC_DOCSTORE_PORT": str(self.ports["docstore"]),
                    "VECTOR_STORE_TYPE": "qdrant", "QDRANT_HOST": "127.0.0.1",
                    "QDRANT_PORT": str(self.ports["vectorstore"]), "VECTOR_STORE_DEVICE": "cpu",
                    "EMBEDDING_BACKEND_TYPE": "mock", "LLM_BACKEND_TYPE": "mock", "MOCK_LATENCY_MS": "0",
                    "ARCHIVE_STORE_TYPE": "local", "ARCHIVE_BASE_PATH": str(tmp / "archives"),
                    "INGESTION_STORAGE_PATH": str(tmp / "ingestion"),
                    "METRICS_TYPE": "noop", "LOG_TYPE": "silent", "ERROR_REPORTER_TYPE": "silent",
                    "SECRET_PROVIDER_TYPE": "env", "JWT_AUTH_ENABLED": "false", "CUDA_VISIBLE_DEVICES": "",
                    "HIP_VISIBLE_DEVICES": "", "OMP_NUM_THREADS": "1"}
        for k, v in (overrides or {}).items():
            if v is None:
                self.env.pop(k, None)
            else:
                self.env[k] = v

    def start(self, name: str, *extra: str) -> None:
        log = open(self.tmp / f"{name}.log", "ab")
        cmd = [sys.executable, "-m", "copilot_for_consensus_amd.services.main", name, "--port", str(self.ports[name]),
               *extra]
        self.procs[name] = subprocess.Popen(cmd, env=self.env, stdout=log, stderr=subprocess.STDOUT,
                                            start_new_session=True)

    def wait_tcp(self, name: str, timeout=60) -> None:
        deadline = time.time() + timeout
        while time.time() < deadline:
            self._alive(name)
            try:
                socket.create_connection(("127.0.0.1", self.ports[name]), timeout=1).close()
                return
            except OSError:
                time.sleep(0.1)
        raise TimeoutError(f"{name} did not listen: {self.log(name)}")

    def wait_ready(self, name: str, timeout=120) -> None:
        deadline = time.time() + timeout
        while time.time() < deadline:
            self._alive(name)
            try:
                if _http("GET", self.url(name, "/readyz"), timeout=2)[0] == 200:
                    return
            except OSError:
                pass
            time.sleep(0.2)
        raise TimeoutError(f"{name} not ready: {self.log(name)}")

    def _alive(self, name):
        p = self.procs[name]
        if p.poll() is not None:
            raise RuntimeError(f"{name} exited {p.returncode}: {self.log(name)}")

    def url(self, name: str, path: str) -> str:
        return f"http://127.0.0.1:{self.ports[name]}{path}"

    def log(self, name: str) -> str:
        try:
            lines = (self.tmp / f"{name}.log").read_text(errors="replace").splitlines()
            return "\n".join(ln for ln in lines if "uvicorn.access" not in ln)[-3000:]
        except OSError:
            return ""

    def kill(self, name: str, sig=signal.SIGKILL) -> None:
        p = self.procs.pop(name)
        os.killpg(p.pid, sig)
        p.wait(30)

    def stop_all(self) -> None:
        for name in list(self.procs):
            p = self.procs.pop(name)
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                    p.wait(15)
                except Exception:
                    os.killpg(p.pid, signal.SIGKILL)
                    p.wait(5)


@pytest.fixture
def deployment(tmp_path):
    made = []

    def make(overrides=None):
        made.append(Deployment(tmp_path, overrides))
        return made[-1]

    yield make
    for d in made:
        d.stop_all()


def _reports(d) -> list:
    code, body = _http("GET", d.url("reporting", "/api/reports?limit=100"))
    return body["reports"] if code == 200 else []


def _wait_reports(d, n, timeout=180) -> list:
    deadline = time.time() + timeout
    while time.time() < deadline:
        r = _reports(d)
        if len(r) >= n:
            return r
        for s in list(d.procs):
            d._alive(s)
        time.sleep(0.3)
    from copilot_for_consensus_amd.bus.cfcbroker import Connection
    stats = Connection("127.0.0.1", d.ports["broker"]).stats()["queues"]
    logs = "\n".join(f"--- {s}\n{d.log(s)}" for s in SERVICES)
    raise TimeoutError(f"{len(_reports(d))} of {n} reports; queues {stats}\n{logs}")


@pytest.mark.timeout(600)
def test_services_as_processes_over_broker_and_stores(deployment, tmp_path):
    """CPU: mock embedding + mock LLM (the reference CI's configuration), HIP index on the CPU path."""
    _run(deployment(), tmp_path)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_services_as_processes_on_the_gpu(deployment, tmp_path):
    """MI355X: the embedding and reporting processes run the HIP MiniLM encoder, the vector store
    process holds the index in HBM behind the Qdrant REST API, the summarization process runs the
    HIP decoder (tiny preset, random init) -- four processes sharing the GPU."""
    _run(deployment({"CUDA_VISIBLE_DEVICES": None, "HIP_VISIBLE_DEVICES": None, "EMBEDDING_BACKEND_TYPE": "hip",
                     "EMBEDDING_DEVICE": "cuda", "VECTOR_STORE_DEVICE": "cuda", "LLM_BACKEND_TYPE": "hip",
                     "LLM_MODEL_PRESET": "tiny", "LLM_MAX_NEW_TOKENS": "32", "LLM_KV_CACHE_TOKENS": "65536"}),
         tmp_path)


@pytest.mark.timeout(600)
def test_summarization_through_llamacpp_api_of_llm_server(deployment, tmp_path):
    """The reference's llama.cpp topology: the summarization service uses the llama.cpp HTTP driver
    (LLM_BACKEND_TYPE=llamacpp, /completion, temperature 0.7, stops) against this framework's LLM
    server process (tiny random-init decoder on the CPU path)."""
    d = deployment({"LLM_BACKEND_TYPE": "llamacpp", "LLM_MODEL_PRESET": "tiny", "LLM_DEVICE": "cpu",
                    "LLM_MAX_BATCH": "4", "LLM_MAX_NEW_TOKENS": "24", "LLM_KV_CACHE_TOKENS": "32768"})
    d.env["LLAMACPP_ENDPOINT"] = f"http://127.0.0.1:{d.ports['llm']}"
    d.start("llm")
    _run(d, tmp_path, extra_infra=("llm",), late_archive=False)


def _run(d, tmp_path, extra_infra=(), late_archive=True):
    from copilot_for_consensus_amd.bus.cfcbroker import Connection
    from copilot_for_consensus_amd.utils.synthetic import SyntheticArchive

    d.start("broker", "--data-dir", str(tmp_path / "broker"))
    d.start("docstore", "--data-dir", str(tmp_path / "docstore"))
    d.start("vectorstore")
    for n in ("broker", "docstore", "vectorstore", *extra_infra):
        d.wait_tcp(n)
    for s in SERVICES:
        d.start(s)
    for s in SERVICES:
        d.wait_ready(s)

    src = tmp_path / "src"
    src.mkdir()
    shutil.copy(FIX, src / "list.mbox")
    code, body = _http("POST", d.url("ingestion", "/api/sources"), {"name": "wg", "source_type": "local",
                                                                     "url": str(src)})
    assert code == 201, body
    code, body = _http("POST", d.url("ingestion", "/api/sources/wg/trigger"))
    assert code == 200 and len(body["archive_ids"]) == 1, body
    reports = _wait_reports(d, 2)
    # a thread's summary_id is written right after its report: poll briefly (busy CI hosts)
    deadline = time.time() + 60
    while True:
        code, threads = _http("GET", d.url("reporting", "/api/threads"))
        if all(t["summary_id"] for t in threads["threads"]) or time.time() > deadline:
            break
        time.sleep(0.2)
    assert all(t["summary_id"] for t in threads["threads"]), (
        threads, [r["_id"] for r in _reports(d)], d.log("orchestrator"), d.log("summarization"))
    code, rep = _http("GET", d.url("reporting", f"/api/reports/{reports[0]['_id']}"))
    assert code == 200 and rep["content_markdown"]
    # semantic topic search: reporting embeds the topic, the vector store answers over REST
    code, msgs = _http("GET", d.url("reporting", f"/api/messages?thread_id={rep['thread_id']}"))
    topic = urllib.request.quote(msgs["messages"][0]["body_normalized"][:120])
    code, hits = _http("GET", d.url("reporting", f"/api/reports/search?topic={topic}&min_score=0.0"))
    assert code == 200 and hits["count"] >= 1, hits

    if not late_archive:
        return
    # chunking dies; a second archive arrives while it is down; its events wait in the broker
    d.kill("chunking")
    mbox = SyntheticArchive(seed=7).mbox(3)
    boundary = "cfcboundary"
    form = (f"--{boundary}\r\nContent-Disposition: form-data; name=\"file\"; filename=\"late.mbox\"\r\n"
            f"Content-Type: application/mbox\r\n\r\n").encode() + mbox + f"\r\n--{boundary}--\r\n".encode()
    code, body = _http("POST", d.url("ingestion", "/api/uploads"), form,
                       headers={"Content-Type": f"multipart/form-data; boundary={boundary}"})
    assert code == 201, body
    code, body = _http("POST", d.url("ingestion", "/api/sources"),
                       {"name": "late", "source_type": "local", "url": body.get("server_path") or body.get("path")})
    code, body = _http("POST", d.url("ingestion", "/api/sources/late/trigger"))
    assert code == 200 and len(body["archive_ids"]) == 1, body
    admin = Connection("127.0.0.1", d.ports["broker"])
    deadline = time.time() + 60
    while time.time() < deadline and admin.stats()["queues"]["chunking"]["ready"] == 0:
        time.sleep(0.2)
    assert admin.stats()["queues"]["chunking"]["ready"] > 0      # parsed, waiting for chunking
    assert len(_reports(d)) == 2
    d.start("chunking")
    reports = _wait_reports(d, 5)
    assert len(reports) == 5
    deadline = time.time() + 60        # the last events (reporting, cleanup) may still be in flight
    while True:
        st = admin.stats()["queues"]
        if all(st[q]["ready"] == 0 and st[q]["unacked"] == 0 for q in SERVICES if q in st) or time.time() > deadline:
            break
        time.sleep(0.2)
    assert all(st[q]["ready"] == 0 and st[q]["unacked"] == 0 for q in SERVICES if q in st), st
    assert not any(q.endswith(".dlq") and v["ready"] for q, v in st.items())


@pytest.mark.timeout(600)
def test_jwt_auth_across_processes(deployment, tmp_path):
    """Auth as its own process (RS256 keys, mock OIDC provider, roles in the shared document store);
    ingestion and reporting in theirs verify bearer tokens against its JWKS (reference
    copilot_auth/middleware.py:122-270, role checks :424; ingestion requires admin, reporting reader)."""
    from copilot_for_consensus_amd.security.jwt import generate_keys
    priv, pub = generate_keys(tmp_path / "secrets")      # what tools.generate_keys writes
    d = deployment({"JWT_AUTH_ENABLED": "true", "AUTH_ENABLE_MOCK_PROVIDER": "true",
                    "AUTH_FIRST_USER_AUTO_PROMOTION_ENABLED": "true", "AUTH_JWT_ALGORITHM": "RS256",
                    "JWT_PRIVATE_KEY": priv.read_text(), "JWT_PUBLIC_KEY": pub.read_text()})
    auth_url = f"http://127.0.0.1:{d.ports['auth']}"
    d.env.update({"INGESTION_AUTH_SERVICE_URL": auth_url, "REPORTING_AUTH_SERVICE_URL": auth_url,
                  "AUTH_PORT": str(d.ports["auth"])})
    d.start("broker", "--data-dir", str(tmp_path / "broker"))
    d.start("docstore")
    d.start("vectorstore")
    for n in ("broker", "docstore", "vectorstore"):
        d.wait_tcp(n)
    d.start("auth")
    d.wait_tcp("auth")
    for s in ("ingestion", "reporting"):
        d.start(s)
    for s in ("ingestion", "reporting"):
        d.wait_ready(s)

    def login(user):
        code, r = _http("GET", d.url("auth", "/login?provider=mock"))
        assert code == 200, r
        state = urllib.parse.parse_qs(urllib.parse.urlparse(r["authorization_url"]).query)["state"][0]
        code, tok = _http("GET", d.url("auth", f"/callback?code={user}&state={state}"))
        assert code == 200, tok
        return tok["access_token"]

    admin = login("alice")            # first user: promoted to admin
    nobody = login("bob")             # second user: no roles until approved
    body = {"name": "wg", "source_type": "local", "url": str(tmp_path)}
    assert _http("POST", d.url("ingestion", "/api/sources"), body)[0] == 401
    assert _http("POST", d.url("ingestion", "/api/sources"), body, {"Authorization": "Bearer junk"})[0] == 401
    assert _http("POST", d.url("ingestion", "/api/sources"), body, {"Authorization": f"Bearer {nobody}"})[0] == 403
    assert _http("POST", d.url("ingestion", "/api/sources"), body, {"Authorization": f"Bearer {admin}"})[0] == 201
    assert _http("GET", d.url("reporting", "/api/reports"))[0] == 401
    code, rep = _http("GET", d.url("reporting", "/api/reports"), headers={"Authorization": f"Bearer {admin}"})
    assert code == 200 and rep["count"] == 0
    assert _http("GET", d.url("reporting", "/health"))[0] == 200            # health stays public
    # the admin grants bob the reader role through the auth admin API; his NEW token reads reports
    code, _ = _http("POST", d.url("auth", "/admin/users/mock:bob/roles"), {"roles": ["reader"]},
                    {"Authorization": f"Bearer {admin}"})
    assert code == 200
    bob2 = login("bob")
    assert _http("GET", d.url("reporting", "/api/reports"), headers={"Authorization": f"Bearer {bob2}"})[0] == 200
    assert _http("POST", d.url("ingestion", "/api/sources"), {**body, "name": "x"},
                 {"Authorization": f"Bearer {bob2}"})[0] == 403


@pytest.mark.timeout(180)
def test_standalone_ingestion_process_runs_its_scheduler(tmp_path):
    """`main ingestion` on its own (the compose topology's ingestion container) starts
    the periodic IngestionScheduler, as the reference's ingestion/main.py does; /health says so."""
    d = Deployment(tmp_path, {"MESSAGE_BUS_TYPE": "noop", "DOCUMENT_STORE_TYPE": "inmemory",
                              "VECTOR_STORE_TYPE": "inmemory", "INGESTION_SCHEDULE_INTERVAL_SECONDS": "3600"})
    d.start("ingestion")
    try:
        d.wait_ready("ingestion")
        code, health = _http("GET", d.url("ingestion", "/health"))
        assert code == 200 and health["scheduler_running"] is True, health
    finally:
        p = d.procs["ingestion"]
        os.killpg(p.pid, signal.SIGTERM)
        p.wait(30)
