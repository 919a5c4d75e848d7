"""The web UI (ui/index.html) rendered by node against the live reporting + ingestion API.

The reference UI is a React app with vitest tests per route (ui/src/routes/*.test.tsx).  Here the
page's script runs in node with a minimal DOM stand-in and ``fetch`` going to a real uvicorn
server in front of a pipeline that has ingested and summarised the sample archive; each view
(ReportsList with filters / paging, ReportDetail, DiscussionsList, ThreadDetail, MessageDetail
with chunks, SourcesList, SourceForm) must render without a script error and show the data.
Skipped when node is not installed.
"""
from __future__ import annotations

import json
import os
import re
import shutil
import subprocess
import threading
import time

import pytest

NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")

HARNESS = r"""
const http = require("http");
const BASE = process.env.UI_BASE;
const store = {};
global.localStorage = {getItem: (k) => store[k] || null, setItem: (k, v) => { store[k] = v; }, removeItem: (k) => { delete store[k]; }};
const el = () => ({value: "", innerHTML: "", textContent: "", hidden: false, classList: {toggle() {}}, getAttribute: () => ""});
const nodes = {"#token": el(), "#view": el(), "#msg": el(), "#nav-admin": el()};
global.document = {querySelector: (s) => nodes[s] || el(), querySelectorAll: () => [], getElementById: () => el(), body: el()};
global.matchMedia = () => ({matches: false});
global.location = {hash: ""};
global.window = global;
global.addEventListener = () => {};
global.confirm = () => true;
global.fetch = (path, opts) => new Promise((resolve, reject) => {
  const u = new URL(path, BASE);
  const req = http.request(u, {method: (opts && opts.method) || "GET", headers: (opts && opts.headers) || {}}, (res) => {
    let body = ""; res.on("data", (c) => body += c);
    res.on("end", () => resolve({ok: res.statusCode < 400, status: res.statusCode, statusText: "", text: async () => body}));
  });
  req.on("error", reject);
  if (opts && opts.body) req.write(opts.body);
  req.end();
});
const SCRIPT = require("fs").readFileSync(process.env.UI_JS, "utf8");
require("vm").runInThisContext(SCRIPT.replace(/\nroute\(\);\s*$/, "\n"));   // page script as a global script
(async () => {
  const out = {};
  for (const h of JSON.parse(process.env.UI_ROUTES)) {
    location.hash = h;
    await route();
    out[h] = nodes["#view"].innerHTML;
    if (h === "#/reports") out["nav_admin_hidden"] = nodes["#nav-admin"].hidden;
  }
  process.stdout.write(JSON.stringify(out));
})().catch((e) => { console.error("UI error", e); process.exit(2); });
"""


@pytest.fixture(scope="module")
def live(tmp_path_factory):
    import uvicorn

    from copilot_for_consensus_amd.embedding import HipEncoderProvider
    from copilot_for_consensus_amd.services.node import Node
    from copilot_for_consensus_amd.summarization import MockSummarizer
    from copilot_for_consensus_amd.vectorstore import HipFlatIndex
    tmp = tmp_path_factory.mktemp("ui")
    env = {"DOCUMENT_STORE_TYPE": "inmemory", "MESSAGE_BUS_TYPE": "inproc", "METRICS_TYPE": "noop",
           "LOG_TYPE": "silent", "ERROR_REPORTER_TYPE": "silent", "EMBEDDING_BACKEND_TYPE": "mock",
           "VECTOR_STORE_TYPE": "inmemory", "LLM_BACKEND_TYPE": "mock", "ARCHIVE_STORE_TYPE": "inmemory",
           "SECRET_PROVIDER_TYPE": "env"}
    emb = HipEncoderProvider(model_name="tiny", device="cpu")
    node = Node(env=env, embedding_provider=emb, vector_store=HipFlatIndex(emb.dimension, device="cpu"),
                summarizer=MockSummarizer(mock_latency_ms=0))
    node.start(threaded=False)
    src = tmp / "src"
    src.mkdir()
    shutil.copy(os.path.join(os.path.dirname(__file__), "fixtures", "sample.mbox"), src / "list.mbox")
    ing = node.services["ingestion"]
    ing.create_source({"name": "wg", "source_type": "local", "url": str(src)})
    ing.trigger_ingestion("wg")
    node.drain()
    app = node.http_app()                      # /reporting, /ingestion, /ui: the gateway layout
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=0, log_level="error"))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    while not server.started:
        time.sleep(0.02)
    port = server.servers[0].sockets[0].getsockname()[1]
    yield f"http://127.0.0.1:{port}", node
    server.should_exit = True
    th.join(5)


def _render(base, hashes, tmp_path):
    import urllib.request
    html = urllib.request.urlopen(base + "/ui", timeout=30).read().decode()      # the page as served
    js = "\n".join(re.findall(r"<script>(.*?)</script>", html, re.S))
    if subprocess.run([NODE, "-e", "null ?? 1"], capture_output=True).returncode != 0:
        js = js.replace("??", "||")            # old node: same result for the values the page handles
    (tmp_path / "ui.js").write_text(js)
    (tmp_path / "harness.js").write_text(HARNESS)
    env = dict(os.environ, UI_BASE=base, UI_JS=str(tmp_path / "ui.js"), UI_ROUTES=json.dumps(hashes))
    r = subprocess.run([NODE, str(tmp_path / "harness.js")], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout)


def test_views_render_live_data(live, tmp_path):
    base, node = live
    store = node.store
    rep = store.query_documents("summaries", {}, limit=10)
    thread = store.query_documents("threads", {}, limit=10)[0]
    msg = store.query_documents("messages", {"thread_id": thread["_id"]}, limit=1)[0]
    hashes = ["#/reports", "#/reports?source=wg&sort_by=generated_at&sort_order=asc&limit=10",
              "#/reports?min_messages=99", f"#/report/{rep[0]['_id']}", "#/threads",
              "#/threads?sort_by=last_message_date&limit=10", f"#/thread/{thread['_id']}", f"#/message/{msg['_id']}",
              "#/sources", "#/source/wg", "#/source/", "#/reports?topic=consensus", f"#/summary/{rep[0]['thread_id']}"]
    out = _render(base, hashes + ["#/admin"], tmp_path)
    # AccessDenied: nobody is signed in, so the admin view is refused and its nav link hidden
    assert "Access denied" in out["#/admin"] and out["nav_admin_hidden"] is True
    assert rep[0]["thread_id"] in out[f"#/summary/{rep[0]['thread_id']}"]
    assert all('class="err"' not in out[h] for h in hashes), {h: out[h][:300] for h in hashes if 'class="err"' in out[h]}
    assert rep[0]["_id"] in out["#/reports"] and "thread start" in out["#/reports"]
    assert "No reports match" in out["#/reports?min_messages=99"]
    assert '<option selected>wg</option>' in out["#/reports?source=wg&sort_by=generated_at&sort_order=asc&limit=10"]
    assert "Citations" in out[f"#/report/{rep[0]['_id']}"]
    assert thread["subject"][:20] in out["#/threads"] or thread["_id"] in out["#/threads"]
    assert "Chunks (" in out[f"#/message/{msg['_id']}"] and "embedded" in out[f"#/message/{msg['_id']}"]
    assert "wg" in out["#/sources"] and "Source wg" in out["#/source/wg"]
    assert "New source" in out["#/source/"] and 'name="password"' in out["#/source/"]
    assert "<th>Score</th>" in out["#/reports?topic=consensus"]


def test_source_form_validation_matches_reference_rules(tmp_path):
    """sourceErrors() mirrors SourceForm.tsx validate(): name / type / url always, port (1..65535),
    username and password when the type is imap."""
    import pathlib
    html = (pathlib.Path(__file__).parents[1] / "copilot_for_consensus_amd" / "ui" / "index.html").read_text()
    js = "\n".join(re.findall(r"<script>(.*?)</script>", html, re.S))
    m = re.search(r"function sourceErrors\(b\) \{.*?\n\}", js, re.S)
    assert m, "sourceErrors not found in the page script"
    cases = [{"name": "a", "source_type": "local", "url": "/x"},
             {"name": "", "source_type": "local", "url": ""},
             {"name": "a", "source_type": "imap", "url": "imap.example.org"},
             {"name": "a", "source_type": "imap", "url": "h", "port": 70000, "username": "u", "password": "p"},
             {"name": "a", "source_type": "imap", "url": "h", "port": 993, "username": "u", "password": "p"}]
    prog = m.group(0) + f"\nprocess.stdout.write(JSON.stringify({json.dumps(cases)}.map(sourceErrors)));"
    (tmp_path / "v.js").write_text(prog)
    r = subprocess.run([NODE, str(tmp_path / "v.js")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    assert out[0] == [] and out[4] == []
    assert out[1] == ["Name is required", "URL is required"]
    assert out[2] == ["Port is required for IMAP sources", "Username is required for IMAP sources",
                      "Password is required for IMAP sources"]
    assert out[3] == ["Port must be between 1 and 65535"]
