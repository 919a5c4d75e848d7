"""API gateway artefacts generated from the services themselves.

Parity target: scripts/generate_service_openapi.py, openapi/gateway.yaml, infra/nginx/nginx.conf
(path-prefix proxy :155-267) and infra/gateway/generate_gateway_config.py of the reference.
Instead of a hand-maintained spec, every service's FastAPI app is instantiated (mock adapters, no
GPU) and its ``openapi()`` taken as the source of truth; the gateway spec prefixes each service's
paths (``/ingestion``, ``/reporting``, ``/auth``, ...) and an nginx config with one upstream per
service is rendered from the same route table, so the three cannot drift apart.

    python -m copilot_for_consensus_amd.tools.gateway --out deploy/gateway
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

# service -> (gateway prefix, default upstream host:port)
SERVICES = {
    "ingestion": ("/ingestion", "ingestion:8080"),
    "parsing": ("/parsing", "parsing:8080"),
    "chunking": ("/chunking", "chunking:8080"),
    "embedding": ("/embedding", "embedding:8080"),
    "orchestrator": ("/orchestrator", "orchestrator:8080"),
    "summarization": ("/summarization", "summarization:8080"),
    "reporting": ("/reporting", "reporting:8080"),
    "auth": ("/auth", "auth:8090"),
}

_MOCK_ENV = {"DOCUMENT_STORE_TYPE": "inmemory", "MESSAGE_BUS_TYPE": "inproc", "METRICS_TYPE": "noop",
             "LOG_TYPE": "silent", "ERROR_REPORTER_TYPE": "silent", "EMBEDDING_BACKEND_TYPE": "mock",
             "VECTOR_STORE_TYPE": "inmemory", "LLM_BACKEND_TYPE": "mock", "ARCHIVE_STORE_TYPE": "inmemory",
             "SECRET_PROVIDER_TYPE": "env"}


def service_apps() -> dict:
    from ..security.auth import AuthService, MockIdentityProvider, RoleStore
    from ..security.jwt import HMACSigner, JWTManager
    from ..storage.document_store import InMemoryDocumentStore
    from .. import services as _s  # noqa: F401
    from ..services.auth import create_auth_app
    from ..services.base import create_app
    from ..services.ingestion import ingestion_routes
    from ..services.node import Node
    from ..services.reporting import reporting_routes

    node = Node(env=_MOCK_ENV)
    apps = {}
    for name in SERVICES:
        if name == "auth":
            store = InMemoryDocumentStore()
            svc = AuthService(JWTManager(HMACSigner("openapi-generation")), RoleStore(store),
                              {"mock": MockIdentityProvider()})
            apps[name] = create_auth_app(svc)
            continue
        extra = {"ingestion": ingestion_routes, "reporting": reporting_routes}.get(name)
        apps[name] = create_app(node.services[name], extra_routes=extra)
    return apps


def service_openapi() -> dict[str, dict]:
    return {name: app.openapi() for name, app in service_apps().items()}


def gateway_openapi(specs: dict[str, dict] | None = None, version: str = "1.0.0") -> dict:
    specs = specs or service_openapi()
    paths, schemas = {}, {}
    for name, spec in specs.items():
        prefix = SERVICES[name][0]
        for p, item in spec.get("paths", {}).items():
            tagged = {}
            for method, op in item.items():
                op = dict(op)
                op["tags"] = [name]
                op["operationId"] = f"{name}_{op.get('operationId', method + p.replace('/', '_'))}"
                tagged[method] = op
            paths[prefix + p] = tagged
        for k, v in spec.get("components", {}).get("schemas", {}).items():
            schemas.setdefault(k, v)
    return {"openapi": "3.1.0",
            "info": {"title": "Copilot-for-Consensus gateway (MI355X build)", "version": version},
            "paths": dict(sorted(paths.items())),
            "components": {"schemas": schemas}}


def nginx_conf(upstreams: dict[str, str] | None = None, listen: int = 8080, max_body_mb: int = 100) -> str:
    ups = {n: (upstreams or {}).get(n, hp) for n, (_, hp) in SERVICES.items()}
    lines = ["worker_processes auto;", "events { worker_connections 1024; }", "http {",
             f"  client_max_body_size {max_body_mb}m;", "  proxy_read_timeout 300s;"]
    for n, hp in ups.items():
        lines.append(f"  upstream {n}_svc {{ server {hp}; }}")
    lines += ["  server {", f"    listen {listen};", "    location = /health { return 200 'ok'; }"]
    for n, (prefix, _) in SERVICES.items():
        lines += [f"    location {prefix}/ {{",
                  f"      proxy_pass http://{n}_svc/;",
                  "      proxy_set_header Host $host;",
                  "      proxy_set_header X-Forwarded-For $proxy_add_x_forwarded_for;",
                  "      proxy_set_header X-Forwarded-Prefix " + prefix + ";",
                  "      proxy_set_header Authorization $http_authorization;",
                  "    }"]
    lines += ["  }", "}"]
    return "\n".join(lines) + "\n"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Generate per-service OpenAPI, gateway spec and nginx config")
    ap.add_argument("--out", default="deploy/gateway")
    a = ap.parse_args(argv)
    out = Path(a.out)
    (out / "services").mkdir(parents=True, exist_ok=True)
    specs = service_openapi()
    for n, s in specs.items():
        (out / "services" / f"{n}.json").write_text(json.dumps(s, indent=2) + "\n", encoding="utf-8")
    (out / "gateway.openapi.json").write_text(json.dumps(gateway_openapi(specs), indent=2) + "\n", encoding="utf-8")
    (out / "nginx.conf").write_text(nginx_conf(), encoding="utf-8")
    print(f"wrote {len(specs)} service specs, gateway spec and nginx.conf to {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
