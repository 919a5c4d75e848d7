"""API gateway artefacts generated from the services themselves.

Parity target: scripts/generate_service_openapi.py, openapi/gateway.yaml, infra/nginx/nginx.conf
(path-prefix proxy :155-267) and infra/gateway/generate_gateway_config.py of the reference.
Instead of a hand-maintained spec, every service's FastAPI app is instantiated (mock adapters, no
GPU) and its ``openapi()`` taken as the source of truth; the gateway spec prefixes each service's
paths (``/ingestion``, ``/reporting``, ``/auth``, ...) and an nginx config with one upstream per
service is rendered from the same route table, so the three cannot drift apart.

    python -m copilot_for_consensus_amd.tools.gateway --out deploy/gateway

Reference: infra/gateway/generate_gateway_config.py:34-119 (per-provider adapters),
infra/nginx/nginx.conf:155-267 (path-prefix proxy), openapi/gateway.yaml.
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


# ---------------------------------------------------------------------------- cloud gateways
# Parity: infra/gateway/{aws,azure,gcp}_adapter.py of the reference (CloudFormation/SAM, APIM
# ARM + policies, Cloud Endpoints/API Gateway).  All three are rendered from the same gateway spec.
_METHODS = ("get", "put", "post", "delete", "patch", "head", "options")
_PUBLIC = ("/health", "/readyz", "/providers", "/login", "/callback", "/keys", "/.well-known/jwks.json")


def _service_of(path: str) -> tuple[str, str]:
    for name, (prefix, hp) in SERVICES.items():
        if path == prefix or path.startswith(prefix + "/"):
            return name, hp
    raise KeyError(path)


def _backend(path: str, base_url: str | None) -> str:
    name, hp = _service_of(path)
    prefix = SERVICES[name][0]
    root = (base_url.rstrip("/") + prefix) if base_url else f"http://{hp}"
    return root + path[len(prefix):]


def _ops(spec: dict):
    for p, item in spec.get("paths", {}).items():
        for m, op in item.items():
            if m in _METHODS:
                yield p, m, op


def aws_openapi(spec: dict, base_url: str | None = None) -> dict:
    """Gateway spec + ``x-amazon-apigateway-integration`` (HTTP proxy) on every operation."""
    out = json.loads(json.dumps(spec))
    for p, m, op in _ops(out):
        params = {f"integration.request.path.{x['name']}": f"method.request.path.{x['name']}"
                  for x in op.get("parameters", []) if x.get("in") == "path"}
        op["x-amazon-apigateway-integration"] = {
            "type": "http_proxy", "httpMethod": m.upper(), "uri": _backend(p, base_url),
            "passthroughBehavior": "when_no_match", "timeoutInMillis": 29000,
            **({"requestParameters": params} if params else {})}
    out["x-amazon-apigateway-binary-media-types"] = ["application/zip", "application/gzip", "application/octet-stream"]
    return out


def aws_cloudformation(spec: dict, base_url: str | None = None, stage: str = "prod") -> dict:
    return {
        "AWSTemplateFormatVersion": "2010-09-09",
        "Description": "Copilot-for-Consensus API gateway (generated from the services' OpenAPI)",
        "Parameters": {"StageName": {"Type": "String", "Default": stage}},
        "Resources": {
            "Api": {"Type": "AWS::ApiGateway::RestApi",
                    "Properties": {"Name": "copilot-for-consensus", "Body": aws_openapi(spec, base_url),
                                   "EndpointConfiguration": {"Types": ["REGIONAL"]}}},
            "Deployment": {"Type": "AWS::ApiGateway::Deployment", "DependsOn": ["Api"],
                           "Properties": {"RestApiId": {"Ref": "Api"}, "StageName": {"Ref": "StageName"}}},
        },
        "Outputs": {"Endpoint": {"Value": {"Fn::Sub": "https://${Api}.execute-api.${AWS::Region}.amazonaws.com/"
                                                      "${StageName}"}}},
    }


def azure_apim_template(spec: dict, base_url: str | None = None, jwks_url: str = "http://auth:8090/keys",
                        audience: str = "copilot-for-consensus", rate_per_minute: int = 600) -> dict:
    """ARM template: one APIM API imported from the gateway spec + a CORS / rate-limit / JWT policy."""
    policy = ("<policies><inbound><base/><cors allow-credentials=\"false\"><allowed-origins><origin>*</origin>"
              "</allowed-origins><allowed-methods><method>*</method></allowed-methods><allowed-headers>"
              "<header>*</header></allowed-headers></cors>"
              f"<rate-limit calls=\"{rate_per_minute}\" renewal-period=\"60\"/>"
              "<choose><when condition=\"@(!context.Request.Url.Path.EndsWith(&quot;/health&quot;))\">"
              f"<validate-jwt header-name=\"Authorization\" failed-validation-httpcode=\"401\">"
              f"<openid-config url=\"{jwks_url}\"/><audiences><audience>{audience}</audience></audiences>"
              "</validate-jwt></when></choose></inbound><backend><base/></backend><outbound><base/></outbound>"
              "</policies>")
    api = "copilot-for-consensus"
    return {
        "$schema": "https://schema.management.azure.com/schemas/2019-04-01/deploymentTemplate.json#",
        "contentVersion": "1.0.0.0",
        "parameters": {"apimServiceName": {"type": "string"},
                       "backendUrl": {"type": "string", "defaultValue": base_url or "http://gateway:8080"}},
        "resources": [
            {"type": "Microsoft.ApiManagement/service/apis", "apiVersion": "2022-08-01",
             "name": f"[concat(parameters('apimServiceName'), '/{api}')]",
             "properties": {"displayName": "Copilot-for-Consensus", "path": "", "protocols": ["https"],
                            "serviceUrl": "[parameters('backendUrl')]", "format": "openapi+json",
                            "value": json.dumps(spec)}},
            {"type": "Microsoft.ApiManagement/service/apis/policies", "apiVersion": "2022-08-01",
             "name": f"[concat(parameters('apimServiceName'), '/{api}/policy')]",
             "dependsOn": [f"[resourceId('Microsoft.ApiManagement/service/apis', parameters('apimServiceName'), "
                           f"'{api}')]"],
             "properties": {"format": "rawxml", "value": policy}},
        ],
    }


def gcp_api_config(spec: dict, base_url: str | None = None, issuer: str = "copilot-auth",
                   jwks_url: str = "http://auth:8090/keys", audience: str = "copilot-for-consensus") -> dict:
    """API Gateway / Cloud Endpoints config: ``x-google-backend`` per operation, JWT auth via the
    auth service's JWKS except on the public routes."""
    out = json.loads(json.dumps(spec))
    out.setdefault("components", {})["securitySchemes"] = {"copilot_jwt": {
        "type": "oauth2", "flows": {"implicit": {"authorizationUrl": "", "scopes": {}}},
        "x-google-issuer": issuer, "x-google-jwks_uri": jwks_url, "x-google-audiences": audience}}
    for p, m, op in _ops(out):
        op["x-google-backend"] = {"address": _backend(p, base_url), "path_translation": "APPEND_PATH_TO_ADDRESS"
                                  if "{" in p else "CONSTANT_ADDRESS", "deadline": 300.0}
        if not p.endswith(_PUBLIC):
            op["security"] = [{"copilot_jwt": []}]
    out["x-google-management"] = {"metrics": [], "quota": {}}
    return out


def validate_cloud_config(spec: dict, provider: str, cfg: dict) -> list[str]:
    """Every gateway operation must be routed by the generated config."""
    errs = []
    if provider == "aws":
        body = cfg["Resources"]["Api"]["Properties"]["Body"]
        errs = [f"{m.upper()} {p}" for p, m, op in _ops(body) if "x-amazon-apigateway-integration" not in op]
    elif provider == "gcp":
        errs = [f"{m.upper()} {p}" for p, m, op in _ops(cfg) if "x-google-backend" not in op]
    elif provider == "azure":
        imported = json.loads(cfg["resources"][0]["properties"]["value"])
        errs = [f"{m.upper()} {p}" for p, m, _ in _ops(spec) if p not in imported.get("paths", {})]
    return errs


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Generate per-service OpenAPI, gateway spec, nginx and cloud gateway configs")
    ap.add_argument("--out", default="deploy/gateway")
    ap.add_argument("--provider", choices=["nginx", "aws", "azure", "gcp", "all"], default="all")
    ap.add_argument("--backend-url", default=None, help="public base URL of the services (default: compose hosts)")
    a = ap.parse_args(argv)
    out = Path(a.out)
    (out / "services").mkdir(parents=True, exist_ok=True)
    specs = service_openapi()
    for n, s in specs.items():
        (out / "services" / f"{n}.json").write_text(json.dumps(s, indent=2) + "\n", encoding="utf-8")
    (out / "gateway.openapi.json").write_text(json.dumps(gateway_openapi(specs), indent=2) + "\n", encoding="utf-8")
    gw = gateway_openapi(specs)
    if a.provider in ("nginx", "all"):
        (out / "nginx.conf").write_text(nginx_conf(), encoding="utf-8")
    rendered = {}
    if a.provider in ("aws", "all"):
        rendered["aws"] = ("aws/cloudformation.json", aws_cloudformation(gw, a.backend_url))
    if a.provider in ("azure", "all"):
        rendered["azure"] = ("azure/apim.json", azure_apim_template(gw, a.backend_url))
    if a.provider in ("gcp", "all"):
        rendered["gcp"] = ("gcp/api_config.json", gcp_api_config(gw, a.backend_url))
    for prov, (rel, cfg) in rendered.items():
        errs = validate_cloud_config(gw, prov, cfg)
        if errs:
            print(f"{prov}: {len(errs)} unrouted operations, e.g. {errs[:3]}", file=sys.stderr)
            return 1
        (out / rel).parent.mkdir(parents=True, exist_ok=True)
        (out / rel).write_text(json.dumps(cfg, indent=2) + "\n", encoding="utf-8")
    print(f"wrote {len(specs)} service specs, the gateway spec and {a.provider} gateway config(s) to {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
