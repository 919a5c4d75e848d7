"""Run one service (uvicorn + consumer thread) or the whole single-node pipeline.

    python -m copilot_for_consensus_amd.services.main node         # all services, in-proc bus
    python -m copilot_for_consensus_amd.services.main reporting    # one service per process

Reference entry points: <service>/main.py (e.g. ingestion/main.py:179, parsing/main.py:101-124).
"""
from __future__ import annotations

import argparse
import sys

from ..config.loader import get_config


def _auth_dep(cfg):
    if not cfg.service_settings.get("jwt_auth_enabled"):
        return None
    from ..security.auth import JWTMiddleware
    return JWTMiddleware(auth_service_url=cfg.auth_service_url, audience=cfg.service_audience,
                         required_roles=["admin"] if cfg.service_name == "ingestion" else
                         ["reader", "admin"] if cfg.service_name == "reporting" else ["processor", "admin"]).dependency()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("service", choices=["node", "ingestion", "parsing", "chunking", "embedding", "orchestrator",
                                        "summarization", "reporting", "auth"])
    ap.add_argument("--port", type=int, default=None)
    args = ap.parse_args(argv)

    if args.service == "auth":
        from ..security.auth import AuthService, MockIdentityProvider, RoleStore, github_provider, google_provider
        from ..security.auth import datatracker_provider, microsoft_provider
        from ..security.jwt import JWTManager, create_jwt_signer
        from ..storage.document_store import create_document_store
        from .auth import create_auth_app
        import uvicorn
        cfg = get_config("auth")
        store = create_document_store(cfg.document_store)
        provs = {"mock": MockIdentityProvider()} if cfg.enable_mock_provider else {}
        for name, fn in (("github", github_provider), ("google", google_provider), ("microsoft", microsoft_provider),
                         ("datatracker", datatracker_provider)):
            pc = cfg.oidc_providers.driver_config.get(name, {})
            if pc.get(f"{name}_client_id"):
                provs[name] = fn(**pc)
        svc = AuthService(JWTManager(create_jwt_signer(cfg.jwt_signer), issuer=cfg.issuer or "copilot-auth",
                                     audience=cfg.audiences, default_expiry=cfg.jwt_default_expiry),
                          RoleStore(store, cfg.role_store_collection,
                                    (cfg.auto_approve_roles or "").split(",") if cfg.auto_approve_enabled else [],
                                    cfg.first_user_auto_promotion_enabled), provs,
                          require_pkce=cfg.require_pkce, require_nonce=cfg.require_nonce)
        uvicorn.run(create_auth_app(svc, cfg.cookie_secure), host=cfg.host, port=args.port or cfg.port)
        return 0

    from .base import create_app, run_service
    from .node import Node
    try:
        node = Node()
        node.connect(None if args.service == "node" else [args.service])
    except Exception as e:  # noqa: BLE001 -- fail fast: a service that cannot reach its bus/store exits 1
        print(f"[{args.service}] start-up failed: {type(e).__name__}: {e}", file=sys.stderr, flush=True)
        return 1
    if args.service == "node":
        import uvicorn
        from .ingestion import ingestion_routes
        from .reporting import reporting_routes
        node.start(threaded=True)
        from ..ui import ui_routes
        app = create_app(node.services["reporting"], extra_routes=reporting_routes)
        ingestion_routes(app, node.services["ingestion"], None)
        ui_routes(app)
        uvicorn.run(app, host="0.0.0.0", port=args.port or 8080)
        node.stop()
        return 0
    svc = node.services[args.service]
    cfg = node.cfgs[args.service]
    extra = None
    if args.service == "reporting":
        from .reporting import reporting_routes as extra
    elif args.service == "ingestion":
        from .ingestion import ingestion_routes as extra
    app = create_app(svc, extra_routes=extra, auth_dependency=_auth_dep(cfg))
    if args.service == "reporting":
        from ..ui import ui_routes
        ui_routes(app)
    run_service(svc, app, cfg.http_host, args.port or cfg.http_port)
    return 0


if __name__ == "__main__":
    sys.exit(main())
