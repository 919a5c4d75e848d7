"""Run one service (uvicorn + consumer thread), the whole single-node pipeline, or the shared
infrastructure a one-process-per-service deployment needs.

    python -m copilot_for_consensus_amd.services.main node         # all services, in-proc bus
    python -m copilot_for_consensus_amd.services.main reporting    # one service per process
    python -m copilot_for_consensus_amd.services.main broker       # native message broker (RabbitMQ role)
    python -m copilot_for_consensus_amd.services.main docstore     # document store server (MongoDB role)
    python -m copilot_for_consensus_amd.services.main vectorstore  # HIP kNN behind Qdrant's REST API
    python -m copilot_for_consensus_amd.services.main llm          # HIP decoder behind llama.cpp / Ollama / OpenAI APIs
    python -m copilot_for_consensus_amd.services.main embedserver  # HIP encoder behind OpenAI / Ollama / TEI embeddings

Reference entry points: <service>/main.py (e.g. ingestion/main.py:179, parsing/main.py:101-124).

Multi-GPU: launched by torchrun (WORLD_SIZE > 1), ``node`` and ``summarization`` run one process
per GPU -- CFC_TP consecutive ranks form one tensor-parallel model, the TP-group leaders are the
data-parallel ranks (ORCHESTRATOR_DP / CFC_DP, if set, must equal WORLD_SIZE / CFC_TP).  Global
rank 0 runs the service(s); every DP rank embeds, indexes (its own HBM shard) and summarizes the
threads it owns, rank 0's services reaching them through the job's TCPStore (parallel/dp_node.py:
owner routing, streaming summaries, heartbeats, takeover of a dead rank's threads); TP followers
replay their leader's engine steps:

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m copilot_for_consensus_amd.services.main node
"""
from __future__ import annotations

import argparse
import os
import sys

# before torch loads (c10 reads it once): the DP control plane parks idle threads in blocking
# TCPStore waits that time out every WAIT_SLICE_S; c10d logs each timeout as a warning
os.environ.setdefault("TORCH_CPP_LOG_LEVEL", "ERROR")

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
                                        "summarization", "reporting", "auth", "broker", "docstore", "vectorstore",
                                        "llm", "embedserver"])
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--host", default=None)
    ap.add_argument("--data-dir", default=None, help="broker journal / docstore WAL / vector index directory")
    args = ap.parse_args(argv)

    if args.service in ("broker", "docstore", "vectorstore", "llm", "embedserver"):
        return _infra(args)

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
                          require_pkce=cfg.require_pkce, require_nonce=cfg.require_nonce,
                          max_session_seconds=cfg.max_session_seconds)
        uvicorn.run(create_auth_app(svc, cfg.cookie_secure), host=cfg.host, port=args.port or cfg.port)
        return 0

    from .base import create_app, run_service
    from .node import Node
    dist_ctx = None
    if args.service in ("node", "summarization"):
        dist_ctx = _distributed()
        if dist_ctx is not None and not dist_ctx["serve"]:
            return _model_rank(dist_ctx)
    try:
        only = None if args.service == "node" else [args.service]
        node = Node(services=only, summarizer=dist_ctx["summarizer"] if dist_ctx else None,
                    vector_store=dist_ctx["vector_store"] if dist_ctx else None,
                    embedding_provider=dist_ctx["embedder"] if dist_ctx else None)
        node.connect(only)
    except Exception as e:  # noqa: BLE001 -- fail fast: a service that cannot reach its bus/store exits 1
        print(f"[{args.service}] start-up failed: {type(e).__name__}: {e}", file=sys.stderr, flush=True)
        return 1
    if args.service == "node":
        import uvicorn
        node.start(threaded=True)
        try:
            uvicorn.run(node.http_app(), host="0.0.0.0", port=args.port or 8080)
        finally:
            node.stop()
            _close_distributed(dist_ctx)
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
        ui_routes(app, bases={"reporting": ""})       # its own API at the root; ingestion / auth via the gateway
    if args.service == "ingestion":
        node.start_scheduler()    # a standalone ingestion process schedules its own fetches (ingestion/main.py)
    try:
        run_service(svc, app, cfg.http_host, args.port or cfg.http_port)
    finally:
        if getattr(svc, "scheduler", None) is not None:
            svc.scheduler.stop()
        _close_distributed(dist_ctx)
    return 0


def _distributed() -> dict | None:
    """torchrun env -> process groups, this rank's models and its role (see the module doc)."""
    import os
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return None
    import torch.distributed as dist

    from ..embedding import create_embedding_provider
    from ..parallel import init_distributed, make_groups
    from ..parallel.dp_node import DPNodeWorker, build_rank0
    from ..parallel.dp_service import TPBroadcast
    from ..summarization import create_llm_backend
    from ..vectorstore import create_vector_store
    env = init_distributed()
    scfg = get_config("summarization")
    llm = scfg.llm_backend
    tp = int((llm.driver_config or {}).get("tensor_parallel") or 1) if llm.driver_name == "hip" else 1
    groups = make_groups(env, tp)
    want_dp = int(get_config("orchestrator").data_parallel or 1)
    if want_dp > 1 and want_dp != groups.dp_size:
        raise SystemExit(f"ORCHESTRATOR_DP={want_dp} but WORLD_SIZE / CFC_TP = {groups.dp_size}")
    over = dict(tensor_parallel=tp, tp_group=groups.tp_group, tp_rank=groups.tp_rank,
                device=str(env.device)) if llm.driver_name == "hip" else {}
    local = create_llm_backend(llm, **over)
    tp_bcast = None
    if tp > 1 and groups.tp_rank == 0:
        tp_bcast = local.tp_hook = TPBroadcast(groups)
    store = dist.distributed_c10d._get_default_store()
    serve = env.rank == 0
    ctx = {"env": env, "groups": groups, "store": store, "local": local, "summarizer": local, "serve": serve,
           "tp_bcast": tp_bcast, "worker": None, "vector_store": None, "embedder": None}
    if groups.dp_size > 1 and groups.tp_rank == 0:
        # every DP rank embeds, indexes and summarizes the threads it owns (parallel/dp_node.py)
        ecfg = get_config("embedding")
        embedder = create_embedding_provider(ecfg.embedding_backend)
        index = create_vector_store(ecfg.vector_store, dimension=int(embedder.dimension))
        worker = DPNodeWorker(store, groups.dp_rank, groups.dp_size, embedder, index, local,
                              continuous=dict(min_admit=int(scfg.min_admit), max_wait_s=scfg.admit_wait_ms / 1000.0))
        ctx.update(worker=worker, embedder=embedder)
        if serve:
            # a rank whose heartbeat is older than this is taken for dead and its threads move
            hb = float(os.environ.get("CFC_DP_HEARTBEAT_TIMEOUT", "10"))
            vs, summ = build_rank0(store, groups.dp_size, worker, heartbeat_timeout=hb)
            ctx.update(vector_store=vs, summarizer=summ)
            worker.start(serve=False)
    return ctx


def _model_rank(ctx: dict) -> int:
    """A rank that only runs models: TP follower, or DP worker (TP-group leader) until shutdown."""
    from ..parallel.dp_service import tp_follow
    g = ctx["groups"]
    if g.tp_rank != 0:
        n = tp_follow(ctx["local"], g)
        print(f"[rank {ctx['env'].rank}] TP follower done after {n} messages", flush=True)
        return 0
    stats = ctx["worker"].run_until_shutdown()
    if ctx["tp_bcast"] is not None:
        ctx["tp_bcast"].stop()
    ctx["worker_stats"] = stats
    print(f"[rank {ctx['env'].rank}] DP worker done: {stats}", flush=True)
    return 0


def _close_distributed(ctx: dict | None) -> None:
    if not ctx:
        return
    if ctx.get("worker") is not None and ctx["serve"]:
        from ..parallel.dp_node import shutdown_workers
        shutdown_workers(ctx["store"])      # DP workers leave their serve loops
        ctx["worker"].stop()
        if ctx.get("vector_store") is not None:
            ctx["vector_store"].close()     # the chunk-text server
    if ctx["tp_bcast"] is not None:
        ctx["tp_bcast"].stop()


def _infra(args) -> int:
    import os
    host = args.host or "0.0.0.0"
    if args.service == "broker":
        import subprocess

        from ..bus.cfcbroker import BROKER_BIN, DEFAULT_PORT
        if not BROKER_BIN.exists():
            from .._build import build_broker
            build_broker(verbose=False)
        cmd = [str(BROKER_BIN), "--host", host, "--port", str(args.port or int(os.environ.get("CFC_BROKER_PORT",
                                                                                               DEFAULT_PORT)))]
        data = args.data_dir or os.environ.get("CFC_BROKER_DATA_DIR")
        if data:
            cmd += ["--data-dir", data]
        cmd += ["--max-redeliveries", os.environ.get("CFC_BROKER_MAX_REDELIVERIES", "5"),
                "--fsync", os.environ.get("CFC_BROKER_FSYNC", "always")]
        proc = subprocess.Popen(cmd)   # a child, not an exec: the broker's exit code is ours
        try:
            return proc.wait()
        except KeyboardInterrupt:
            proc.terminate()
            return proc.wait()
    if args.service == "docstore":
        from ..storage.server import DocumentStoreServer
        srv = DocumentStoreServer(host=host, port=args.port or int(os.environ.get("CFC_DOCSTORE_PORT", 27027)),
                                  data_dir=args.data_dir or os.environ.get("CFC_DOCSTORE_DATA_DIR"),
                                  fsync=os.environ.get("CFC_DOCSTORE_FSYNC", "false").lower() == "true")
        print(f"cfc-docstore listening on {host}:{srv.port} (replayed {srv.replayed} log records)", flush=True)
        import signal
        import threading
        # serve_forever() returns once shutdown() runs (from another thread); close() then snapshots
        signal.signal(signal.SIGTERM, lambda *_: threading.Thread(target=srv.server.shutdown, daemon=True).start())
        try:
            srv.serve_forever()
        except KeyboardInterrupt:
            pass
        return 0
    import uvicorn

    from ..config.loader import load_adapter_config
    if args.service == "llm":
        from ..serving import build_from_config
        llm = load_adapter_config("llm_backend", driver="hip").driver_config     # LLM_* of the hip driver
        app, _ = build_from_config(llm)
        port = args.port or load_adapter_config("llm_backend", driver="llamacpp").driver_config.get("port") or 8081
        uvicorn.run(app, host=host, port=int(port), log_level="warning")
        return 0
    if args.service == "embedserver":
        from ..embedding import HipEncoderProvider
        from ..serving import create_embedding_app
        emb = load_adapter_config("embedding_backend", driver="hip").driver_config   # EMBEDDING_MODEL_NAME / _DEVICE
        app = create_embedding_app(HipEncoderProvider(**{k: v for k, v in emb.items() if v is not None}))
        uvicorn.run(app, host=host, port=args.port or 8082, log_level="warning")
        return 0
    from ..vectorstore.server import create_vector_app
    hip = load_adapter_config("vector_store", driver="hip").driver_config     # VECTOR_STORE_* of the hip driver
    port = args.port or load_adapter_config("vector_store", driver="qdrant").driver_config["port"]   # QDRANT_PORT
    app = create_vector_app(device=hip["device"], capacity=hip["capacity"], index_type=hip["index_type"],
                            nlist=hip["nlist"], nprobe=hip["nprobe"], persist_dir=args.data_dir or hip["persist_path"])
    uvicorn.run(app, host=host, port=port, log_level="warning")
    return 0


if __name__ == "__main__":
    sys.exit(main())
