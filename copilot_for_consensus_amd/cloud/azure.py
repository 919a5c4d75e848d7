"""Azure-hosted drivers (the reference's Azure deployment: Service Bus, Cosmos DB, Blob Storage,
Key Vault, Azure Monitor).

Parity targets: copilot_message_bus azureservicebuspublisher.py:30 / azureservicebussubscriber.py:29
(topic or queue target, ``subject`` = routing key for subscription filters, complete on success,
abandon on handler error, dead-letter malformed JSON), copilot_storage azure_cosmos_document_store.py:35,
copilot_archive_store azure_blob_archive_store.py:33, copilot_secrets azurekeyvault_provider.py:16,
copilot_metrics azure_monitor_metrics.py, copilot_jwt_signer keyvault_signer.py:102.

None of the Azure SDKs is installed in this image: each class imports its SDK when constructed
and raises ImportError naming the package otherwise, so the factories can offer the drivers
without a hard dependency.  The GPU data plane never touches these.
"""
from __future__ import annotations

import base64
import hashlib
import json
import threading
from typing import Any, Callable

from ..bus.base import EventPublisher, EventSubscriber, topic_matches
from ..contracts.events import ROUTING_KEYS


def _need(mod: str, pkg: str):
    import importlib
    try:
        return importlib.import_module(mod)
    except ImportError as e:
        raise ImportError(f"this driver needs the '{pkg}' package, which is not installed") from e


def _credential(use_managed_identity: bool):
    if not use_managed_identity:
        return None
    return _need("azure.identity", "azure-identity").DefaultAzureCredential()


# ----------------------------------------------------------------------------- Service Bus

class AzureServiceBusPublisher(EventPublisher):
    def __init__(self, connection_string: str | None = None, fully_qualified_namespace: str | None = None,
                 topic_name: str | None = "copilot.events", queue_name: str | None = None,
                 use_managed_identity: bool = False, **_):
        sb = _need("azure.servicebus", "azure-servicebus")
        self._Message = sb.ServiceBusMessage
        if connection_string:
            self.client = sb.ServiceBusClient.from_connection_string(conn_str=connection_string)
        else:
            self.client = sb.ServiceBusClient(fully_qualified_namespace, _credential(True))
        self.topic, self.queue = topic_name, queue_name
        self._lock = threading.Lock()
        self._sender = None

    def connect(self) -> None:
        with self._lock:
            if self._sender is None:
                self._sender = (self.client.get_queue_sender(self.queue) if self.queue
                                else self.client.get_topic_sender(self.topic))

    def publish(self, exchange: str, routing_key: str, event: dict[str, Any]) -> None:
        self.connect()
        msg = self._Message(json.dumps(event), content_type="application/json", subject=routing_key)
        msg.application_properties = {"event_type": event.get("event_type", ""), "exchange": exchange,
                                      "routing_key": routing_key}
        with self._lock:
            self._sender.send_messages(msg)

    def disconnect(self) -> None:
        with self._lock:
            if self._sender is not None:
                self._sender.close()
                self._sender = None
        self.client.close()


class AzureServiceBusSubscriber(EventSubscriber):
    def __init__(self, connection_string: str | None = None, fully_qualified_namespace: str | None = None,
                 topic_name: str | None = "copilot.events", subscription_name: str | None = None,
                 queue_name: str | None = None, use_managed_identity: bool = False, max_wait_time: float = 5.0,
                 batch: int = 32, **_):
        sb = _need("azure.servicebus", "azure-servicebus")
        if connection_string:
            self.client = sb.ServiceBusClient.from_connection_string(conn_str=connection_string)
        else:
            self.client = sb.ServiceBusClient(fully_qualified_namespace, _credential(True))
        self.topic, self.sub, self.queue = topic_name, subscription_name, queue_name
        self.max_wait, self.batch = max_wait_time, batch
        self._handlers: list[tuple[str, str, Callable]] = []
        self._stop = threading.Event()

    def connect(self) -> None:
        pass

    def subscribe(self, event_type: str, callback, routing_key: str | None = None, exchange: str | None = None):
        self._handlers.append((event_type, routing_key or ROUTING_KEYS.get(event_type, event_type), callback))

    def _dispatch(self, event: dict, subject: str | None) -> bool:
        hit = False
        for et, rk, cb in self._handlers:
            if event.get("event_type") == et or (subject and topic_matches(rk, subject)):
                cb(event)
                hit = True
        return hit

    def start_consuming(self) -> None:
        recv = (self.client.get_queue_receiver(self.queue) if self.queue
                else self.client.get_subscription_receiver(self.topic, self.sub))
        with recv:
            while not self._stop.is_set():
                for msg in recv.receive_messages(max_message_count=self.batch, max_wait_time=self.max_wait):
                    try:
                        event = json.loads(str(msg))
                    except ValueError:
                        recv.dead_letter_message(msg, reason="malformed-json")
                        continue
                    try:
                        self._dispatch(event, getattr(msg, "subject", None))
                    except Exception:
                        recv.abandon_message(msg)      # redelivered; Service Bus dead-letters after max count
                        continue
                    recv.complete_message(msg)

    def stop_consuming(self) -> None:
        self._stop.set()

    def disconnect(self) -> None:
        self.client.close()


# ----------------------------------------------------------------------------- Cosmos DB

class AzureCosmosDocumentStore:
    """DocumentStore over Cosmos DB (NoSQL API); Mongo-style filters translated to a SQL subset."""

    def __init__(self, endpoint: str | None = None, key: str | None = None, database: str = "copilot",
                 use_managed_identity: bool = False, partition_key: str = "/id", **_):
        if not endpoint:
            raise ValueError("azure_cosmosdb document store: endpoint is required (COSMOS_ENDPOINT)")
        cosmos = _need("azure.cosmos", "azure-cosmos")
        self._cosmos = cosmos
        cred = key if key else _credential(True)
        self.client = cosmos.CosmosClient(endpoint, credential=cred)
        self.db = self.client.create_database_if_not_exists(database)
        self.pk = partition_key
        self._containers: dict[str, Any] = {}

    def _c(self, coll):
        c = self._containers.get(coll)
        if c is None:
            c = self._containers[coll] = self.db.create_container_if_not_exists(
                id=coll, partition_key=self._cosmos.PartitionKey(path=self.pk))
        return c

    @staticmethod
    def _to_cosmos(doc):
        d = dict(doc)
        d["id"] = str(d.get("_id") or d.get("id"))
        return d

    @staticmethod
    def _from_cosmos(doc):
        return {k: v for k, v in doc.items() if not k.startswith("_") or k == "_id"}

    @staticmethod
    def sql_filter(flt: dict, params: list) -> str:
        """Mongo filter -> Cosmos SQL WHERE clause (equality, $in, $ne, comparisons, $exists, $and/$or)."""
        ops = {"$gt": ">", "$gte": ">=", "$lt": "<", "$lte": "<=", "$ne": "!="}
        parts = []
        for k, v in flt.items():
            if k in ("$and", "$or"):
                sub = [f"({AzureCosmosDocumentStore.sql_filter(x, params)})" for x in v]
                parts.append(f" {'AND' if k == '$and' else 'OR'} ".join(sub) or "true")
                continue
            f = "c." + k if "." not in k else "c." + ".".join(k.split("."))
            conds = v if isinstance(v, dict) and v and all(x.startswith("$") for x in v) else {"$eq": v}
            for op, val in conds.items():
                name = f"@p{len(params)}"
                if op == "$eq":
                    params.append({"name": name, "value": val})
                    parts.append(f"{f} = {name}")
                elif op in ops:
                    params.append({"name": name, "value": val})
                    parts.append(f"{f} {ops[op]} {name}")
                elif op == "$in":
                    params.append({"name": name, "value": list(val)})
                    parts.append(f"ARRAY_CONTAINS({name}, {f})")
                elif op == "$nin":
                    params.append({"name": name, "value": list(val)})
                    parts.append(f"NOT ARRAY_CONTAINS({name}, {f})")
                elif op == "$exists":
                    parts.append(f"{'' if val else 'NOT '}IS_DEFINED({f})")
                else:
                    raise ValueError(f"operator {op} not supported on Cosmos")
        return " AND ".join(parts) or "true"

    def insert_document(self, collection, doc):
        d = self._to_cosmos(doc)
        self._c(collection).create_item(d)
        return d["id"]

    def get_document(self, collection, doc_id):
        try:
            return self._from_cosmos(self._c(collection).read_item(str(doc_id), partition_key=str(doc_id)))
        except self._cosmos.exceptions.CosmosResourceNotFoundError:
            return None

    def query_documents(self, collection, filter_dict=None, limit=100, sort_by=None, sort_order="desc", skip=0):
        params: list = []
        q = f"SELECT * FROM c WHERE {self.sql_filter(filter_dict or {}, params)}"
        if sort_by:
            q += f" ORDER BY c.{sort_by} {'DESC' if sort_order == 'desc' else 'ASC'}"
        q += f" OFFSET {int(skip)} LIMIT {int(limit)}"
        return [self._from_cosmos(x) for x in self._c(collection).query_items(
            q, parameters=params, enable_cross_partition_query=True)]

    def update_document(self, collection, doc_id, patch):
        from ..storage.query import apply_update
        cur = self._c(collection).read_item(str(doc_id), partition_key=str(doc_id))
        self._c(collection).replace_item(cur["id"], apply_update(cur, patch))

    def delete_document(self, collection, doc_id):
        self._c(collection).delete_item(str(doc_id), partition_key=str(doc_id))

    def count_documents(self, collection, filter_dict=None):
        params: list = []
        q = f"SELECT VALUE COUNT(1) FROM c WHERE {self.sql_filter(filter_dict or {}, params)}"
        return int(next(iter(self._c(collection).query_items(q, parameters=params,
                                                              enable_cross_partition_query=True)), 0))


# ----------------------------------------------------------------------------- Blob archive store

class AzureBlobArchiveStore:
    """Archives as blobs ``<source>/<archive_id>.mbox`` with metadata (id = sha256(content)[:16])."""

    def __init__(self, connection_string: str | None = None, account_url: str | None = None,
                 container_name: str = "raw-archives", use_managed_identity: bool = False, **_):
        blob = _need("azure.storage.blob", "azure-storage-blob")
        if connection_string:
            svc = blob.BlobServiceClient.from_connection_string(connection_string)
        else:
            svc = blob.BlobServiceClient(account_url, credential=_credential(True))
        self.container = svc.get_container_client(container_name)
        try:
            self.container.create_container()
        except Exception:  # already exists
            pass

    def store_archive(self, source_name: str, file_path: str, content: bytes) -> str:
        aid = hashlib.sha256(content).hexdigest()[:16]
        self.container.upload_blob(f"{source_name}/{aid}.mbox", content, overwrite=True,
                                   metadata={"archive_id": aid, "source_name": source_name,
                                             "original_path": base64.urlsafe_b64encode(file_path.encode()).decode(),
                                             "file_hash": hashlib.sha256(content).hexdigest()})
        return aid

    def _find(self, archive_id: str):
        for b in self.container.list_blobs(include=["metadata"]):
            if b.name.endswith(f"/{archive_id}.mbox"):
                return b
        return None

    def get_archive(self, archive_id: str) -> bytes | None:
        b = self._find(archive_id)
        return None if b is None else self.container.download_blob(b.name).readall()

    def get_archive_by_hash(self, content_hash: str) -> str | None:
        for b in self.container.list_blobs(include=["metadata"]):
            if (b.metadata or {}).get("file_hash") == content_hash:
                return (b.metadata or {}).get("archive_id")
        return None

    def archive_exists(self, archive_id: str) -> bool:
        return self._find(archive_id) is not None

    def delete_archive(self, archive_id: str) -> bool:
        b = self._find(archive_id)
        if b is None:
            return False
        self.container.delete_blob(b.name)
        return True

    def list_archives(self, source_name: str) -> list[dict]:
        return [dict(b.metadata or {}) for b in self.container.list_blobs(name_starts_with=f"{source_name}/",
                                                                          include=["metadata"])]


# ----------------------------------------------------------------------------- Key Vault

class AzureKeyVaultSecretProvider:
    def __init__(self, vault_url: str | None = None, vault_name: str | None = None, **_):
        vault_url = vault_url or (f"https://{vault_name}.vault.azure.net" if vault_name else None)
        if not vault_url:
            raise ValueError("azure_key_vault secret provider: vault_url (AZURE_KEY_VAULT_URI) or vault_name "
                             "(AZURE_KEY_VAULT_NAME) is required")
        sec = _need("azure.keyvault.secrets", "azure-keyvault-secrets")
        self.client = sec.SecretClient(vault_url=vault_url, credential=_credential(True))

    @staticmethod
    def _name(n: str) -> str:
        return n.replace("_", "-")    # Key Vault names allow [0-9a-zA-Z-]

    def get_secret(self, name: str) -> str:
        from ..security.secrets import SecretNotFoundError
        try:
            return self.client.get_secret(self._name(name)).value
        except Exception as e:
            raise SecretNotFoundError(name) from e

    def get_secret_bytes(self, name: str) -> bytes:
        return self.get_secret(name).encode()

    def secret_exists(self, name: str) -> bool:
        try:
            self.get_secret(name)
            return True
        except KeyError:
            return False


class KeyVaultJWTSigner:
    """RS256 signing with a Key Vault key (the private key never leaves the vault)."""

    algorithm = "RS256"

    def __init__(self, vault_url: str, key_name: str, key_id: str | None = None, **_):
        keys = _need("azure.keyvault.keys", "azure-keyvault-keys")
        crypto = _need("azure.keyvault.keys.crypto", "azure-keyvault-keys")
        cred = _credential(True)
        self.key = keys.KeyClient(vault_url=vault_url, credential=cred).get_key(key_name)
        self.crypto = crypto.CryptographyClient(self.key, credential=cred)
        self._alg = crypto.SignatureAlgorithm.rs256
        self.key_id = key_id or self.key.properties.version

    def sign(self, message: bytes) -> bytes:
        return self.crypto.sign(self._alg, hashlib.sha256(message).digest()).signature

    def verify(self, message: bytes, signature: bytes) -> bool:
        return bool(self.crypto.verify(self._alg, hashlib.sha256(message).digest(), signature).is_valid)

    def get_public_key_jwk(self) -> dict:
        from ..security.jwt import b64u
        k = self.key.key
        return {"kty": "RSA", "use": "sig", "alg": "RS256", "kid": self.key_id, "n": b64u(bytes(k.n)),
                "e": b64u(bytes(k.e))}

    def health_check(self) -> bool:
        return self.key is not None


# ----------------------------------------------------------------------------- Azure Monitor

class AzureMonitorMetricsCollector:
    """OpenTelemetry metrics exported to Azure Monitor (counters / histograms / observable gauges)."""

    def __init__(self, connection_string: str | None = None, namespace: str = "copilot", export_interval_ms: int = 60000,
                 **_):
        if not connection_string:
            raise ValueError("azure_monitor metrics: connection_string is required "
                             "(the Application Insights connection string, a secret)")
        otel = _need("opentelemetry.metrics", "opentelemetry-api")
        sdk = _need("opentelemetry.sdk.metrics", "opentelemetry-sdk")
        reader_mod = _need("opentelemetry.sdk.metrics.export", "opentelemetry-sdk")
        exp = _need("azure.monitor.opentelemetry.exporter", "azure-monitor-opentelemetry-exporter")
        reader = reader_mod.PeriodicExportingMetricReader(
            exp.AzureMonitorMetricExporter(connection_string=connection_string),
            export_interval_millis=export_interval_ms)
        self.provider = sdk.MeterProvider(metric_readers=[reader])
        self.meter = self.provider.get_meter(namespace)
        self._otel = otel
        self._counters: dict[str, Any] = {}
        self._hists: dict[str, Any] = {}
        self._gauges: dict[str, dict] = {}
        self._lock = threading.Lock()

    def increment(self, name, value=1.0, tags=None):
        with self._lock:
            c = self._counters.get(name) or self._counters.setdefault(name, self.meter.create_counter(name))
        c.add(value, attributes=tags or {})

    def observe(self, name, value, tags=None):
        with self._lock:
            h = self._hists.get(name) or self._hists.setdefault(name, self.meter.create_histogram(name))
        h.record(value, attributes=tags or {})

    def gauge(self, name, value, tags=None):
        key = tuple(sorted((tags or {}).items()))
        with self._lock:
            if name not in self._gauges:
                vals = self._gauges[name] = {}

                def cb(_opts, vals=vals):
                    return [self._otel.Observation(v, dict(k)) for k, v in list(vals.items())]

                self.meter.create_observable_gauge(name, callbacks=[cb])
            self._gauges[name][key] = value

    def push(self):
        self.provider.force_flush()

    def safe_push(self):
        try:
            self.push()
        except Exception:
            pass
