"""Cloud drivers with stand-in SDK modules (the Azure / Sentry SDKs are not installed): the
drivers' call patterns against the SDK surface, the Cosmos filter translation, the
DocumentStore-backed archive store, and ES256 JWTs (RFC 6979 test vector)."""
import json
import sys
import types

import pytest

from copilot_for_consensus_amd.archive import create_archive_store
from copilot_for_consensus_amd.cloud.azure import AzureCosmosDocumentStore
from copilot_for_consensus_amd.security.jwt import ECKey, ECSigner, JWTError, create_jwt_signer, decode, encode


def _fake_servicebus(monkeypatch, inbox):
    sb = types.ModuleType("azure.servicebus")

    class Msg:
        def __init__(self, body, content_type=None, subject=None):
            self.body, self.content_type, self.subject = body, content_type, subject
            self.application_properties = {}

        def __str__(self):
            return self.body

    class Sender:
        def send_messages(self, m):
            inbox.append(m)

        def close(self):
            pass

    class Receiver:
        def __init__(self):
            self.done, self.abandoned, self.dead = [], [], []
            self.owner = None

        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

        def receive_messages(self, max_message_count, max_wait_time):
            out = list(inbox)
            inbox.clear()
            if not out:
                self.owner.stop_consuming()
            return out

        def complete_message(self, m):
            self.done.append(m)

        def abandon_message(self, m):
            self.abandoned.append(m)

        def dead_letter_message(self, m, reason=None):
            self.dead.append(m)

    class Client:
        receiver = Receiver()

        @classmethod
        def from_connection_string(cls, conn_str):
            return cls()

        def get_topic_sender(self, topic):
            return Sender()

        def get_subscription_receiver(self, topic, sub):
            return Client.receiver

        def close(self):
            pass

    sb.ServiceBusClient, sb.ServiceBusMessage = Client, Msg
    azure = sys.modules.get("azure") or types.ModuleType("azure")
    monkeypatch.setitem(sys.modules, "azure", azure)
    monkeypatch.setitem(sys.modules, "azure.servicebus", sb)
    return Client, Msg


def test_azure_service_bus_publish_consume(monkeypatch):
    inbox = []
    Client, Msg = _fake_servicebus(monkeypatch, inbox)
    from copilot_for_consensus_amd.cloud.azure import AzureServiceBusPublisher, AzureServiceBusSubscriber
    pub = AzureServiceBusPublisher(connection_string="Endpoint=sb://x/")
    pub.publish("copilot.events", "json.parsed", {"event_type": "JSONParsed", "data": {}})
    assert inbox[0].subject == "json.parsed" and inbox[0].application_properties["event_type"] == "JSONParsed"
    inbox.append(Msg("not json"))
    inbox.append(Msg(json.dumps({"event_type": "ChunksPrepared"}), subject="chunks.prepared"))
    sub = AzureServiceBusSubscriber(connection_string="Endpoint=sb://x/", subscription_name="s")
    Client.receiver.owner = sub
    got = []
    sub.subscribe("JSONParsed", got.append)

    def boom(e):
        raise RuntimeError("handler failure")

    sub.subscribe("ChunksPrepared", boom)
    sub.start_consuming()
    assert [e["event_type"] for e in got] == ["JSONParsed"]
    r = Client.receiver
    assert len(r.done) == 1 and len(r.dead) == 1 and len(r.abandoned) == 1


def test_missing_sdk_raises_clear_import_error():
    from copilot_for_consensus_amd.cloud.azure import AzureBlobArchiveStore
    with pytest.raises(ImportError, match="azure-storage-blob"):
        AzureBlobArchiveStore(connection_string="x")


def test_cosmos_sql_translation():
    p = []
    w = AzureCosmosDocumentStore.sql_filter({"status": {"$in": ["pending", "processing"]}, "attemptCount": {"$lt": 3},
                                             "$or": [{"a": 1}, {"b": {"$exists": False}}]}, p)
    assert w == ("ARRAY_CONTAINS(@p0, c.status) AND c.attemptCount < @p1 AND "
                 "(c.a = @p2) OR (NOT IS_DEFINED(c.b))")
    assert [x["value"] for x in p] == [["pending", "processing"], 3, 1]


def test_document_store_archive_store():
    st = create_archive_store("document_store")
    aid = st.store_archive("list", "/x/a.mbox", b"From a\n\nbody\n")
    assert st.store_archive("list", "/x/a.mbox", b"From a\n\nbody\n") == aid and len(aid) == 16
    assert st.get_archive(aid) == b"From a\n\nbody\n" and st.archive_exists(aid)
    assert st.get_archive_by_hash(st.list_archives("list")[0]["file_hash"]) == aid
    assert st.delete_archive(aid) and not st.archive_exists(aid)


def test_es256_rfc6979_vector_and_jwks():
    d = 0xC9AFA9D845BA75166B5C215767B1D6934E50C3DB36E89B127B8A622B120F6721
    k = ECKey(0x60FED4BA255A9D31C961EB74C6356D68C049B8923B61FA6CE669622E60F29FB6,
              0x7903FE1008B8BC99A41AE9E95628BC64F2F1B20C2D7E9F5177A3C294D4462299, d)
    sig = k.sign(b"sample")
    assert sig.hex().upper() == ("EFD48B2AACB6A8FD1140DD9CD45E81D69D2C877B56AAF991C34D0EA84EAF3716"
                                 "F7CB1C942D657C41D436C7A1B6E29F65F3E900DBB9AFF4064DC4AB2F843ACDA8")
    assert k.verify(b"sample", sig) and not k.verify(b"sample!", sig)
    s = create_jwt_signer(algorithm="ES256", key_id="k1")
    assert isinstance(s, ECSigner)
    tok = encode({"sub": "u", "aud": "svc"}, s)
    assert decode(tok, {"keys": [s.get_public_key_jwk()]}, audience="svc")["sub"] == "u"
    other = ECSigner(key_id="k1")
    with pytest.raises(JWTError):
        decode(tok, {"keys": [other.get_public_key_jwk()]})
    again = ECSigner(s.key.private_json(), key_id="k1")
    assert again.verify(b"m", s.sign(b"m"))


def test_sentry_reporter_with_fake_sdk(monkeypatch):
    calls = []
    sdk = types.ModuleType("sentry_sdk")
    sdk.init = lambda **kw: calls.append(("init", kw["dsn"]))

    class Scope:
        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

        def set_extra(self, k, v):
            calls.append(("extra", k))

    sdk.push_scope = Scope
    sdk.capture_exception = lambda e: calls.append(("exc", type(e).__name__))
    monkeypatch.setitem(sys.modules, "sentry_sdk", sdk)
    from copilot_for_consensus_amd.observability import create_error_reporter
    r = create_error_reporter("sentry", dsn="https://k@o.ingest/1")
    r.report(ValueError("x"), {"doc": "1"})
    assert calls == [("init", "https://k@o.ingest/1"), ("extra", "doc"), ("exc", "ValueError")]
