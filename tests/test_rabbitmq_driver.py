"""The RabbitMQ bus driver (bus/rabbitmq.py) against a stand-in pika SDK (tests/fake_pika.py).

pika is not in this image, so the driver runs against an in-memory AMQP broker with RabbitMQ's
semantics.  Checks the reference driver's observable behaviour (rabbitmq_publisher.py:334-424,
rabbitmq_subscriber.py:376-610): mandatory publishes fail loudly when unroutable, broker nacks
propagate, declared queues survive a reconnect, handler failures requeue, malformed envelopes are
dropped, the consume loop and the publisher reconnect by themselves after the broker drops every
connection, and the reconnect circuit breaker throttles and gives up.
"""
from __future__ import annotations

import json
import threading
import time

import pytest

from copilot_for_consensus_amd.bus import create_publisher, create_subscriber
from copilot_for_consensus_amd.contracts.events import EXCHANGE, Event

import fake_pika


@pytest.fixture
def broker(monkeypatch):
    return fake_pika.install(monkeypatch)


class _Cfg:
    driver_name = "rabbitmq"

    def __init__(self, **kw):
        self.driver_config = {"rabbitmq_host": "127.0.0.1", "rabbitmq_port": 5672, "reconnect_delay": 0.01, **kw}


def _ev(event_type="ArchiveIngested", **over):
    data = dict(archive_id="a" * 16, source_name="s", source_type="local", source_url="file:///x",
                file_size_bytes=1, file_hash_sha256="0" * 64, ingestion_started_at="2025-01-01T00:00:00Z",
                ingestion_completed_at="2025-01-01T00:00:01Z")
    data.update(over)
    return Event.create(event_type, **data).to_dict()


def _wait(pred, timeout=10.0):
    end = time.time() + timeout
    while not pred() and time.time() < end:
        time.sleep(0.01)
    return pred()


def _consume(sub):
    t = threading.Thread(target=sub.start_consuming, daemon=True)
    t.start()
    return t


def test_unroutable_and_nack_fail_loudly(broker):
    pub = create_publisher(_Cfg(), enable_validation=False)
    pub.connect()
    with pytest.raises(fake_pika.exceptions.UnroutableError):
        pub.publish(EXCHANGE, "archive.ingested", _ev())       # no queue bound: not silently dropped
    pub.declare_queue("parsing", "archive.ingested")
    pub.publish(EXCHANGE, "archive.ingested", _ev())
    assert broker.depth("parsing") == 1
    broker.nack_next = 1
    with pytest.raises(fake_pika.exceptions.NackError):
        pub.publish(EXCHANGE, "archive.ingested", _ev())
    assert pub.declare_queues([{"queue_name": "chunking", "routing_key": "json.parsed"}, {"routing_key": "x"}]) is False
    assert "chunking" in broker.queues


def test_roundtrip_requeue_and_malformed(broker):
    pub = create_publisher(_Cfg())
    sub = create_subscriber(_Cfg(), queue_name="parsing")
    got, fail = [], {"n": 1}

    def cb(ev):
        if fail["n"]:
            fail["n"] -= 1
            raise RuntimeError("transient")                    # nack(requeue) -> redelivered
        got.append(ev["data"]["archive_id"])

    sub.subscribe("ArchiveIngested", cb)
    sub.connect()
    pub.connect()
    pub.publish(EXCHANGE, "archive.ingested", _ev(archive_id="1" * 16))
    # malformed bodies straight onto the queue: acked and dropped, they do not block it
    ch = fake_pika.BlockingConnection().channel()
    ch.basic_publish("copilot.events", "archive.ingested", b"{not json")
    ch.basic_publish("copilot.events", "archive.ingested", json.dumps({"data": {}}).encode())
    pub.publish(EXCHANGE, "archive.ingested", _ev(archive_id="2" * 16))
    t = _consume(sub)
    assert _wait(lambda: len(got) == 2)
    sub.stop_consuming()
    t.join(5)
    inner = sub._inner
    assert sorted(got) == ["1" * 16, "2" * 16]
    assert inner.stats["requeued"] == 1 and inner.stats["dropped"] == 2 and inner.stats["acked"] == 2
    assert broker.depth("parsing") == 0


def test_broker_drop_reconnects_both_sides(broker):
    pub = create_publisher(_Cfg(), enable_validation=False)
    sub = create_subscriber(_Cfg(), enable_validation=False, queue_name="parsing")
    got = []
    sub.subscribe("ArchiveIngested", lambda ev: got.append(ev["data"]["archive_id"]))
    sub.connect()
    pub.connect()
    pub.declare_queue("audit", "archive.*")
    t = _consume(sub)
    pub.publish(EXCHANGE, "archive.ingested", _ev(archive_id="1" * 16))
    assert _wait(lambda: got == ["1" * 16])
    broker.kill()                                   # every connection drops
    pub.publish(EXCHANGE, "archive.ingested", _ev(archive_id="2" * 16))   # reconnect + redeclare + send
    assert _wait(lambda: got == ["1" * 16, "2" * 16])
    sub.stop_consuming()
    t.join(5)
    assert sub.stats["reconnects"] >= 1
    assert broker.depth("audit") == 2 and ("copilot.events", "audit", "archive.*") in broker.bindings


def test_unacked_delivery_survives_consumer_loss(broker):
    pub = create_publisher(_Cfg(), enable_validation=False)
    pub.connect()
    pub.declare_queue("parsing", "archive.ingested")
    pub.publish(EXCHANGE, "archive.ingested", _ev())
    sub = create_subscriber(_Cfg(), enable_validation=False, queue_name="parsing")
    entered, release, got = threading.Event(), threading.Event(), []

    def slow(ev):
        if not entered.is_set():
            entered.set()
            release.wait(5)
            broker.kill()                           # connection lost while the handler runs
            return
        got.append(ev)

    sub.subscribe("ArchiveIngested", slow)
    t = _consume(sub)
    assert entered.wait(5)
    release.set()
    assert _wait(lambda: len(got) == 1)             # redelivered after the reconnect, exactly once more
    sub.stop_consuming()
    t.join(5)
    assert broker.depth("parsing") == 0


def test_reconnect_circuit_breaker(broker):
    from copilot_for_consensus_amd.bus.rabbitmq import RabbitMQPublisher
    pub = RabbitMQPublisher(reconnect_delay=10.0, max_reconnect_attempts=3)
    now = [0.0]
    pub.link.clock = lambda: now[0]
    broker.up = False
    with pytest.raises(ConnectionError):
        pub.publish(EXCHANGE, "k", _ev())
    assert pub.link.failures == 1
    with pytest.raises(ConnectionError):
        pub.publish(EXCHANGE, "k", _ev())           # throttled: no attempt inside the backoff window
    assert pub.link.failures == 1
    now[0] += 20.0
    with pytest.raises(ConnectionError):
        pub.publish(EXCHANGE, "k", _ev())
    assert pub.link.failures == 2
    now[0] += 1000.0
    broker.up = True
    pub.connect()                                   # explicit connect always allowed
    pub.declare_queue("q", "k")
    pub.publish(EXCHANGE, "k", _ev())
    assert broker.depth("q") == 1
    pub.link.failures = 3                           # exhausted: gives up without trying
    broker.kill()
    with pytest.raises(ConnectionError):
        pub.publish(EXCHANGE, "k", _ev())


def test_services_pipeline_over_rabbitmq_driver(broker, tmp_path):
    """The whole service pipeline on MESSAGE_BUS_TYPE=rabbitmq, one consumer thread per service
    (the reference's compose deployment shape): the services run unchanged on this driver."""
    import os
    import shutil

    from copilot_for_consensus_amd.contracts.events import ROUTING_KEYS
    from copilot_for_consensus_amd.embedding import HipEncoderProvider
    from copilot_for_consensus_amd.services.node import Node
    from copilot_for_consensus_amd.summarization import MockSummarizer
    from copilot_for_consensus_amd.vectorstore import HipFlatIndex

    env = {"DOCUMENT_STORE_TYPE": "inmemory", "MESSAGE_BUS_TYPE": "rabbitmq", "RABBITMQ_HOST": "127.0.0.1",
           "METRICS_TYPE": "noop", "LOG_TYPE": "silent", "ERROR_REPORTER_TYPE": "silent",
           "EMBEDDING_BACKEND_TYPE": "mock", "VECTOR_STORE_TYPE": "inmemory", "LLM_BACKEND_TYPE": "mock",
           "ARCHIVE_STORE_TYPE": "inmemory", "SECRET_PROVIDER_TYPE": "env",
           # required by the rabbitmq driver schema (secrets rabbitmq_username / rabbitmq_password)
           "RABBITMQ_USERNAME": "guest", "RABBITMQ_PASSWORD": "guest"}
    emb = HipEncoderProvider(model_name="tiny", device="cpu")
    node = Node(env=env, embedding_provider=emb, vector_store=HipFlatIndex(emb.dimension, device="cpu"),
                summarizer=MockSummarizer(mock_latency_ms=0))
    # the broker definitions (deploy/rabbitmq, the reference's definitions.json): a durable queue per
    # routing key, so failure / terminal events are routable too
    admin = create_publisher(_Cfg(), enable_validation=False)
    admin.connect()
    assert admin.declare_queues([{"queue_name": f"q.{k}", "routing_key": k} for k in sorted(set(ROUTING_KEYS.values()))])
    node.start(threaded=True)
    try:
        src = tmp_path / "src"
        src.mkdir()
        shutil.copy(os.path.join(os.path.dirname(__file__), "fixtures", "sample.mbox"), src / "list.mbox")
        ing = node.services["ingestion"]
        ing.create_source({"name": "wg", "source_type": "local", "url": str(src)})
        ing.trigger_ingestion("wg")
        assert _wait(lambda: len(node.store.query_documents("summaries", {}, limit=100)) == 2, 60)
    finally:
        node.stop()
    assert all(s.subscriber.stats["reconnects"] == 0 for s in node.services.values() if s.subscriber is not None)
    assert broker.depth("q.summary.complete") >= 2


def test_failed_queue_cli_backend_on_rabbitmq(broker):
    """scripts/manage_failed_queues.py's RabbitMQ path (list / inspect / requeue / purge over
    basic_get) through tools/failed_queues.RabbitMQFailedQueues."""
    from copilot_for_consensus_amd.tools.failed_queues import FailedQueueManager, RabbitMQFailedQueues
    pub = create_publisher(_Cfg(), enable_validation=False)
    pub.connect()
    pub.declare_queue("parsing.failed")
    pub.declare_queue("parsing", "archive.ingested")
    failed = Event.create("ParsingFailed", archive_id="a" * 16, error_message="boom", error_type="ValueError",
                          failed_at="2025-01-01T00:00:00Z", retry_count=0,
                          messages_parsed_before_failure=0).to_dict()
    for _ in range(3):
        pub.publish(EXCHANGE, "parsing.failed", failed)
    m = FailedQueueManager(RabbitMQFailedQueues("127.0.0.1", 5672))
    rows = {r["queue"]: r["message_count"] for r in m.list_failed_queues()}
    assert rows == {"parsing.failed": 3}                        # queues never declared are skipped
    assert [e["event_type"] for e in m.inspect_messages("parsing.failed", limit=2)] == ["ParsingFailed"] * 2
    assert broker.depth("parsing.failed") == 3                  # inspect does not consume
    assert m.requeue_messages("parsing.failed", limit=2) == 2   # -> archive.ingested (QUEUE_MAPPINGS)
    assert broker.depth("parsing") == 2 and broker.depth("parsing.failed") == 1
    assert m.purge_messages("parsing.failed") == 1 and broker.depth("parsing.failed") == 0
