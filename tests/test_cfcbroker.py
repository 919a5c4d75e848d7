"""The native cfc-broker (csrc/broker/cfc_broker.cpp) through its Python driver (bus/cfcbroker.py).

Covers the RabbitMQ behaviours the reference relies on: topic routing, publisher
confirms + durability across a broker restart (including a kill -9), prefetch, ack / nack(requeue),
redelivery of a dead consumer's unacked messages, the redelivery limit -> ``<queue>.dlq``, the
failed-queue CLI backend, and the services' reconnecting consume loop.
"""
from __future__ import annotations

import json
import signal
import threading
import time

import pytest

from copilot_for_consensus_amd.bus import create_publisher, create_subscriber
from copilot_for_consensus_amd.bus.cfcbroker import (CfcBrokerFailedQueues, CfcBrokerPublisher, CfcBrokerSubscriber,
                                                      Connection, spawn_broker)
from copilot_for_consensus_amd.contracts.events import EXCHANGE, Event


@pytest.fixture
def broker(tmp_path):
    procs = []

    def start(data_dir=tmp_path / "data", port=0, **kw):
        p, port = spawn_broker(port=port, data_dir=data_dir, **kw)
        procs.append(p)
        return p, port

    yield start
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
            try:
                p.wait(5)
            except Exception:
                p.kill()


def _ev(event_type="ArchiveIngested", **over):
    data = dict(archive_id="a" * 16, source_name="s", source_type="local", source_url="file:///x",
                file_size_bytes=1, file_hash_sha256="0" * 64, ingestion_started_at="2025-01-01T00:00:00Z",
                ingestion_completed_at="2025-01-01T00:00:01Z")
    data.update(over)
    return Event.create(event_type, **data).to_dict()


def test_topic_routing_and_confirms(broker):
    _, port = broker()
    c = Connection("127.0.0.1", port)
    for q, pat in (("exact", "archive.ingested"), ("star", "*.ingested"), ("hash", "archive.#"), ("all", "#"),
                   ("none", "json.parsed")):
        c.declare(q)
        c.bind(q, EXCHANGE, pat)
    assert c.publish(EXCHANGE, "archive.ingested", b"{}") == 4
    assert c.publish(EXCHANGE, "archive.ingestion.failed", b"{}") == 2     # hash + all
    assert c.publish(EXCHANGE, "nobody.listens", b"{}") == 1               # all
    assert c.publish("other.exchange", "archive.ingested", b"{}") == 0
    q = c.stats()["queues"]
    assert {k: v["ready"] for k, v in q.items()} == {"exact": 1, "star": 1, "hash": 2, "all": 3, "none": 0}
    assert c.ping() < 1.0


def test_prefetch_ack_nack_and_dead_consumer_redelivery(broker):
    _, port = broker()
    admin = Connection("127.0.0.1", port)
    admin.declare("work")
    admin.bind("work", EXCHANGE, "k")
    for i in range(5):
        admin.publish(EXCHANGE, "k", str(i).encode())
    a = Connection("127.0.0.1", port)
    a.consume("work", prefetch=2)
    d0, d1 = a.next_delivery(2), a.next_delivery(2)
    assert (d0.body, d1.body) == (b"0", b"1")
    assert a.next_delivery(0.3) is None                    # prefetch 2: nothing more until a settle
    a.ack(d0.tag)
    d2 = a.next_delivery(2)
    assert d2.body == b"2"
    a.nack(d1.tag, requeue=True)                            # back to the head, redelivery count 1
    d1b = a.next_delivery(2)
    assert (d1b.body, d1b.redeliveries) == (b"1", 1)
    a.close()                                               # dies holding d2 and d1b unacked
    b = Connection("127.0.0.1", port)
    b.consume("work", prefetch=10)
    got = {}
    while True:
        d = b.next_delivery(1.0)
        if d is None:
            break
        got[d.body] = d.redeliveries
        b.ack(d.tag)
    assert got == {b"1": 2, b"2": 1, b"3": 0, b"4": 0}
    st = admin.stats()["queues"]["work"]
    assert (st["ready"], st["unacked"], st["acked"]) == (0, 0, 5)


def test_redelivery_limit_moves_to_dlq(broker):
    _, port = broker(max_redeliveries=2)
    c = Connection("127.0.0.1", port)
    c.declare("svc")
    c.bind("svc", EXCHANGE, "k")
    c.publish(EXCHANGE, "k", b"poison")
    c.publish(EXCHANGE, "k", b"reject")
    c.consume("svc", prefetch=1)
    seen = 0
    while True:
        d = c.next_delivery(1.0)
        if d is None:
            break
        if d.body == b"reject":
            c.nack(d.tag, requeue=False)                    # straight to the DLQ
        else:
            seen += 1
            c.nack(d.tag, requeue=True)
    assert seen == 3                                        # first delivery + 2 redeliveries
    st = c.stats()["queues"]
    assert st["svc"]["ready"] == 0 and st["svc"]["dead_lettered"] == 2
    assert sorted(d.body for d in c.peek("svc.dlq", 10)) == [b"poison", b"reject"]


def test_durability_across_restart_and_kill(broker, tmp_path):
    data = tmp_path / "data"
    p, port = broker(data_dir=data)
    c = Connection("127.0.0.1", port)
    c.declare("durable")
    c.bind("durable", EXCHANGE, "x.*")
    c.declare("transient", durable=False)
    c.bind("transient", EXCHANGE, "x.*")
    for i in range(20):
        c.publish(EXCHANGE, "x.y", json.dumps({"i": i}).encode())
    c.consume("durable", prefetch=5)
    for _ in range(5):
        d = c.next_delivery(2)
        if json.loads(d.body)["i"] < 3:
            c.ack(d.tag)                                    # 0..2 settled; 3, 4 unacked when it dies
    c.ping()
    p.send_signal(signal.SIGKILL)                           # no clean shutdown: the journal must hold
    p.wait(5)
    _, port2 = broker(data_dir=data)
    c2 = Connection("127.0.0.1", port2)
    st = c2.stats()["queues"]
    assert "transient" not in st
    assert st["durable"]["ready"] == 17
    assert st["durable"]["bindings"] == [[EXCHANGE, "x.*"]]
    left = sorted(json.loads(d.body)["i"] for d in c2.peek("durable", 100))
    assert left == list(range(3, 20))
    assert c2.publish(EXCHANGE, "x.z", b"{}") == 1          # bindings survived


def test_driver_roundtrip_with_validation_and_reconnect(broker, tmp_path):
    data = tmp_path / "data"
    p, port = broker(data_dir=data, port=0)
    cfg = {"broker_host": "127.0.0.1", "broker_port": port}

    class Cfg:
        driver_name = "cfcbroker"
        driver_config = cfg

    pub = create_publisher(Cfg())
    sub = create_subscriber(Cfg(), queue_name="parsing")
    got, fail_once = [], {"n": 1}

    def cb(ev):
        if fail_once["n"]:
            fail_once["n"] -= 1
            raise RuntimeError("transient")                 # nack + requeue, then succeeds
        got.append(ev["data"]["archive_id"])

    sub.subscribe("ArchiveIngested", cb)
    sub.connect()
    pub.connect()
    pub.publish(EXCHANGE, "archive.ingested", _ev(archive_id="1" * 16))
    t = threading.Thread(target=sub.start_consuming, daemon=True)
    t.start()
    deadline = time.time() + 10
    while not got and time.time() < deadline:
        time.sleep(0.05)
    assert got == ["1" * 16]
    # broker restart on the same port: the consume loop and the publisher reconnect by themselves
    p.send_signal(signal.SIGTERM)
    p.wait(5)
    broker(data_dir=data, port=port)
    pub.publish(EXCHANGE, "archive.ingested", _ev(archive_id="2" * 16))
    deadline = time.time() + 15
    while len(got) < 2 and time.time() < deadline:
        time.sleep(0.05)
    sub.stop_consuming()
    t.join(5)
    assert got == ["1" * 16, "2" * 16]
    assert sub._inner.reconnects >= 1


def test_failed_queue_backend(broker):
    from copilot_for_consensus_amd.tools.failed_queues import FailedQueueManager
    _, port = broker()
    fq = CfcBrokerFailedQueues("127.0.0.1", port)
    pub = CfcBrokerPublisher(broker_host="127.0.0.1", broker_port=port)
    pub.connect()
    failed = Event.create("ParsingFailed", archive_id="a" * 16, error_message="boom", error_type="ValueError",
                          failed_at="2025-01-01T00:00:00Z", retry_count=0,
                          messages_parsed_before_failure=0).to_dict()
    pub.publish(EXCHANGE, "parsing.failed", failed)
    c = Connection("127.0.0.1", port)
    c.declare("parsing")
    c.bind("parsing", EXCHANGE, "archive.ingested")
    m = FailedQueueManager(fq)
    rows = {r["queue"]: r["message_count"] for r in m.list_failed_queues()}
    assert rows["parsing.failed"] == 1
    assert m.inspect_messages("parsing.failed")[0]["event_type"] == "ParsingFailed"
    assert m.requeue_messages("parsing.failed") == 1       # -> archive.ingested (QUEUE_MAPPINGS)
    assert c.stats()["queues"]["parsing"]["ready"] == 1
    assert fq.count("parsing.failed") == 0


def test_subscriber_drain_and_malformed(broker):
    _, port = broker()
    sub = CfcBrokerSubscriber(broker_host="127.0.0.1", broker_port=port, queue_name="chunking")
    seen = []
    sub.subscribe("JSONParsed", lambda ev: seen.append(ev["event_type"]))
    sub.connect()
    c = Connection("127.0.0.1", port)
    c.publish(EXCHANGE, "json.parsed", b"not json")
    c.publish(EXCHANGE, "json.parsed", json.dumps({"event_type": "JSONParsed", "data": {}}).encode())
    assert sub.drain(idle_timeout=0.5) == 2
    assert seen == ["JSONParsed"] and sub.failed == 1
    assert c.stats()["queues"]["chunking"]["unacked"] == 0


def test_exporter_reads_native_broker(broker):
    from copilot_for_consensus_amd.bus.cfcbroker import CfcBrokerMonitor
    from copilot_for_consensus_amd.storage.document_store import InMemoryDocumentStore
    from copilot_for_consensus_amd.tools.exporters import PipelineExporter
    _, port = broker(max_redeliveries=0)
    c = Connection("127.0.0.1", port)
    c.declare("parsing", max_redeliveries=1)
    c.bind("parsing", EXCHANGE, "archive.ingested")
    c.publish(EXCHANGE, "archive.ingested", b"{}")
    c.publish(EXCHANGE, "archive.ingested", b"{}")
    c.consume("parsing", prefetch=1)
    d = c.next_delivery(2)
    c.nack(d.tag, requeue=False)
    c.ping()
    text = PipelineExporter(InMemoryDocumentStore(), broker=CfcBrokerMonitor("127.0.0.1", port)).render()
    assert 'copilot_queue_messages{queue="parsing"} 0' in text          # the other one is unacked
    assert 'copilot_queue_messages_unacked{queue="parsing"} 1' in text
    assert 'copilot_queue_dead_lettered_total{queue="parsing"} 1' in text
    assert 'copilot_queue_messages{queue="parsing.dlq"} 1' in text
    assert 'copilot_queue_consumers{queue="parsing"} 1' in text


def test_failed_queues_cli_on_native_broker(broker, capsys):
    from copilot_for_consensus_amd.tools.failed_queues import main
    _, port = broker()
    CfcBrokerFailedQueues("127.0.0.1", port)        # declares the *.failed queues
    c = Connection("127.0.0.1", port)
    c.publish(EXCHANGE, "chunking.failed", json.dumps({"event_type": "ChunkingFailed", "data": {}}).encode())
    assert main(["--backend", "cfcbroker", "--port", str(port), "list"]) == 0
    rows = {r["queue"]: r["message_count"] for r in json.loads(capsys.readouterr().out)}
    assert rows["chunking.failed"] == 1
    assert main(["--backend", "cfcbroker", "--port", str(port), "purge", "chunking.failed", "--confirm"]) == 0
    assert capsys.readouterr().out.strip() == "1"
