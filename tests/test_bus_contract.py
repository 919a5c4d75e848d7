"""Message-bus contract: in-process broker, noop fakes, validating decorators and factories.

Mirrors the behaviours the reference's copilot_message_bus tests pin down (noop publisher
recording and filtering, noop subscriber injection, validating publisher / subscriber in strict and
non-strict mode, pass-through of connect / disconnect / attributes, factory per driver, routing-key
derivation from event types, requeue of a failing callback, malformed bodies acked) plus the
in-process broker's own guarantees: fan-out per bound queue, competing consumers see each message
once, topic wildcards, redelivery limit -> ``<queue>.dlq`` (schema-invalid events dead-lettered at
once), blocking consume loop stopped from another thread, consumer counts."""
from __future__ import annotations

import json
import threading
import time

import pytest

from copilot_for_consensus_amd.bus import (CountingPublisher, EventValidationError, InProcBroker, InProcPublisher,
                                           InProcSubscriber, NoopPublisher, NoopSubscriber, ValidatingEventPublisher,
                                           ValidatingEventSubscriber, create_publisher, create_subscriber,
                                           default_broker, reset_default_broker)
from copilot_for_consensus_amd.contracts.events import EXCHANGE, ROUTING_KEYS, Event

H16 = "0123456789abcdef"


def parsed(i=0):
    return Event("JSONParsed", {"archive_id": H16, "message_count": 1, "message_doc_ids": [f"{i:016x}"],
                                "thread_count": 1, "thread_ids": [H16], "parsing_duration_seconds": 0.1}).to_dict()


def chunks_prepared():
    return Event("ChunksPrepared", {"message_doc_ids": [H16], "chunk_count": 1, "chunk_ids": [H16],
                                    "chunks_ready": True, "chunking_strategy": "token_window",
                                    "avg_chunk_size_tokens": 10.0}).to_dict()


@pytest.fixture
def broker():
    return InProcBroker(max_redeliveries=3)


# ------------------------------------------------------------------ routing
def test_every_event_type_has_a_dotted_lower_case_routing_key():
    assert len(ROUTING_KEYS) == 17
    for et, key in ROUTING_KEYS.items():
        assert key == key.lower() and "." in key, (et, key)
    assert ROUTING_KEYS["JSONParsed"] == "json.parsed"
    assert ROUTING_KEYS["SummarizationRequested"] == "summarization.requested"


def test_subscribe_binds_routing_key_derived_from_event_type(broker):
    sub = InProcSubscriber(broker=broker, queue_name="parsing")
    sub.subscribe("ChunksPrepared", lambda e: None)
    assert (EXCHANGE, "chunks.prepared") in broker.declare_queue("parsing").bindings
    sub.subscribe("JSONParsed", lambda e: None, routing_key="json.#", exchange="other")
    assert ("other", "json.#") in broker.declare_queue("parsing").bindings


def test_publish_to_unbound_key_reaches_no_queue(broker):
    InProcSubscriber(broker=broker, queue_name="q").subscribe("JSONParsed", lambda e: None)
    assert broker.publish(EXCHANGE, "chunks.prepared", b"{}") == 0
    assert broker.publish("wrong-exchange", "json.parsed", b"{}") == 0
    assert broker.queue_depth("q") == 0
    assert broker.publish(EXCHANGE, "json.parsed", b"{}") == 1


def test_fanout_one_copy_per_bound_queue(broker):
    subs = [InProcSubscriber(broker=broker, queue_name=f"q{i}") for i in range(3)]
    got = {i: [] for i in range(3)}
    for i, s in enumerate(subs):
        s.subscribe("JSONParsed", got[i].append)
    InProcPublisher(broker=broker).publish(EXCHANGE, "json.parsed", parsed())
    for s in subs:
        s.drain()
    assert all(len(v) == 1 for v in got.values())


def test_competing_consumers_on_one_queue_see_each_message_once(broker):
    seen, lock = [], threading.Lock()

    def cb(e):
        with lock:
            seen.append(e["data"]["message_doc_ids"][0])

    subs = [InProcSubscriber(broker=broker, queue_name="shared") for _ in range(4)]
    for s in subs:
        s.subscribe("JSONParsed", cb)
    pub = InProcPublisher(broker=broker)
    for i in range(200):
        pub.publish(EXCHANGE, "json.parsed", parsed(i))
    threads = [threading.Thread(target=s.start_consuming) for s in subs]
    for t in threads:
        t.start()
    deadline = time.time() + 10
    while len(seen) < 200 and time.time() < deadline:
        time.sleep(0.01)
    for s in subs:
        s.stop_consuming()
    for t in threads:
        t.join(5)
    assert sorted(seen) == sorted(f"{i:016x}" for i in range(200))
    assert not any(t.is_alive() for t in threads)


def test_wildcard_binding_receives_every_failure_event(broker):
    sub = InProcSubscriber(broker=broker, queue_name="failures")
    got = []
    for et in ("ParsingFailed", "ChunkingFailed"):
        sub.subscribe(et, got.append, routing_key="#.failed")
    broker.publish(EXCHANGE, "parsing.failed", json.dumps({"event_type": "ParsingFailed"}).encode())
    broker.publish(EXCHANGE, "chunking.failed", json.dumps({"event_type": "ChunkingFailed"}).encode())
    broker.publish(EXCHANGE, "json.parsed", json.dumps({"event_type": "JSONParsed"}).encode())
    assert sub.drain() == 2
    assert [e["event_type"] for e in got] == ["ParsingFailed", "ChunkingFailed"]


# ------------------------------------------------------------------ delivery semantics
def test_failing_callback_requeued_then_succeeds(broker):
    sub = InProcSubscriber(broker=broker, queue_name="q")
    calls = []

    def flaky(e):
        calls.append(1)
        if len(calls) < 2:
            raise RuntimeError("transient")

    sub.subscribe("JSONParsed", flaky)
    InProcPublisher(broker=broker).publish(EXCHANGE, "json.parsed", parsed())
    sub.drain()
    assert len(calls) == 2 and sub.processed == 1 and sub.failed == 1
    assert broker.dead_letters["q"] == []


def test_redelivery_limit_dead_letters(broker):
    sub = InProcSubscriber(broker=broker, queue_name="q")
    sub.subscribe("JSONParsed", lambda e: (_ for _ in ()).throw(RuntimeError("down")))
    ev = parsed()
    InProcPublisher(broker=broker).publish(EXCHANGE, "json.parsed", ev)
    sub.drain()
    assert sub.failed == broker.max_redeliveries
    assert [d["event_id"] for d in broker.dead_letters["q"]] == [ev["event_id"]]


def test_schema_invalid_event_dead_lettered_without_redelivery(broker):
    inner = InProcSubscriber(broker=broker, queue_name="q")
    sub = ValidatingEventSubscriber(inner)
    seen = []
    sub.subscribe("JSONParsed", seen.append)
    bad = parsed()
    del bad["data"]["thread_ids"]
    broker.publish(EXCHANGE, "json.parsed", json.dumps(bad).encode())
    inner.drain()
    assert seen == [] and inner.failed == 1
    assert broker.dead_letters["q"][0]["event_id"] == bad["event_id"]


@pytest.mark.parametrize("body", [b"{not json", b"[]", b'{"no_type": 1}', b"\xff\xfe"])
def test_malformed_bodies_acked_and_dropped(broker, body):
    sub = InProcSubscriber(broker=broker, queue_name="q")
    sub.subscribe("JSONParsed", lambda e: None)
    broker.publish(EXCHANGE, "json.parsed", body)
    assert sub.drain() == 1
    assert sub.failed == 1 and broker.queue_depth("q") == 0 and broker.dead_letters["q"] == []


def test_event_type_without_callback_is_acked(broker):
    sub = InProcSubscriber(broker=broker, queue_name="q")
    sub.subscribe("JSONParsed", lambda e: None, routing_key="#")
    broker.publish(EXCHANGE, "chunks.prepared", json.dumps(chunks_prepared()).encode())
    assert sub.drain() == 1 and sub.processed == 0 and sub.failed == 0


def test_callback_gets_a_private_copy(broker):
    a = InProcSubscriber(broker=broker, queue_name="q")
    got = []
    a.subscribe("JSONParsed", lambda e: (e["data"].clear(), got.append(e)))
    ev = parsed()
    InProcPublisher(broker=broker).publish(EXCHANGE, "json.parsed", ev)
    a.drain()
    assert "archive_id" in ev["data"] and got[0]["data"] == {}


def test_drain_max_items_and_queue_depth(broker):
    sub = InProcSubscriber(broker=broker, queue_name="q")
    sub.subscribe("JSONParsed", lambda e: None)
    pub = InProcPublisher(broker=broker)
    for i in range(5):
        pub.publish(EXCHANGE, "json.parsed", parsed(i))
    assert broker.queue_depth("q") == 5 and broker.queues() == {"q": 5}
    assert sub.drain(max_items=2) == 2 and broker.queue_depth("q") == 3
    assert sub.drain() == 3 and broker.queue_depth("q") == 0
    assert broker.published == 5


def test_consumer_counts_follow_consume_loop(broker):
    sub = InProcSubscriber(broker=broker, queue_name="q")
    sub.subscribe("JSONParsed", lambda e: None)
    assert broker.consumer_counts() == {"q": 0}
    t = threading.Thread(target=sub.start_consuming)
    t.start()
    deadline = time.time() + 5
    while broker.consumer_counts()["q"] != 1 and time.time() < deadline:
        time.sleep(0.01)
    assert broker.consumer_counts() == {"q": 1}
    sub.stop_consuming()
    t.join(5)
    assert not t.is_alive() and broker.consumer_counts() == {"q": 0}


def test_concurrent_publishers_lose_nothing(broker):
    sub = InProcSubscriber(broker=broker, queue_name="q")
    sub.subscribe("JSONParsed", lambda e: None)

    def worker(k):
        p = InProcPublisher(broker=broker)
        for i in range(100):
            p.publish(EXCHANGE, "json.parsed", parsed(k * 1000 + i))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert broker.queue_depth("q") == 800 and sub.drain() == 800


def test_default_broker_is_shared_and_resettable():
    reset_default_broker()
    a, b = default_broker(), default_broker()
    assert a is b
    assert InProcPublisher().broker is a and InProcSubscriber().broker is a
    reset_default_broker()
    assert default_broker() is not a
    reset_default_broker()


# ------------------------------------------------------------------ noop fakes
def test_noop_publisher_records_filters_and_clears():
    p = NoopPublisher()
    p.connect()
    assert p.connected
    p.publish(EXCHANGE, "json.parsed", parsed())
    p.publish(EXCHANGE, "chunks.prepared", chunks_prepared())
    assert len(p.get_events()) == 2
    assert [e["event_type"] for e in p.get_events("ChunksPrepared")] == ["ChunksPrepared"]
    assert p.published_events[0]["routing_key"] == "json.parsed"
    ev = parsed()
    p.publish(EXCHANGE, "json.parsed", ev)
    ev["data"]["archive_id"] = "changed"      # recorded events are snapshots
    assert p.get_events("JSONParsed")[-1]["data"]["archive_id"] == H16
    p.clear_events()
    assert p.get_events() == []
    p.disconnect()
    assert not p.connected


def test_counting_publisher():
    p = CountingPublisher()
    for _ in range(3):
        p.publish(EXCHANGE, "json.parsed", parsed())
    p.publish(EXCHANGE, "chunks.prepared", chunks_prepared())
    assert p.counts == {"JSONParsed": 3, "ChunksPrepared": 1}


def test_noop_subscriber_injection_and_blocking_consume():
    s = NoopSubscriber()
    got = []
    s.subscribe("JSONParsed", got.append, routing_key="json.parsed")
    assert s.get_subscriptions() == ["JSONParsed"] and s.routing_keys["JSONParsed"] == "json.parsed"
    s.inject_event(parsed())
    s.inject_event(chunks_prepared())       # no callback for that type: ignored
    assert len(got) == 1
    t = threading.Thread(target=s.start_consuming)
    t.start()
    time.sleep(0.05)
    assert s.consuming and t.is_alive()
    s.stop_consuming()
    t.join(5)
    assert not t.is_alive() and not s.consuming


# ------------------------------------------------------------------ validating decorators
def test_validating_publisher_passthrough():
    inner = NoopPublisher()
    pub = ValidatingEventPublisher(inner)
    pub.connect()
    assert inner.connected
    pub.publish(EXCHANGE, "json.parsed", parsed())
    assert pub.get_events("JSONParsed")          # attribute access reaches the wrapped publisher
    pub.disconnect()
    assert not inner.connected


@pytest.mark.parametrize("mutate", [
    lambda e: e.pop("event_id"),
    lambda e: e.update(event_type="NoSuchEvent"),
    lambda e: e["data"].update(message_count="one"),
    lambda e: e["data"].update(unexpected=True),
    lambda e: e.update(extra_envelope_field=1),
])
def test_validating_publisher_rejects_invalid_envelopes(mutate):
    inner = NoopPublisher()
    pub = ValidatingEventPublisher(inner)
    ev = parsed()
    mutate(ev)
    with pytest.raises(EventValidationError) as ei:
        pub.publish(EXCHANGE, "json.parsed", ev)
    assert ei.value.errors
    assert inner.get_events() == []              # nothing reached the transport


def test_validating_publisher_non_strict_forwards():
    inner = NoopPublisher()
    ev = parsed()
    ev["data"]["message_count"] = "one"
    ValidatingEventPublisher(inner, strict=False).publish(EXCHANGE, "json.parsed", ev)
    assert len(inner.get_events()) == 1


def test_validating_subscriber_non_strict_skips_invalid_events():
    sub = ValidatingEventSubscriber(NoopSubscriber(), strict=False)
    seen = []
    sub.subscribe("JSONParsed", seen.append)
    bad = parsed()
    bad["data"]["message_count"] = "one"
    sub._inner.inject_event(bad)                 # logged and skipped, no exception
    sub._inner.inject_event(parsed())
    assert len(seen) == 1 and len(sub.rejected) == 1


def test_validating_subscriber_passthrough():
    inner = NoopSubscriber()
    sub = ValidatingEventSubscriber(inner)
    sub.connect()
    assert inner.connected
    sub.subscribe("JSONParsed", lambda e: None)
    assert sub.get_subscriptions() == ["JSONParsed"]
    t = threading.Thread(target=sub.start_consuming)
    t.start()
    time.sleep(0.02)
    sub.stop_consuming()
    t.join(5)
    assert not t.is_alive()
    sub.disconnect()
    assert not inner.connected


# ------------------------------------------------------------------ factories
@pytest.mark.parametrize("name", ["inproc", "noop"])
def test_factory_wraps_in_validation_by_default(name):
    broker = InProcBroker()
    assert isinstance(create_publisher(name, broker=broker), ValidatingEventPublisher)
    assert isinstance(create_subscriber(name, broker=broker), ValidatingEventSubscriber)
    assert not isinstance(create_publisher(name, enable_validation=False, broker=broker), ValidatingEventPublisher)


def test_factory_config_object_and_end_to_end_flow():
    class Cfg:
        driver_name = "inproc"
        driver_config = {}

    broker = InProcBroker()
    pub = create_publisher(Cfg(), broker=broker)
    sub = create_subscriber(Cfg(), broker=broker, queue_name="chunking")
    got = []
    sub.subscribe("JSONParsed", got.append)
    pub.publish(EXCHANGE, "json.parsed", parsed())
    sub._inner.drain()
    assert len(got) == 1 and got[0]["event_type"] == "JSONParsed"


@pytest.mark.parametrize("name", ["kafka", "sqs", ""])
def test_factory_unknown_driver(name):
    with pytest.raises(ValueError):
        create_publisher(name or "unknown")
    with pytest.raises(ValueError):
        create_subscriber(name or "unknown")
