"""RESP2 codec, FakeRedis engine/server, Redis client semantics, schema helpers.

Mirrors the reference's Redis test sequence (reference pkg/redis/client/client_test.go:
set key1=value1, set key1=value2, get -> value2, getRange(1,2) -> "al", keys) but
against an in-process RESP server instead of a live 172.20.0.5:32767.
"""
import json
import os

import pytest

from k8s_gpu_scheduler_amd.store import schema
from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine, FakeRedisServer
from k8s_gpu_scheduler_amd.store.resp import (ConnectionFailed, Parser, Redis, RedisError, RedisNil,
                                              encode_command, encode_reply)


def test_codec_roundtrip():
    p = Parser()
    p.feed(encode_reply(["OK", b"bulk", 3, None, [b"x", 1]]) + encode_reply(RedisError("ERR bad")))
    v, ok = p.get()
    assert ok and v == ["OK", b"bulk", 3, None, [b"x", 1]]
    v, ok = p.get()
    assert ok and isinstance(v, RedisError)
    p.feed(encode_command(["SET", "k", "v"])[:7])
    assert p.get() == (None, False)                      # incomplete frame
    p.feed(encode_command(["SET", "k", "v"])[7:])
    assert p.get() == ([b"SET", b"k", b"v"], True)


@pytest.fixture()
def server():
    srv = FakeRedisServer(FakeRedisEngine(password="1234")).start()
    yield srv
    srv.stop()


def test_reference_sequence_over_tcp(server):
    r = Redis.connect(server.addr, "1234")
    r.set("key1", "value1")
    r.set("key1", "value2")
    assert r.get("key1") == "value2"
    assert r.get_range("key1", 1, 2) == "al"
    assert r.append("key1", "X") == 7
    assert r.get_keys() == ["key1"]
    with pytest.raises(RedisNil):
        r.get("missing")
    r.flush()
    assert r.get_keys() == []
    r.close()


def test_auth_required(server):
    r = Redis.connect(server.addr)
    with pytest.raises(RedisError):
        r.get("x")
    with pytest.raises(RedisError):
        Redis.connect(server.addr, "wrong").get("x")


def test_lists_hashes_expiry_pipeline():
    eng = FakeRedisEngine()
    r = Redis(FakeRedisBackend(eng))
    assert r.rpush("l", "a", "b", "c") == 3
    r.ltrim("l", -2, -1)
    assert r.lrange("l", 0, -1) == ["b", "c"]
    r.hset("h", {"x": "1", "y": "2"})
    assert r.hgetall("h") == {"x": "1", "y": "2"}
    r.set("t", "v", ex_s=100)
    assert eng.execute("TTL", "t") > 0
    eng.execute("SET", "gone", "v", "PX", 1)
    import time
    time.sleep(0.01)
    assert r.get_or("gone") is None
    assert r.pipeline([["SET", "a", "1"], ["GET", "a"]]) == ["OK", "1"]


def test_db_select_is_honoured(server):
    a = Redis.connect(server.addr, "1234", db=0)
    b = Redis.connect(server.addr, "1234", db=3)
    a.set("k", "zero")
    b.set("k", "three")
    assert a.get("k") == "zero" and b.get("k") == "three"


def test_persistence_snapshot(tmp_path):
    eng = FakeRedisEngine()
    r = Redis(FakeRedisBackend(eng))
    r.set("node-a", json.dumps(["GPU-1"]))
    r.rpush("l", "x")
    r.hset("h", {"a": "b"})
    p = str(tmp_path / "dump.json")
    eng.save(p)
    eng2 = FakeRedisEngine()
    eng2.load(p)
    r2 = Redis(FakeRedisBackend(eng2))
    assert r2.get("node-a") == '["GPU-1"]' and r2.lrange("l", 0, -1) == ["x"] and r2.hgetall("h") == {"a": "b"}


def test_reconnect_after_server_restart():
    eng = FakeRedisEngine()
    srv = FakeRedisServer(eng).start()
    port = int(srv.addr.rsplit(":", 1)[1])
    r = Redis.connect(srv.addr)
    r.set("a", "1")
    srv.stop()
    with pytest.raises(ConnectionFailed):
        r.get("a")
    srv2 = FakeRedisServer(eng, port=port).start()
    assert r.get("a") == "1"
    srv2.stop()


def test_fault_injection():
    eng = FakeRedisEngine()
    r = Redis(FakeRedisBackend(eng))
    eng.fail_next("GET")
    with pytest.raises(RedisError):
        r.get("x")
    assert r.get_or("x") is None


def test_schema_uuid_filter_and_publish():
    """Profiler semantics: any MIG UUID -> keep only MIG ones
    (reference pkg/profiler/cmd/client/client.go:37-46; test.sh fixture)."""
    raw = "['GPU-ac0112df-7098-6c59-5c4f-a57fa666f808', 'MIG-7a700938-2114-5d88-a93c-167c2a498910', " \
          "'MIG-c8956631-ac65-59d3-9065-c8764799febf']"
    uuids = raw.replace("[", "").replace("]", "").replace("'", "").replace(" ", "").split(",")
    assert schema.filter_partition_uuids(uuids) == [u for u in uuids if u.startswith("MIG")]
    r = Redis(FakeRedisBackend(FakeRedisEngine()))
    schema.publish_uuids(r, "node1", ["GPU-a", "GPU-b"])
    assert r.get("node1") == '["GPU-a","GPU-b"]'
    assert schema.read_uuids(r, "node1") == ["GPU-a", "GPU-b"]
    assert schema.read_uuids(r, "nope") is None
    for i in range(5):
        schema.append_history(r, "pod-a", {"i": i}, keep=3)
    assert [h["i"] for h in schema.read_history(r, "pod-a")] == [2, 3, 4]
