"""RESP2 protocol codec + a small synchronous Redis client.

The reference uses go-redis v8 through a thin wrapper: Set (no TTL) / Get / GetRange /
GetKeys (`KEYS *`) / FlushAll, `New(addr, pw, db)` ignoring db
(reference pkg/redis/client/client.go:11-67).  No `redis` Python package exists here, so
the wire protocol is implemented directly.  Fixes vs the reference:
one pooled connection per client (not one per Score), honoured `db`, bounded
connect/read timeouts and reconnect-with-retry.
"""
from __future__ import annotations

import socket
import threading
import time
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

Bulk = Optional[bytes]


class RedisError(Exception):
    """-ERR replies from the server."""


class RedisNil(Exception):
    """Key does not exist (go-redis `redis.Nil`)."""


class ConnectionFailed(Exception):
    pass


# --------------------------------------------------------------------------- codec
def encode_command(args: Sequence[Union[str, bytes, int, float]]) -> bytes:
    out = [b"*%d\r\n" % len(args)]
    for a in args:
        if isinstance(a, bytes):
            b = a
        elif isinstance(a, str):
            b = a.encode()
        else:
            b = str(a).encode()
        out.append(b"$%d\r\n%s\r\n" % (len(b), b))
    return b"".join(out)


def encode_reply(v: Any) -> bytes:
    """Server-side encoder: str -> simple string, bytes -> bulk, int -> integer,
    None -> nil bulk, list -> array, RedisError -> error."""
    if isinstance(v, RedisError):
        return b"-%s\r\n" % str(v).encode()
    if v is None:
        return b"$-1\r\n"
    if isinstance(v, bool):
        return b":%d\r\n" % int(v)
    if isinstance(v, int):
        return b":%d\r\n" % v
    if isinstance(v, str):
        return b"+%s\r\n" % v.encode()
    if isinstance(v, (bytes, bytearray)):
        return b"$%d\r\n%s\r\n" % (len(v), bytes(v))
    if isinstance(v, (list, tuple)):
        return b"*%d\r\n" % len(v) + b"".join(encode_reply(x) for x in v)
    raise TypeError(f"cannot encode {type(v)}")


class Parser:
    """Incremental RESP2 parser (client replies and server commands)."""

    def __init__(self) -> None:
        self.buf = bytearray()

    def feed(self, data: bytes) -> None:
        self.buf += data

    def _line(self, pos: int) -> Tuple[Optional[bytes], int]:
        i = self.buf.find(b"\r\n", pos)
        if i < 0:
            return None, pos
        return bytes(self.buf[pos:i]), i + 2

    def _parse(self, pos: int) -> Tuple[Any, int, bool]:
        if pos >= len(self.buf):
            return None, pos, False
        t = self.buf[pos:pos + 1]
        line, nxt = self._line(pos + 1)
        if line is None:
            return None, pos, False
        if t == b"+":
            return line.decode(), nxt, True
        if t == b"-":
            return RedisError(line.decode()), nxt, True
        if t == b":":
            return int(line), nxt, True
        if t == b"$":
            n = int(line)
            if n < 0:
                return None, nxt, True
            if len(self.buf) < nxt + n + 2:
                return None, pos, False
            return bytes(self.buf[nxt:nxt + n]), nxt + n + 2, True
        if t == b"*":
            n = int(line)
            if n < 0:
                return None, nxt, True
            items = []
            p = nxt
            for _ in range(n):
                v, p, ok = self._parse(p)
                if not ok:
                    return None, pos, False
                items.append(v)
            return items, p, True
        # inline command (telnet style)
        return [w.encode() for w in bytes(self.buf[pos:nxt - 2]).decode().split()], nxt, True

    def get(self) -> Tuple[Any, bool]:
        v, p, ok = self._parse(0)
        if ok:
            del self.buf[:p]
        return v, ok


# --------------------------------------------------------------------------- client
class RespClient:
    """Minimal synchronous Redis client (thread-safe, one connection, auto-reconnect)."""

    def __init__(self, addr: str, password: str = "", db: int = 0, timeout_s: float = 2.0,
                 retries: int = 2):
        host, _, port = addr.rpartition(":")
        self.host, self.port = host or "127.0.0.1", int(port or 6379)
        self.addr = addr
        self.password, self.db = password, db
        self.timeout_s, self.retries = timeout_s, retries
        self._sock: Optional[socket.socket] = None
        self._parser = Parser()
        self._lock = threading.Lock()

    def _connect(self) -> None:
        try:
            s = socket.create_connection((self.host, self.port), timeout=self.timeout_s)
        except OSError as e:
            raise ConnectionFailed(f"redis {self.addr}: {e}") from e
        s.settimeout(self.timeout_s)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._sock, self._parser = s, Parser()
        if self.password:
            self._roundtrip(["AUTH", self.password])
        if self.db:
            self._roundtrip(["SELECT", self.db])

    def _roundtrip_many(self, cmds: List[Sequence[Any]]) -> List[Any]:
        assert self._sock is not None
        self._sock.sendall(b"".join(encode_command(c) for c in cmds))
        out = []
        while len(out) < len(cmds):
            v, ok = self._parser.get()
            if ok:
                out.append(v)
                continue
            data = self._sock.recv(65536)
            if not data:
                raise ConnectionFailed("connection closed")
            self._parser.feed(data)
        return out

    def _roundtrip(self, cmd: Sequence[Any]) -> Any:
        v = self._roundtrip_many([cmd])[0]
        if isinstance(v, RedisError):
            raise v
        return v

    def execute(self, *cmd: Any) -> Any:
        return self.pipeline([cmd])[0]

    def pipeline(self, cmds: List[Sequence[Any]], raise_errors: bool = True) -> List[Any]:
        last: Optional[Exception] = None
        with self._lock:
            for attempt in range(self.retries + 1):
                try:
                    if self._sock is None:
                        self._connect()
                    res = self._roundtrip_many(cmds)
                    if raise_errors:
                        for r in res:
                            if isinstance(r, RedisError):
                                raise r
                    return res
                except (OSError, ConnectionFailed) as e:
                    last = e
                    self.close_nolock()
                    time.sleep(0.01 * (2 ** attempt))
            raise ConnectionFailed(str(last))

    def close_nolock(self) -> None:
        if self._sock is not None:
            try:
                self._sock.close()
            except OSError:
                pass
            self._sock = None

    def close(self) -> None:
        with self._lock:
            self.close_nolock()


class Redis:
    """The `client.Client` interface of the reference (Set/Get/GetRange/GetKeys, FlushRedis)
    over either a RespClient (TCP) or an in-process FakeRedis engine."""

    def __init__(self, backend: Any):
        self.backend = backend

    @classmethod
    def connect(cls, addr: str, password: str = "", db: int = 0, timeout_s: float = 2.0) -> "Redis":
        return cls(RespClient(addr, password, db, timeout_s))

    def _x(self, *cmd: Any) -> Any:
        return self.backend.execute(*cmd)

    @staticmethod
    def _s(v: Any) -> Any:
        return v.decode() if isinstance(v, bytes) else v

    def set(self, key: str, value: str, ex_s: Optional[int] = None) -> None:
        if ex_s:
            self._x("SET", key, value, "EX", ex_s)
        else:
            self._x("SET", key, value)

    def get(self, key: str) -> str:
        v = self._x("GET", key)
        if v is None:
            raise RedisNil(key)
        return self._s(v)

    def get_or(self, key: str, default: Optional[str] = None) -> Optional[str]:
        v = self._x("GET", key)
        return default if v is None else self._s(v)

    def get_range(self, key: str, start: int, end: int) -> str:
        return self._s(self._x("GETRANGE", key, start, end))

    def append(self, key: str, value: str) -> int:
        return int(self._x("APPEND", key, value))

    def get_keys(self, pattern: str = "*") -> List[str]:
        return [self._s(k) for k in self._x("KEYS", pattern)]

    def delete(self, *keys: str) -> int:
        return int(self._x("DEL", *keys))

    def flush(self) -> None:
        self._x("FLUSHALL")

    def rpush(self, key: str, *values: str) -> int:
        return int(self._x("RPUSH", key, *values))

    def lrange(self, key: str, start: int, stop: int) -> List[str]:
        return [self._s(v) for v in self._x("LRANGE", key, start, stop)]

    def ltrim(self, key: str, start: int, stop: int) -> None:
        self._x("LTRIM", key, start, stop)

    def hset(self, key: str, mapping: Dict[str, str]) -> int:
        args: List[Any] = []
        for k, v in mapping.items():
            args += [k, v]
        return int(self._x("HSET", key, *args))

    def hgetall(self, key: str) -> Dict[str, str]:
        v = self._x("HGETALL", key) or []
        return {self._s(v[i]): self._s(v[i + 1]) for i in range(0, len(v), 2)}

    def ping(self) -> bool:
        return self._s(self._x("PING")) == "PONG"

    def pipeline(self, cmds: List[Sequence[Any]]) -> List[Any]:
        if hasattr(self.backend, "pipeline"):
            return [self._s(v) if not isinstance(v, list) else v for v in self.backend.pipeline(cmds)]
        return [self._s(self.backend.execute(*c)) for c in cmds]

    def close(self) -> None:
        c = getattr(self.backend, "close", None)
        if c:
            c()
