"""FakeRedis: an in-memory Redis engine + a RESP2 TCP server around it.

The reference's only Redis test needs a live server at 172.20.0.5:32767
(reference pkg/redis/client/client_test.go:153-156).  This engine implements the
commands the framework uses (strings, lists, hashes, keys, expiry, AUTH/SELECT, FLUSH*)
and can persist to a JSON snapshot (the AOF/RDB persistence the reference configures in
deploy/redis/redis-config.yaml:318-320,1073 becomes `save()`/`load()`).  Fault
injection: `fail_next`, `latency_s`, `down`.
"""
from __future__ import annotations

import fnmatch
import json
import os
import socket
import socketserver
import threading
import time
from typing import Any, Dict, List, Optional

from .resp import Parser, RedisError, encode_reply


def _b(x: Any) -> bytes:
    if isinstance(x, bytes):
        return x
    return str(x).encode()


class FakeRedisEngine:
    def __init__(self, password: str = "", databases: int = 16):
        self._lock = threading.RLock()
        self.password = password
        self.dbs: List[Dict[bytes, Any]] = [dict() for _ in range(databases)]
        self.expiry: List[Dict[bytes, float]] = [dict() for _ in range(databases)]
        self.latency_s = 0.0
        self.down = False
        self._faults: List[List[Any]] = []
        self.commands = 0

    def fail_next(self, cmd: str, times: int = 1, error: str = "ERR injected fault") -> None:
        self._faults.append([cmd.upper(), times, error])

    # --------------------------------------------------------------- persistence
    def save(self, path: str) -> None:
        with self._lock:
            out = []
            for db, exp in zip(self.dbs, self.expiry):
                d = {}
                for k, v in db.items():
                    if isinstance(v, bytes):
                        d[k.decode("latin1")] = {"t": "s", "v": v.decode("latin1")}
                    elif isinstance(v, list):
                        d[k.decode("latin1")] = {"t": "l", "v": [x.decode("latin1") for x in v]}
                    elif isinstance(v, dict):
                        d[k.decode("latin1")] = {"t": "h", "v": {a.decode("latin1"): b.decode("latin1")
                                                                for a, b in v.items()}}
                    if k in exp:
                        d[k.decode("latin1")]["e"] = exp[k] - time.time()
                out.append(d)
            tmp = path + ".tmp"
            with open(tmp, "w") as f:
                json.dump(out, f)
            os.replace(tmp, path)

    def load(self, path: str) -> None:
        with open(path) as f:
            data = json.load(f)
        with self._lock:
            for i, d in enumerate(data):
                self.dbs[i].clear()
                self.expiry[i].clear()
                for k, e in d.items():
                    kb = k.encode("latin1")
                    if e["t"] == "s":
                        self.dbs[i][kb] = e["v"].encode("latin1")
                    elif e["t"] == "l":
                        self.dbs[i][kb] = [x.encode("latin1") for x in e["v"]]
                    else:
                        self.dbs[i][kb] = {a.encode("latin1"): b.encode("latin1") for a, b in e["v"].items()}
                    if "e" in e:
                        self.expiry[i][kb] = time.time() + e["e"]

    # --------------------------------------------------------------- dispatch
    def _expired(self, db: int, k: bytes) -> bool:
        t = self.expiry[db].get(k)
        if t is not None and t <= time.time():
            self.dbs[db].pop(k, None)
            self.expiry[db].pop(k, None)
            return True
        return False

    def _get(self, db: int, k: bytes, typ: type) -> Any:
        self._expired(db, k)
        v = self.dbs[db].get(k)
        if v is not None and not isinstance(v, typ):
            raise RedisError("WRONGTYPE Operation against a key holding the wrong kind of value")
        return v

    def execute(self, *args: Any, session: Optional[Dict[str, Any]] = None) -> Any:
        """Run one command; `session` carries per-connection auth/db state."""
        if session is None:
            session = {"auth": True, "db": 0}
        if self.down:
            raise ConnectionError("fake redis is down")
        if self.latency_s:
            time.sleep(self.latency_s)
        a = [_b(x) for x in args]
        cmd = a[0].decode().upper()
        for f in self._faults:
            if f[0] == cmd and f[1] > 0:
                f[1] -= 1
                return RedisError(f[2])
        with self._lock:
            self.commands += 1
            try:
                return self._dispatch(cmd, a[1:], session)
            except RedisError as e:
                return e
            except (IndexError, ValueError):
                return RedisError(f"ERR wrong number of arguments or bad value for '{cmd.lower()}' command")

    def _dispatch(self, cmd: str, a: List[bytes], s: Dict[str, Any]) -> Any:
        if cmd == "AUTH":
            pw = a[-1].decode()
            if not self.password or pw == self.password:
                s["auth"] = True
                return "OK"
            return RedisError("WRONGPASS invalid username-password pair or user is disabled.")
        if cmd in ("PING",):
            return "PONG" if not a else a[0]
        if cmd in ("QUIT",):
            return "OK"
        if self.password and not s.get("auth"):
            return RedisError("NOAUTH Authentication required.")
        db = s.get("db", 0)
        D = self.dbs[db]
        if cmd == "SELECT":
            i = int(a[0])
            if not 0 <= i < len(self.dbs):
                return RedisError("ERR DB index is out of range")
            s["db"] = i
            return "OK"
        if cmd == "SET":
            k, v = a[0], a[1]
            opts = [x.decode().upper() for x in a[2:]]
            if "NX" in opts and (not self._expired(db, k)) and k in D:
                return None
            if "XX" in opts and (self._expired(db, k) or k not in D):
                return None
            D[k] = v
            self.expiry[db].pop(k, None)
            if "EX" in opts:
                self.expiry[db][k] = time.time() + float(a[2 + opts.index("EX") + 1])
            if "PX" in opts:
                self.expiry[db][k] = time.time() + float(a[2 + opts.index("PX") + 1]) / 1000
            return "OK"
        if cmd == "GET":
            return self._get(db, a[0], bytes)
        if cmd == "MGET":
            return [self._get(db, k, bytes) for k in a]
        if cmd == "GETRANGE":
            v = self._get(db, a[0], bytes) or b""
            st, en = int(a[1]), int(a[2])
            n = len(v)
            if st < 0:
                st = max(n + st, 0)
            if en < 0:
                en = n + en
            en = min(en, n - 1)
            return v[st:en + 1] if st <= en else b""
        if cmd == "APPEND":
            v = (self._get(db, a[0], bytes) or b"") + a[1]
            D[a[0]] = v
            return len(v)
        if cmd == "STRLEN":
            return len(self._get(db, a[0], bytes) or b"")
        if cmd == "INCR" or cmd == "INCRBY":
            inc = int(a[1]) if cmd == "INCRBY" else 1
            v = int(self._get(db, a[0], bytes) or b"0") + inc
            D[a[0]] = str(v).encode()
            return v
        if cmd == "DEL":
            n = 0
            for k in a:
                self._expired(db, k)
                if D.pop(k, None) is not None:
                    n += 1
                self.expiry[db].pop(k, None)
            return n
        if cmd == "EXISTS":
            return sum(1 for k in a if not self._expired(db, k) and k in D)
        if cmd == "EXPIRE":
            if self._expired(db, a[0]) or a[0] not in D:
                return 0
            self.expiry[db][a[0]] = time.time() + float(a[1])
            return 1
        if cmd == "TTL":
            if self._expired(db, a[0]) or a[0] not in D:
                return -2
            t = self.expiry[db].get(a[0])
            return -1 if t is None else int(round(t - time.time()))
        if cmd == "KEYS":
            pat = a[0].decode() if a else "*"
            out = []
            for k in list(D):
                if not self._expired(db, k) and fnmatch.fnmatchcase(k.decode("latin1"), pat):
                    out.append(k)
            return sorted(out)
        if cmd == "DBSIZE":
            return len([k for k in list(D) if not self._expired(db, k)])
        if cmd == "FLUSHALL":
            for d, e in zip(self.dbs, self.expiry):
                d.clear()
                e.clear()
            return "OK"
        if cmd == "FLUSHDB":
            D.clear()
            self.expiry[db].clear()
            return "OK"
        if cmd in ("RPUSH", "LPUSH"):
            lst = self._get(db, a[0], list)
            if lst is None:
                lst = []
                D[a[0]] = lst
            for v in a[1:]:
                if cmd == "RPUSH":
                    lst.append(v)
                else:
                    lst.insert(0, v)
            return len(lst)
        if cmd == "LRANGE":
            lst = self._get(db, a[0], list) or []
            st, en = int(a[1]), int(a[2])
            n = len(lst)
            st = max(n + st, 0) if st < 0 else st
            en = n + en if en < 0 else min(en, n - 1)
            return lst[st:en + 1] if st <= en else []
        if cmd == "LLEN":
            return len(self._get(db, a[0], list) or [])
        if cmd == "LTRIM":
            lst = self._get(db, a[0], list)
            if lst is None:
                return "OK"
            st, en = int(a[1]), int(a[2])
            n = len(lst)
            st = max(n + st, 0) if st < 0 else st
            en = n + en if en < 0 else min(en, n - 1)
            D[a[0]] = lst[st:en + 1] if st <= en else []
            return "OK"
        if cmd == "HSET" or cmd == "HMSET":
            h = self._get(db, a[0], dict)
            if h is None:
                h = {}
                D[a[0]] = h
            n = 0
            for i in range(1, len(a) - 1, 2):
                if a[i] not in h:
                    n += 1
                h[a[i]] = a[i + 1]
            return n if cmd == "HSET" else "OK"
        if cmd == "HGET":
            h = self._get(db, a[0], dict) or {}
            return h.get(a[1])
        if cmd == "HGETALL":
            h = self._get(db, a[0], dict) or {}
            out: List[bytes] = []
            for k, v in h.items():
                out += [k, v]
            return out
        if cmd == "HDEL":
            h = self._get(db, a[0], dict) or {}
            return sum(1 for k in a[1:] if h.pop(k, None) is not None)
        if cmd == "INFO":
            return b"# Server\r\nredis_version:6.2.3-fake\r\n"
        if cmd == "CONFIG":
            return []
        if cmd == "SAVE" or cmd == "BGSAVE":
            return "OK"
        return RedisError(f"ERR unknown command '{cmd.lower()}'")


class FakeRedisBackend:
    """In-process backend for `store.resp.Redis` (no sockets)."""

    def __init__(self, engine: FakeRedisEngine, password: str = "", db: int = 0):
        self.engine = engine
        self.session = {"auth": not engine.password, "db": 0}
        if password:
            r = engine.execute("AUTH", password, session=self.session)
            if isinstance(r, RedisError):
                raise r
        if db:
            engine.execute("SELECT", db, session=self.session)

    def execute(self, *cmd: Any) -> Any:
        r = self.engine.execute(*cmd, session=self.session)
        if isinstance(r, RedisError):
            raise r
        return r

    def pipeline(self, cmds: List[Any]) -> List[Any]:
        return [self.execute(*c) for c in cmds]


class _Handler(socketserver.BaseRequestHandler):
    def handle(self) -> None:
        engine: FakeRedisEngine = self.server.engine  # type: ignore[attr-defined]
        session = {"auth": not engine.password, "db": 0}
        p = Parser()
        sock: socket.socket = self.request
        self.server.clients.add(sock)  # type: ignore[attr-defined]
        while True:
            try:
                data = sock.recv(65536)
            except OSError:
                return
            if not data:
                return
            p.feed(data)
            out = []
            while True:
                cmd, ok = p.get()
                if not ok:
                    break
                if not cmd:
                    continue
                try:
                    r = engine.execute(*cmd, session=session)
                except ConnectionError:
                    return
                out.append(encode_reply(r))
                if cmd[0].upper() == b"QUIT":
                    sock.sendall(b"".join(out))
                    return
            if out:
                try:
                    sock.sendall(b"".join(out))
                except OSError:
                    return


class FakeRedisServer(socketserver.ThreadingMixIn, socketserver.TCPServer):
    daemon_threads = True
    allow_reuse_address = True

    def __init__(self, engine: Optional[FakeRedisEngine] = None, host: str = "127.0.0.1", port: int = 0):
        self.engine = engine or FakeRedisEngine()
        self.clients: set = set()
        super().__init__((host, port), _Handler)
        self._thread: Optional[threading.Thread] = None

    @property
    def addr(self) -> str:
        h, p = self.server_address[:2]
        return f"{h}:{p}"

    def start(self) -> "FakeRedisServer":
        self._thread = threading.Thread(target=self.serve_forever, daemon=True, name="fake-redis")
        self._thread.start()
        return self

    def stop(self) -> None:
        """Stop accepting and drop every client connection (a server crash, as seen by
        clients)."""
        self.shutdown()
        self.server_close()
        for c in list(self.clients):
            try:
                c.shutdown(socket.SHUT_RDWR)
                c.close()
            except OSError:
                pass
        self.clients.clear()
