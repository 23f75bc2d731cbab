"""Recommender clients and the scheduler-side prediction providers.

* `RecommenderClient` -- the Go wrappers `ImputeConfigurations(url, index)` /
  `ImputeInterference(url, index)` (reference pkg/recommender/go_client/pkg/client_call.go:11-37)
  but with one persistent channel and a deadline (the reference dials per call,
  SURVEY §2.9 #9).
* `PredictionProvider` -- what the GPU plugin consumes: `configurations(name)` /
  `interference(name)` -> {column: value}.
  - `RpcPredictions`: one RPC per lookup (parity mode; same call pattern as the
    reference's Score).
  - `CachedPredictions`: the whole completed matrices are pulled once per model version
    (ExportTable) or computed in-process from a `TrainedTable`; a lookup is then a dict
    hit + the reference's substring row match, memoised per request string.  Score does
    zero I/O (SURVEY §6.3 "the bar the MI355X build beats").
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

import grpc

from . import proto as P
from .tables import TrainedTable, find_index_for_request

log = logging.getLogger(__name__)


class RecommenderClient:
    def __init__(self, addr: str, timeout_s: float = 1.0, new_channel_per_call: bool = False):
        self.addr, self.timeout_s = addr, timeout_s
        self.new_channel_per_call = new_channel_per_call
        self._ch: Optional[grpc.Channel] = None
        self._lock = threading.Lock()

    def _channel(self) -> grpc.Channel:
        with self._lock:
            if self._ch is None:
                self._ch = grpc.insecure_channel(self.addr)
            return self._ch

    def _call(self, method: str, req: Any) -> Any:
        if self.new_channel_per_call:
            with grpc.insecure_channel(self.addr) as ch:
                return P.stub_method(ch, method)(req, timeout=self.timeout_s)
        return P.stub_method(self._channel(), method)(req, timeout=self.timeout_s)

    def impute_configurations(self, index: str) -> Any:
        return self._call(f"/{P.SERVICE}/ImputeConfigurations", P.Request(index=index))

    def impute_interference(self, index: str) -> Any:
        return self._call(f"/{P.SERVICE}/ImputeInterference", P.Request(index=index))

    def export_table(self, table: str) -> Any:
        return self._call(f"/{P.EXT_SERVICE}/ExportTable", P.TableRequest(table=table))

    def recommend_resources(self, pod: str, cu: int, hbm_gib: float, slo: float) -> Any:
        return self._call(f"/{P.EXT_SERVICE}/RecommendResources",
                          P.ResizeRequest(pod=pod, requested_cu=cu, requested_hbm_gib=hbm_gib, slo=slo))

    def version(self) -> Any:
        return self._call(f"/{P.EXT_SERVICE}/Version", P.Empty())

    def observe_corun(self, groups: List[Dict[str, Any]]) -> Any:
        """Send co-run groups (dicts: workloads, iters, ms[, start_ms, target, mfma_share,
        cu_fill]) for the
        recommender's online co-run model (ExportTable("corun") then serves the refined one)."""
        req = P.ObserveCorunRequest()
        for g in groups:
            x = req.groups.add()
            x.workloads.extend(g["workloads"])
            x.iters.extend(float(v) for v in g["iters"])
            x.ms.extend(float(v) for v in g["ms"])
            if g.get("start_ms") is not None:
                x.start_ms.extend(float(v) for v in g["start_ms"])
            if g.get("target") is not None:
                x.target.extend(bool(v) for v in g["target"])
            if g.get("mfma_share") is not None:
                x.mfma_share.extend(float(v) for v in g["mfma_share"])
            if g.get("cu_fill") is not None:
                x.cu_fill.extend(float(v) for v in g["cu_fill"])
        return self._call(f"/{P.EXT_SERVICE}/ObserveCorun", req)

    def observe_interference(self, observations: List[Tuple[str, List[str], float]]) -> Any:
        """Send (pod, co-runner pods, throughput loss) observations for online learning."""
        req = P.ObserveRequest()
        for pod, others, loss in observations:
            req.observations.add(pod=pod, co_runners=list(others), loss=float(loss))
        return self._call(f"/{P.EXT_SERVICE}/ObserveInterference", req)

    def close(self) -> None:
        with self._lock:
            if self._ch is not None:
                self._ch.close()
                self._ch = None


def reply_to_map(reply: Any) -> Dict[str, float]:
    """zip(columns, result) like reference gpu_plugins.go:322-325 (an unknown index reply
    has result=[0] and no columns -> empty map)."""
    return {c: float(v) for c, v in zip(reply.columns, reply.result)}


class PredictionProvider:
    def configurations(self, name: str) -> Dict[str, float]:
        raise NotImplementedError

    def interference(self, name: str) -> Dict[str, float]:
        raise NotImplementedError

    def corun(self) -> Any:
        """The multi-way co-run model (models.corun.CorunModel) the recommender serves, or
        None (then Score falls back to the reference's pairwise interference terms)."""
        return None


class RpcPredictions(PredictionProvider):
    def __init__(self, client: RecommenderClient):
        self.client = client
        self.calls = 0

    def configurations(self, name: str) -> Dict[str, float]:
        self.calls += 1
        return reply_to_map(self.client.impute_configurations(name))

    def interference(self, name: str) -> Dict[str, float]:
        self.calls += 1
        return reply_to_map(self.client.impute_interference(name))


class _Tab:
    def __init__(self, index: List[str], columns: List[str], rows: List[List[float]], version: str):
        self.index, self.columns, self.version = index, columns, version
        self.by_label = {lab: dict(zip(columns, vals)) for lab, vals in zip(index, rows)}
        self.memo: Dict[str, Dict[str, float]] = {}

    def lookup(self, request: str) -> Dict[str, float]:
        hit = self.memo.get(request)
        if hit is not None:
            return hit
        lab = find_index_for_request(request.replace("-", "_"), self.index)
        out = self.by_label.get(lab, {}) if lab else {}
        self.memo[request] = out
        return out


class CachedPredictions(PredictionProvider):
    """In-process, zero-I/O predictions.  Source: a RecommenderClient (ExportTable, pulled
    again every `refresh_s` by a background thread so a retrained model version reaches the
    scheduler -- the reference sees new versions because it calls the recommender per
    prediction) or local TrainedTables.  An unreachable recommender (it may start after the
    scheduler) is not fatal: lookups return no predictions until the first pull succeeds,
    retried every `retry_s`."""

    def __init__(self, client: Optional[RecommenderClient] = None,
                 conf: Optional[TrainedTable] = None, intf: Optional[TrainedTable] = None,
                 refresh_s: float = 30.0, retry_s: float = 2.0, background: bool = True, corun: Any = None):
        self.client = client
        self.refresh_s = refresh_s
        self.retry_s = retry_s
        self._last = 0.0
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._conf: Optional[_Tab] = None
        self._intf: Optional[_Tab] = None
        self._corun: Any = corun            # models.corun.CorunModel
        if conf is not None:
            self._conf = _Tab(conf.table.index, conf.table.columns, conf.completed().tolist(), conf.version)
        if intf is not None:
            self._intf = _Tab(intf.table.index, intf.table.columns, intf.completed().tolist(), intf.version)
        if client is not None:
            ok = self.try_refresh(force=True)
            if background:
                self._thread = threading.Thread(target=self._loop, args=(ok,), name="predictions-refresh",
                                                daemon=True)
                self._thread.start()

    def _loop(self, ok: bool) -> None:
        while not self._stop.wait(self.refresh_s if ok else self.retry_s):
            ok = self.try_refresh(force=True)

    def close(self) -> None:
        self._stop.set()

    def try_refresh(self, force: bool = False) -> bool:
        try:
            self.refresh(force)
            return self._conf is not None and self._intf is not None
        except Exception as e:
            log.warning("predictions refresh failed (keeping the previous tables): %s", e)
            return False

    def refresh(self, force: bool = False) -> None:
        if self.client is None:
            return
        now = time.monotonic()
        if not force and now - self._last < self.refresh_s:
            return
        self._last = now
        for name in ("configurations", "interference"):
            t = self.client.export_table(name)
            cur = self._conf if name == "configurations" else self._intf
            if cur is not None and cur.version == t.version:
                continue
            tab = _Tab([r.index for r in t.rows], list(t.columns), [list(r.values) for r in t.rows], t.version)
            if name == "configurations":
                self._conf = tab
            else:
                self._intf = tab
        # the co-run model (an older recommender answers with an empty table: keep what we have)
        try:
            t = self.client.export_table("corun")
        except Exception as e:
            log.debug("co-run model unavailable: %s", e)
            return
        cur = self._corun
        if t.rows and (cur is None or cur.version != t.version):
            from ..models.corun import CorunModel
            m = CorunModel.from_table([r.index for r in t.rows], list(t.columns), [list(r.values) for r in t.rows],
                                      t.version)
            if m is not None:
                self._corun = m

    def configurations(self, name: str) -> Dict[str, float]:
        return self._conf.lookup(name) if self._conf else {}

    def interference(self, name: str) -> Dict[str, float]:
        return self._intf.lookup(name) if self._intf else {}

    def corun(self) -> Any:
        return self._corun

    def install_corun(self, model: Any) -> None:
        """Swap in a new co-run model (e.g. the online-refined one)."""
        self._corun = model

    def tables(self) -> "tuple[Optional[_Tab], Optional[_Tab]]":
        return self._conf, self._intf

    def version(self) -> tuple:
        """Changes whenever a new configurations / interference table or co-run model is
        installed (callers memoising per-pod lookups key their memo by it)."""
        c, i, m = self._conf, self._intf, self._corun
        return (id(c), c.version if c else None, id(i), i.version if i else None, id(m))

    def install_interference(self, index: List[str], columns: List[str], rows: List[List[float]],
                             version: str) -> None:
        """Swap in a new interference table (e.g. the online-learned one)."""
        self._intf = _Tab(list(index), list(columns), rows, version)
