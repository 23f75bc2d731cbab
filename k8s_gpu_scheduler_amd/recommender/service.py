"""Recommender gRPC server.

Behaviour of the reference server (reference pkg/recommender/recom_server.py):
* env CONFIGURATIONS_DATA_PATH / INTERFERENCE_DATA_PATH / PORT (50051) / JOB_DELAY (30)
  (:30-52);
* fit one imputer per matrix at start (:215-235), retrain in the background when the
  file's md5 changes (:74-134), swap the new model in (:141-148);
* RPC: `-`→`_`, first row label that is a substring, impute that row, reply
  (values, column names); unknown index or no model -> result=[0], columns=[]
  (:150-170).

Fixes: existence is checked before hashing, the swap is under a lock
(§5.2 race), the retrain loop survives exceptions, the thread pool size is configurable.
Extensions (separate `gpusched.recommender.Extended` service): ExportTable (completed
matrices for the scheduler's in-process cache, and table "corun": the multi-way co-run model
of models.corun, one row per workload), RecommendResources (resize from Redis history),
Version.
"""
from __future__ import annotations

import json
import logging
import os
import threading
from concurrent import futures
from typing import Any, Callable, Dict, List, Optional

import grpc
import numpy as np

from ..api import constants as C
from . import proto as P
from .resize import recommend
from .tables import Table, TrainedTable, file_version

log = logging.getLogger(__name__)

DEFAULT_CONF = "configurations_train.ods"
DEFAULT_INTF = "interference_train.ods"


class ModelSlot:
    """One matrix + model with md5-driven hot reload and a locked swap."""

    def __init__(self, name: str, path: str, kind: str = "iterative", **model_kw: Any):
        self.name, self.path, self.kind, self.model_kw = name, path, kind, model_kw
        self._lock = threading.Lock()
        self.current: Optional[TrainedTable] = None
        self.version: Optional[str] = None         # version served (file md5, or online-N)
        self.file_version: Optional[str] = None    # md5 of the training file last fitted

    def load_if_changed(self, store: Any = None) -> bool:
        """Re-fit when the training file's md5 changed.  With a Redis `store`, every newly
        trained version is persisted (`schema.model_key(name)`: version + training table),
        and a missing training file falls back to the last persisted version -- so a
        restarted recommender serves immediately."""
        v = file_version(self.path)
        if v is None:
            if store is not None and self.version is None:
                return self._load_persisted(store)
            log.info("%s: train data not found at %s", self.name, self.path)
            return False
        if v == self.file_version:
            return False
        table = Table.read_tsv(self.path)
        trained = TrainedTable.fit(table, self.kind, v, **self.model_kw)
        with self._lock:
            self.current, self.version, self.file_version = trained, v, v
        if store is not None:
            try:
                from ..store import schema
                store.set(schema.model_key(self.name), json.dumps(
                    {"version": v, "kind": self.kind, "table": table.to_json()}, separators=(",", ":")))
            except Exception as e:
                log.warning("%s: persisting model version %s failed: %s", self.name, v[:8], e)
        log.info("%s: trained version %s (%d x %d)", self.name, v[:8], len(trained.table.index),
                 len(trained.table.columns))
        return True

    def _load_persisted(self, store: Any) -> bool:
        from ..store import schema
        try:
            raw = store.get(schema.model_key(self.name))
        except Exception as e:
            log.info("%s: no persisted model (%s)", self.name, e)
            return False
        if not raw:
            return False
        d = json.loads(raw)
        trained = TrainedTable.fit(Table.from_json(d["table"]), self.kind, d["version"], **self.model_kw)
        with self._lock:
            self.current, self.version = trained, d["version"]
        log.info("%s: restored persisted version %s", self.name, d["version"][:8])
        return True

    def set_table(self, table: Table, version: str = "mem") -> None:
        trained = TrainedTable.fit(table, self.kind, version, **self.model_kw)
        with self._lock:
            self.current, self.version = trained, version

    def serve_table(self, table: Table, version: str) -> None:
        """Serve a learned table (no NaN) without touching the file bookkeeping: a later
        change of the training file still re-fits from the file."""
        self.set_table(table, version)

    def get(self) -> Optional[TrainedTable]:
        with self._lock:
            return self.current


class CorunSlot:
    """The multi-way co-run model (models.corun, a JSON file) with the same md5-driven hot
    reload and locked swap as the matrices; served through ExportTable("corun")."""

    def __init__(self, path: str):
        self.path = path
        self._lock = threading.Lock()
        self.model: Any = None
        self.version: Optional[str] = None
        self.file_version: Optional[str] = None
        self.file_label = ""

    def file_version_label(self) -> str:
        """The version of the file model (what online / cold-start versions extend)."""
        return self.file_label or (self.version or "").split("+")[0]

    def load_if_changed(self) -> bool:
        v = file_version(self.path) if self.path else None
        if v is None or v == self.file_version:
            return False
        from ..models.corun import CorunModel
        m = CorunModel.load(self.path)
        if m is None:
            return False
        with self._lock:
            self.model, self.file_version = m, v
            self.version = self.file_label = f"{m.version}@{v[:8]}"
        log.info("corun: loaded %s (%d workloads)", self.version, len(m.names))
        return True

    def get(self) -> Any:
        with self._lock:
            return self.model

    def serve(self, model: Any, version: str) -> None:
        """Serve an online-refined model (the file bookkeeping is untouched: a changed file
        is loaded again and replaces it)."""
        with self._lock:
            self.model, self.version = model, version


class RecommenderService:
    def __init__(self, configurations_path: str = "", interference_path: str = "",
                 kind: str = "iterative", job_delay_s: float = C.RECOMMENDER_JOB_DELAY_S,
                 history_source: Optional[Callable[[str], Any]] = None, model: str = "MI355X",
                 corun_path: str = ""):
        self.conf = ModelSlot("configurations", configurations_path, kind)
        self.intf = ModelSlot("interference", interference_path, kind)
        self.corun = CorunSlot(corun_path)
        self._corun_online: Any = None      # models.corun.OnlineCorun on the served file model
        self._corun_online_base: Optional[str] = None
        # workload -> alone observations (ms per iteration, MFMA share or None) of workloads
        # the co-run model file does not know (cold start, models.coldstart)
        self._cold: Dict[str, List[Any]] = {}
        self._corun_refit_mode: Any = "process"
        # OnlineCorun knobs (from_env: CORUN_MIN_OBS, CORUN_MIN_CALIB, CORUN_REFIT_EVERY)
        self.corun_online_kw: Dict[str, int] = {}
        self.job_delay_s = job_delay_s
        self.history_source = history_source
        self.model = model
        self.store: Any = None          # Redis: persisted model versions (set by the CLI / tests)
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.calls = 0
        self._online: Any = None            # recommender.online.OnlineInterference
        self._online_base: Optional[str] = None
        self._online_lock = threading.Lock()

    @classmethod
    def from_env(cls, **kw: Any) -> "RecommenderService":
        """Env as the reference's server, plus CORUN_MODEL_PATH (default: the shipped MI355X
        co-run model, data/corun_mi355x.json)."""
        from ..models.corun import DATA as CORUN_DATA
        kw.setdefault("corun_path", os.getenv("CORUN_MODEL_PATH", CORUN_DATA))
        svc = cls(os.getenv("CONFIGURATIONS_DATA_PATH", DEFAULT_CONF),
                  os.getenv("INTERFERENCE_DATA_PATH", DEFAULT_INTF),
                  job_delay_s=float(os.getenv("JOB_DELAY", C.RECOMMENDER_JOB_DELAY_S)), **kw)
        for env, k in (("CORUN_MIN_OBS", "min_obs"), ("CORUN_MIN_CALIB", "min_calib"),
                       ("CORUN_REFIT_EVERY", "refit_every")):
            if os.getenv(env):
                svc.corun_online_kw[k] = int(os.environ[env])
        return svc

    # ------------------------------------------------------------------ training loop
    def train(self) -> None:
        for slot in (self.conf, self.intf):
            try:
                changed = slot.load_if_changed(self.store)
                if changed and slot is self.intf and self.store is not None:
                    self.restore_online()
            except Exception as e:
                log.warning("%s: training failed: %s", slot.name, e)
        try:
            self.corun.load_if_changed()
        except Exception as e:
            log.warning("corun: loading %s failed: %s", self.corun.path, e)

    def start_retrain_loop(self) -> None:
        def loop() -> None:
            while not self._stop.wait(self.job_delay_s):
                self.train()
        self._thread = threading.Thread(target=loop, daemon=True, name="recommender-retrain")
        self._thread.start()

    def stop(self) -> None:
        self._stop.set()

    # ------------------------------------------------------------------ RPC logic
    @staticmethod
    def _impute(slot: ModelSlot, index: str) -> Any:
        self_reply = P.Reply()
        t = slot.get()
        if t is None:
            self_reply.result.append(0)
            return self_reply
        res = t.lookup(index)
        if not res:
            self_reply.result.append(0)
            return self_reply
        return P.set_protobuf_reply(list(res.values()), list(res.keys()), self_reply)

    def ImputeConfigurations(self, request: Any, context: Any) -> Any:
        self.calls += 1
        return self._impute(self.conf, request.index)

    def ImputeInterference(self, request: Any, context: Any) -> Any:
        self.calls += 1
        return self._impute(self.intf, request.index)

    def ExportTable(self, request: Any, context: Any) -> Any:
        out = P.Table()
        if request.table == "corun":
            m = self.corun.get()
            if m is None:
                return out
            out.columns.extend(m.table_columns())
            out.version = self.corun.version or ""
            for lab, vals in zip(m.names, m.table_rows()):
                r = out.rows.add()
                r.index = lab
                r.values.extend(float(v) for v in vals)
            return out
        slot = self.conf if request.table in ("", "configurations") else self.intf
        t = slot.get()
        if t is None:
            return out
        full = t.completed()
        out.columns.extend(t.table.columns)
        out.version = t.version or ""
        for lab, vals in zip(t.table.index, full):
            r = out.rows.add()
            r.index = lab
            r.values.extend(float(v) for v in vals)
        return out

    def RecommendResources(self, request: Any, context: Any) -> Any:
        hist = self.history_source(request.pod) if self.history_source else []
        t = self.conf.get()
        conf = t.lookup(request.pod) if t is not None else None
        adv = recommend(hist or [], request.requested_cu or 256, request.requested_hbm_gib or 0.0,
                        request.slo, conf, self.model)
        return P.ResizeReply(recommended_cu=adv.cu, recommended_hbm_gib=adv.hbm_gib, samples=adv.samples,
                             reason=adv.reason)

    def ObserveInterference(self, request: Any, context: Any) -> Any:
        """Online interference learning (recommender.online): each observation is a pod's
        throughput loss next to its co-runners; the refitted matrix becomes the served
        interference table (version online-N) until the training file changes."""
        from .online import OnlineInterference
        from .tables import find_index_for_request
        with self._online_lock:
            t = self.intf.get()
            if t is None:
                return P.ObserveReply(accepted=0, interference="", observations=0)
            base = self.intf.file_version or self.intf.version
            if self._online is None or self._online_base != base:
                self._online = OnlineInterference(t.table.index, t.table.columns, t.completed(),
                                                  refit_every=max(1, int(os.getenv("ONLINE_REFIT_EVERY", "32"))),
                                                  scale=os.getenv("ONLINE_PRIOR_SCALE", "0") == "1")
                self._online_base = base
            on = self._online
            cols = list(t.table.columns)
            accepted, refit = 0, False
            for ob in request.observations:
                lab = find_index_for_request(ob.pod.replace("-", "_"), t.table.index)
                others = []
                for c in ob.co_runners:
                    nm = c.replace("-", "_")
                    j = next((k for k, col in enumerate(cols) if col in nm), None)
                    if j is not None:
                        others.append(j)
                if not lab or not others:
                    continue
                refit |= on.observe(t.table.index.index(lab), others, float(ob.loss))
                accepted += 1
            if refit:
                learned = Table(list(t.table.index), cols, np.asarray(on.rows()))
                version = f"online-{on.version}"
                self.intf.serve_table(learned, version)
                self._persist_online(learned, version, base)
            return P.ObserveReply(accepted=accepted, interference=self.intf.version or "",
                                  observations=int(on.mae()["n"]))

    def _persist_online(self, table: Table, version: str, base: Optional[str]) -> None:
        """Keep the learned interference table in Redis so a restarted
        recommender serves it again -- as long as the training file it was learned on top
        of (`base` md5) is still the current one."""
        if self.store is None:
            return
        try:
            from ..store import schema
            self.store.set(schema.model_key("interference-online"), json.dumps(
                {"version": version, "base": base, "table": table.to_json()}, separators=(",", ":")))
        except Exception as e:
            log.warning("persisting the online interference table failed: %s", e)

    def restore_online(self) -> bool:
        """Serve a persisted online table learned on the current training file."""
        if self.store is None or self.intf.get() is None:
            return False
        from ..store import schema
        try:
            raw = self.store.get(schema.model_key("interference-online"))
        except Exception:
            return False
        if not raw:
            return False
        d = json.loads(raw)
        if d.get("base") != (self.intf.file_version or self.intf.version):
            return False
        self.intf.serve_table(Table.from_json(d["table"]), d["version"])
        log.info("interference: restored online table %s", d["version"])
        return True

    def ObserveCorun(self, request: Any, context: Any) -> Any:
        """Online co-run learning (models.corun.OnlineCorun, refits in a worker process): each
        group is one GPU's co-running pods with their measured wall ms; the refined model is
        served through ExportTable("corun") under version `<file version>+online-N` until
        the model file changes."""
        from ..models.corun import OnlineCorun
        reply = P.ObserveCorunReply()
        with self._online_lock:
            if self.corun.file_version is None:
                self.corun.load_if_changed()
            base = self.corun.get()
            if base is None:
                return reply
            if self._corun_online is None or self._corun_online_base != self.corun.file_version:
                # the served model may already be an online one: learn on the file's model
                from ..models.corun import CorunModel
                fm = CorunModel.load(self.corun.path) if self.corun.path else base
                self._corun_online = OnlineCorun(fm or base, background=self._corun_refit_mode,
                                                 **self.corun_online_kw)
                self._corun_online_base = self.corun.file_version
                reload_cold = bool(self._cold)      # a new model file: cold-start the known rows again
            else:
                reload_cold = False
            # cold start (models.coldstart): a workload the model does not know that ran
            # ALONE on its device (a 1-pod group) gets a row imputed from its alone profile
            fresh = reload_cold
            for g in request.groups:
                if len(g.workloads) == 1 and len(g.ms) == 1 and len(g.iters) == 1 and g.ms[0] > 0 \
                        and g.iters[0] > 0 and self._corun_online.base.wid(g.workloads[0]) < 0:
                    mf = float(g.mfma_share[0]) if len(g.mfma_share) == 1 and g.mfma_share[0] >= 0 else None
                    cf = float(g.cu_fill[0]) if len(g.cu_fill) == 1 and g.cu_fill[0] > 0 else None
                    self._cold.setdefault(g.workloads[0], []).append((g.ms[0] / g.iters[0], mf, cf))
                    fresh = True
            if fresh:
                self._cold_start_rows()
            on = self._corun_online
            base = on.base
            for g in request.groups:
                w = [base.wid(n) for n in g.workloads]
                k = len(w)
                if not k or min(w) < 0 or len(g.ms) != k or len(g.iters) != k:
                    continue
                st = list(g.start_ms) if len(g.start_ms) == k else None
                tg = list(g.target) if len(g.target) == k else None
                on.observe_group(w, list(g.iters), list(g.ms), st, tg)
                reply.accepted += 1
            if on.model is not self.corun.get() and (on.refits or fresh):
                ver = f"{self.corun.file_version_label()}" + (f"+cold-{len(self._cold)}" if self._cold else "")
                self.corun.serve(on.model, ver + (f"+online-{on.version}" if on.refits else ""))
            reply.corun = self.corun.version or ""
            reply.observations = int(on.err["n"])
        return reply

    def _cold_start_rows(self) -> None:
        """Rebuild the online co-run learner on the file model plus every cold-started
        workload (median alone ms per iteration of its alone observations), carrying the
        learner's state over: its observation window, error bookkeeping and per-workload
        refit parameters (new workloads start at 0: the imputed row as is)."""
        import numpy as np
        from ..models.coldstart import with_workload
        from ..models.corun import CorunModel, OnlineCorun
        old = self._corun_online
        fm = CorunModel.load(self.corun.path) if self.corun.path else old.base
        ext = fm
        # arrival order (dicts keep insertion order), never re-sorted: a new workload's row is
        # appended after every earlier cold-started one
        for name, obs in self._cold.items():
            if fm.wid(name) >= 0:
                continue
            a = float(np.median([x[0] for x in obs]))
            shares = [x[1] for x in obs if x[1] is not None]
            fills = [x[2] for x in obs if len(x) > 2 and x[2] is not None]
            ext = with_workload(ext, name, a, float(np.median(shares)) if shares else None,
                                fill=float(np.median(fills)) if fills else None)
        on = OnlineCorun(ext, background=self._corun_refit_mode, **self.corun_online_kw)
        # carry the learner's state over BY NAME (copying by position shifted an
        # earlier cold row's refit parameters and observations onto another workload)
        old_names = list(old.base.names)
        n_old = len(old_names)
        x = np.asarray(old._x)
        new_of_old = [ext.names.index(nm) if nm in ext.names else -1 for nm in old_names]
        nx = np.zeros(len(ext.names) + (len(x) - n_old))
        for i, j in enumerate(new_of_old):
            if j >= 0:
                nx[j] = x[i]
        nx[len(ext.names):] = x[n_old:]
        on._x = nx
        obs = []
        for o in old._obs:
            w = [new_of_old[i] if 0 <= i < n_old else -1 for i in o[0]]
            if min(w, default=-1) >= 0:
                obs.append((tuple(w),) + tuple(o[1:]))
        on._obs, on.err, on.version, on.refits, on.time_scale = obs, dict(old.err), old.version, \
            old.refits, old.time_scale
        n = len(ext.names)
        on.model = CorunModel(ext.names, ext.alone_ms * np.exp(on._x[:n]) * on.time_scale,
                              ext.u * np.exp(on._x[n]), ext.v, dict(ext.meta))
        self._corun_online = on
        log.info("corun: cold-started %s", list(self._cold))

    def Version(self, request: Any, context: Any) -> Any:
        return P.VersionReply(configurations=self.conf.version or "", interference=self.intf.version or "",
                              model=self.conf.kind, corun=self.corun.version or "")

    # ------------------------------------------------------------------ server
    def make_server(self, port: int = C.RECOMMENDER_PORT, workers: int = C.RECOMMENDER_WORKERS,
                    host: str = "[::]") -> "tuple[grpc.Server, int]":
        server = grpc.server(futures.ThreadPoolExecutor(max_workers=workers))
        server.add_generic_rpc_handlers((
            P.generic_handler(P.SERVICE, {"ImputeConfigurations": self.ImputeConfigurations,
                                          "ImputeInterference": self.ImputeInterference}),
            P.generic_handler(P.EXT_SERVICE, {"ExportTable": self.ExportTable,
                                              "RecommendResources": self.RecommendResources,
                                              "Version": self.Version,
                                              "ObserveInterference": self.ObserveInterference,
                                              "ObserveCorun": self.ObserveCorun}),
        ))
        bound = server.add_insecure_port(f"{host}:{port}")
        server.start()
        return server, bound


def serve(port: int = C.RECOMMENDER_PORT, workers: int = C.RECOMMENDER_WORKERS) -> None:
    svc = RecommenderService.from_env()
    svc.train()
    svc.start_retrain_loop()
    server, bound = svc.make_server(port, workers)
    log.info("recommender listening on %d", bound)
    server.wait_for_termination()
