"""Lease-based leader election (coordination.k8s.io/v1 Lease).

The reference inherits kube-scheduler's leader election, configured in its profile
(`leaderElection: {leaderElect: true, resourceName: gpu-scheduler, resourceNamespace:
kube-system}`, reference deploy/scheduler.yaml:10-13).  Same semantics here: a replica
acquires the Lease when it is unheld or its renewTime + leaseDurationSeconds has
passed, renews every retry period, and steps down (callback) when a renewal cannot be
written before the renew deadline.  Optimistic concurrency (resourceVersion) makes the
acquire race-free across replicas.
"""
from __future__ import annotations

import datetime as dt
import logging
import math
import threading
import time
from typing import Callable, Optional

from .client import AlreadyExists, ApiError, Conflict, KubeClient, NotFound

log = logging.getLogger(__name__)


def _now() -> dt.datetime:
    return dt.datetime.now(dt.timezone.utc)


def _fmt(t: dt.datetime) -> str:
    return t.strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def _parse(s: str) -> dt.datetime:
    for f in ("%Y-%m-%dT%H:%M:%S.%fZ", "%Y-%m-%dT%H:%M:%SZ"):
        try:
            return dt.datetime.strptime(s, f).replace(tzinfo=dt.timezone.utc)
        except ValueError:
            continue
    return dt.datetime.fromtimestamp(0, dt.timezone.utc)


class LeaderElector:
    def __init__(self, client: KubeClient, name: str, namespace: str, identity: str,
                 lease_duration_s: float = 15.0, renew_deadline_s: float = 10.0, retry_period_s: float = 2.0,
                 on_started_leading: Optional[Callable[[], None]] = None,
                 on_stopped_leading: Optional[Callable[[], None]] = None):
        self.client, self.name, self.ns, self.identity = client, name, namespace, identity
        self.lease_duration_s, self.renew_deadline_s, self.retry_period_s = lease_duration_s, renew_deadline_s, retry_period_s
        self.on_started, self.on_stopped = on_started_leading, on_stopped_leading
        self.leading = False
        self._stop = threading.Event()
        self._last_renew = 0.0

    def try_acquire_or_renew(self) -> bool:
        now = _now()
        spec = {"holderIdentity": self.identity, "leaseDurationSeconds": max(1, int(math.ceil(self.lease_duration_s))),
                "renewTime": _fmt(now)}
        try:
            lease = self.client.get("leases", self.name, self.ns)
        except NotFound:
            spec["acquireTime"] = _fmt(now)
            spec["leaseTransitions"] = 0
            try:
                self.client.create("leases", {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                                              "metadata": {"name": self.name, "namespace": self.ns}, "spec": spec},
                                   self.ns)
                return True
            except (AlreadyExists, Conflict):
                return False
        cur = lease.get("spec") or {}
        holder = cur.get("holderIdentity", "")
        expired = _parse(cur.get("renewTime", "")) + dt.timedelta(
            seconds=float(cur.get("leaseDurationSeconds", self.lease_duration_s))) < now
        if holder and holder != self.identity and not expired:
            return False
        if holder != self.identity:
            spec["acquireTime"] = _fmt(now)
            spec["leaseTransitions"] = int(cur.get("leaseTransitions", 0)) + 1
        else:
            spec["acquireTime"] = cur.get("acquireTime", _fmt(now))
            spec["leaseTransitions"] = int(cur.get("leaseTransitions", 0))
        lease["spec"] = spec
        try:
            self.client.update("leases", lease, self.ns)
            return True
        except (Conflict, ApiError):
            return False

    def step(self) -> bool:
        ok = self.try_acquire_or_renew()
        mono = time.monotonic()
        if ok:
            self._last_renew = mono
            if not self.leading:
                self.leading = True
                log.info("%s became leader of %s/%s", self.identity, self.ns, self.name)
                if self.on_started:
                    self.on_started()
        elif self.leading and mono - self._last_renew > self.renew_deadline_s:
            self.leading = False
            log.warning("%s lost leadership of %s/%s", self.identity, self.ns, self.name)
            if self.on_stopped:
                self.on_stopped()
        return self.leading

    def run(self) -> None:
        while not self._stop.is_set():
            try:
                self.step()
            except Exception as e:
                log.warning("leader election error: %s", e)
            self._stop.wait(self.retry_period_s)

    def start(self) -> "LeaderElector":
        threading.Thread(target=self.run, daemon=True, name="leader-elector").start()
        return self

    def stop(self, release: bool = True) -> None:
        self._stop.set()
        if release and self.leading:
            try:
                lease = self.client.get("leases", self.name, self.ns)
                if (lease.get("spec") or {}).get("holderIdentity") == self.identity:
                    lease["spec"]["holderIdentity"] = ""
                    self.client.update("leases", lease, self.ns)
            except ApiError:
                pass
            self.leading = False
