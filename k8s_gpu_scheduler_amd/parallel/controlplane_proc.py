"""The bench's control plane (apiserver + scheduler + arrivals) in its own process.

In a real cluster the scheduler is a separate process from the kubelets/executors; here
that separation also matters for performance: rank 0 spends its CPU enqueueing its GPU's
pod kernels, and running the (Python) scheduler in the same interpreter would serialise
the two on the GIL.  The child is spawned BEFORE the parent touches the GPU (the parent
must never exec after GPU initialisation) and never initialises the GPU itself.

Protocol (multiprocessing Pipe, in order):
  ("schedule",)                -> child: finish the live epoch's pods, schedule the next
                                  epoch, reply ("placements", arr, sched_s, unscheduled)
  ("telemetry", per_gpu, ms)   -> child: update the TelemetryCache (no reply)
  ("reset_stats",)             -> child: zero sched_s / unscheduled counters, realign the
                                  planner's backlog (the bench drained every GPU before timing)
  ("interference_mae",)        -> child: reply ("interference_mae", online-model error summary)
  ("stop",)                    -> child exits
"""
from __future__ import annotations

import multiprocessing as mp
from typing import Any

import numpy as np


def _serve(conn: Any, kwargs: dict) -> None:
    from .podbench import ControlPlane
    cp = ControlPlane(**kwargs)
    while True:
        msg = conn.recv()
        kind = msg[0]
        if kind == "schedule":
            cp.finish_live()
            arr = cp.schedule_epoch()
            conn.send(("placements", arr, cp.sched_s, cp.unscheduled, cp.side_total_s))
        elif kind == "telemetry":
            cp.update_telemetry(msg[1], msg[2])
        elif kind == "reset_stats":
            cp.reset_stats()
        elif kind == "interference_mae":
            conn.send(("interference_mae", cp.interference_mae()))
        elif kind == "planner_stats":
            conn.send(("planner_stats", cp.planner_stats()))
        elif kind == "stop":
            conn.close()
            return


class ControlPlaneProc:
    """Same surface as podbench.ControlPlane, asynchronous scheduling."""

    def __init__(self, **kwargs: Any):
        ctx = mp.get_context("spawn")
        self._conn, child = ctx.Pipe()
        self._p = ctx.Process(target=_serve, args=(child, kwargs), daemon=True, name="gpusched-control-plane")
        self._p.start()
        child.close()
        self._outstanding = 0
        self.sched_s = 0.0
        self.side_total_s = 0.0
        self.unscheduled = 0

    def request_schedule(self) -> None:
        self._conn.send(("schedule",))
        self._outstanding += 1

    def get_schedule(self) -> np.ndarray:
        while True:
            # never block forever on a dead child: torchrun then tears the job down
            # instead of every rank hanging at the next placement broadcast
            while not self._conn.poll(1.0):
                if not self._p.is_alive():
                    raise RuntimeError(f"control-plane process exited (code {self._p.exitcode})")
            try:
                msg = self._conn.recv()
            except (EOFError, OSError) as e:
                raise RuntimeError(f"control-plane process connection lost: {e}") from e
            if msg[0] == "placements":
                self._outstanding -= 1
                _, arr, self.sched_s, self.unscheduled, self.side_total_s = msg
                return arr

    def schedule_epoch(self) -> np.ndarray:
        self.request_schedule()
        return self.get_schedule()

    def update_telemetry(self, per_gpu: np.ndarray, wall_ms: float) -> None:
        self._conn.send(("telemetry", np.asarray(per_gpu), float(wall_ms)))

    def reset_stats(self) -> None:
        self._conn.send(("reset_stats",))

    def interference_mae(self):
        while self._outstanding > 0:           # drain pending placements first
            self.get_schedule()
        self._conn.send(("interference_mae",))
        while not self._conn.poll(1.0):
            if not self._p.is_alive():
                raise RuntimeError(f"control-plane process exited (code {self._p.exitcode})")
        msg = self._conn.recv()
        return msg[1] if msg[0] == "interference_mae" else None

    def planner_stats(self):
        while self._outstanding > 0:
            self.get_schedule()
        self._conn.send(("planner_stats",))
        while not self._conn.poll(1.0):
            if not self._p.is_alive():
                raise RuntimeError(f"control-plane process exited (code {self._p.exitcode})")
        msg = self._conn.recv()
        return msg[1] if msg[0] == "planner_stats" else None

    def close(self) -> None:
        try:
            while self._outstanding > 0:
                self.get_schedule()
            self._conn.send(("stop",))
        except (OSError, EOFError):
            pass
        self._p.join(timeout=10)
        if self._p.is_alive():
            self._p.terminate()
