"""Garbage-collector policy of the long-running control-plane processes.

The scheduler's live set -- informer caches, the node ledger, co-run model, timelines, compiled
plugin state -- is built at start-up and then mostly only grows by the pods it handles.  With
CPython's default policy every gen-2 collection walks all of it: on the box CPU a ~1 ms pause
that lands inside an 8-GPU epoch's planning every few epochs (tools/cp_breakdown.py, CP_GC=off:
the burst planner's mean cost per epoch 3.49 -> 2.47 ms at effort level 1).  `settle()` after
start-up collects once and moves every surviving object to the permanent generation
(gc.freeze), so later collections only scan what was allocated since, and raises the gen-0
threshold so short-lived per-cycle garbage (cycle states, status objects) is collected in
fewer, larger batches.  Reference cycles are still collected.
"""
from __future__ import annotations

import gc

GEN0_THRESHOLD = 20000


def settle(gen0: int = GEN0_THRESHOLD) -> None:
    gc.collect()
    gc.freeze()
    t = gc.get_threshold()
    gc.set_threshold(max(int(gen0), t[0]), t[1], t[2])
