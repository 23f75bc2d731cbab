"""Idle slot-time of a bench run, split by where it happens.

Input: the per-pod timeline that `GPUSCHED_BENCH_TRACE=<file> python bench.py ...` writes
(podbench.py: one tuple per timed pod -- epoch collected, slot's first unit, workload, start and
end ms after the timed region's reference event, host ms when collected, SLO, host ms after
collect).  Every slot stream (first unit) is busy from its pods' start to end events; the rest
of [0, ms_total] is idle, split into

  fill     before the slot's first timed pod starts
  drain    after the slot's last pod ends, to the end of the timed window
  gap      between two consecutive pods of the slot (in-window starvation: the next pod was
           not enqueued yet, or it waited on another slot's pod for a unit)

Prints a JSON summary (ms per step and % of slot-time).  CPU only.
"""
from __future__ import annotations

import argparse
import json
from collections import defaultdict
from typing import Any, Dict, List


def split_idle(trace: Dict[str, Any], steps: int) -> Dict[str, Any]:
    total = float(trace["ms_total"])
    by_slot: Dict[int, List[tuple]] = defaultdict(list)
    for p in trace["pods"]:
        by_slot[int(p[1])].append((float(p[3]), float(p[4])))
    fill = drain = gap = busy = 0.0
    gaps_gt_1ms = transitions = 0
    for slot, iv in by_slot.items():
        iv.sort()
        fill += max(iv[0][0], 0.0)
        drain += max(total - max(e for _, e in iv), 0.0)
        end = iv[0][1]
        busy += iv[0][1] - iv[0][0]
        for s, e in iv[1:]:
            transitions += 1
            if s > end:
                gap += s - end
                gaps_gt_1ms += (s - end) > 1.0
            busy += e - s
            end = max(end, e)
    slots = max(len(by_slot), 1)
    cap = slots * total
    per = lambda v: round(v / steps, 4)          # noqa: E731
    pct = lambda v: round(100.0 * v / cap, 2)    # noqa: E731
    return {"slots": slots, "ms_total": round(total, 3), "steps": steps,
            "ms_per_step": {"busy": per(busy / slots), "fill": per(fill / slots), "drain": per(drain / slots),
                            "gap": per(gap / slots)},
            "pct_of_slot_time": {"busy": pct(busy), "fill": pct(fill), "drain": pct(drain), "gap": pct(gap)},
            "transitions": transitions, "gaps_over_1ms": gaps_gt_1ms}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    print(json.dumps(split_idle(json.load(open(a.trace)), a.steps), indent=1))


if __name__ == "__main__":
    main()
