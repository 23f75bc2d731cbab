"""SLO ceiling of the bench's arrivals: planner vs greedy vs a hindsight oracle.

The bench's SLO attainment (57.5 % at N=1) had nothing to be judged against.  This tool replays
one run's arrivals -- the placements dump of `bench.py --dump-placements F` (every epoch's pods:
workload, iterations, SLO, and the GPU / CU slot the scheduler gave them) -- through the co-run
model's pipeline simulator (parallel.modelpipe.ModelPipelineExecutor, noise 0: the bench's
launch-ahead loop with the model as the truth) under different placements of the SAME pods:

  planner    the slots (and GPUs) the scheduler chose in that run
  fixed      arrival order onto the slots in turn (no placement intelligence)
  lpt        longest predicted pod first onto the slot with the least predicted work (the
             executor's old LPT re-slotting; a throughput-greedy policy blind to SLOs)
  greedy     (--greedy F) the placements of a second dump, e.g. `--plan-bursts 0`
  myopic     an ONLINE policy with the model as the truth: each epoch takes the slot permutation
             (N=1) that maximises (SLOs met, -time) over the pods placed so far, knowing nothing
             of later arrivals -- how much of the oracle's gain needs no hindsight
  oracle     hindsight search over every epoch's placement: coordinate descent over the 24
             slot permutations of each epoch (N=1) or pairwise pod swaps between GPUs / slots
             (N > 1), from every policy above as a start, maximising (SLOs met, -time) over the
             timed epochs with every later epoch's co-running known -- a LOWER bound on the true
             optimum (a local optimum of an exact objective), which is what "the planner is
             within x points of the oracle" needs

Writes --out (JSON) and prints one line per policy.  CPU only (native _core).
"""
from __future__ import annotations

import argparse
import collections
import itertools
import json
import os
import random
import sys
import time
from typing import Any, Dict, List, Sequence, Tuple

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_gpu_scheduler_amd.models import workloads as W  # noqa: E402
from k8s_gpu_scheduler_amd.parallel.executor import PodRun  # noqa: E402
from k8s_gpu_scheduler_amd.parallel.modelpipe import ModelPipelineExecutor  # noqa: E402

Pod = Tuple[int, int, float, int]          # workload id, iterations, SLO (it/s), n_units
Place = Tuple[int, int]                     # (gpu, first unit)


def load(path: str) -> Tuple[List[List[Pod]], List[List[Place]], List[bool], Dict[str, Any]]:
    d = json.load(open(path))
    names = d["workloads"]
    assert names == list(W.NAMES), "dump from another workload catalog"
    pods, places, timed = [], [], []
    for e in d["epochs"]:
        pods.append([(int(r[3]), int(r[4]), r[5] / 1000.0, int(r[2])) for r in e["arr"] if int(r[0]) >= 0])
        places.append([(int(r[0]), int(r[1])) for r in e["arr"] if int(r[0]) >= 0])
        timed.append(bool(e["timed"]))
    return pods, places, timed, d


def simulate(pods: List[List[Pod]], places: List[List[Place]], timed: Sequence[bool], lookahead: int = 2,
             model: Any = None, outcomes: Any = None) -> Tuple[int, int, float]:
    """(SLOs met, pods, simulated ms) over the timed epochs: the bench's loop -- warm-up epochs,
    drained, then the timed ones, `lookahead` epochs in flight -- on the model pipeline."""
    ex = ModelPipelineExecutor(model=model, noise=0.0)
    ok = n = 0
    t0 = t1 = 0.0
    pid = 0
    for phase in (False, True):
        pend: "collections.deque[List[PodRun]]" = collections.deque()
        if phase:
            t0 = ex.elapsed_ms
        for ep, pl, tm in zip(pods, places, timed):
            if tm != phase:
                continue
            runs = []
            for (wid, it, slo, nu), (g, u0) in zip(ep, pl):
                runs.append(PodRun(pid, W.NAMES[wid], u0, nu, it, slo, masked=False, gpu=g))
                pid += 1
            ex.launch_epoch(runs)
            pend.append(runs)
            while len(pend) > lookahead:
                rs = pend.popleft()
                ex.wait_epoch(rs)
                if phase:
                    ok += sum(1 for r in rs if r.slo <= 0 or r.throughput >= r.slo)
                    n += len(rs)
                    if outcomes is not None:
                        outcomes.extend((r.workload, r.iters, r.slo, r.throughput) for r in rs)
        while pend:
            rs = pend.popleft()
            ex.wait_epoch(rs)
            if phase:
                ok += sum(1 for r in rs if r.slo <= 0 or r.throughput >= r.slo)
                n += len(rs)
                if outcomes is not None:
                    outcomes.extend((r.workload, r.iters, r.slo, r.throughput) for r in rs)
        if phase:
            t1 = ex.elapsed_ms
    return ok, n, t1 - t0


def fixed_places(places: List[List[Place]]) -> List[List[Place]]:
    """Each GPU's pods of an epoch onto its slots in arrival order."""
    out = []
    for pl in places:
        slots: Dict[int, List[int]] = collections.defaultdict(list)
        for g, u in pl:
            slots[g].append(u)
        for g in slots:
            slots[g].sort()
        nxt = collections.defaultdict(int)
        row = []
        for g, _ in pl:
            row.append((g, slots[g][nxt[g]]))
            nxt[g] += 1
        out.append(row)
    return out


def lpt_places(pods: List[List[Pod]], places: List[List[Place]], model: Any) -> List[List[Place]]:
    """Per GPU: longest predicted pod first onto the slot with the least cumulative work."""
    work: Dict[Place, float] = collections.defaultdict(float)
    out = []
    for ep, pl in zip(pods, places):
        row = list(pl)
        by: Dict[int, List[int]] = collections.defaultdict(list)
        for i, (g, _) in enumerate(pl):
            by[g].append(i)
        for g, idx in by.items():
            free = sorted(pl[i][1] for i in idx)
            for i in sorted(idx, key=lambda i: -model.alone_ms[ep[i][0]] * ep[i][1]):
                u = min(free, key=lambda s: (work[(g, s)], s))
                free.remove(u)
                row[i] = (g, u)
                work[(g, u)] += model.alone_ms[ep[i][0]] * ep[i][1]
        out.append(row)
    return out


def myopic_places(pods, places, timed, model: Any) -> List[List[Place]]:
    """Online: epoch by epoch, the permutation of its pods over its (gpu, slot) positions that
    is best for the pods known so far (N=1: all 24; N>1: the planner's and pairwise swaps)."""
    cur: List[List[Place]] = []
    multi = any(g != 0 for pl in places for g, _ in pl)
    for e in range(len(pods)):
        if multi:
            cands = [list(places[e])]
            for i, j in itertools.combinations(range(len(places[e])), 2):
                c = list(places[e])
                c[i], c[j] = c[j], c[i]
                cands.append(c)
        else:
            cands = [list(p) for p in itertools.permutations(places[e])]
        known = [True] * (e + 1)
        best, best_c = None, None
        for c in cands:
            # every pod placed so far counts (score the prefix as if it were all timed)
            r = simulate(pods[:e + 1], cur + [c], known, model=model)
            if best is None or _key(r) > _key(best):
                best, best_c = r, c
        cur.append(best_c)
    return cur


def _key(res: Tuple[int, int, float]) -> Tuple[int, float]:
    return res[0], -res[2]


def oracle(pods, places, timed, starts: Dict[str, List[List[Place]]], model: Any, budget_s: float,
           seed: int = 0) -> Tuple[List[List[Place]], Tuple[int, int, float], Dict[str, Any]]:
    """Coordinate descent from each start; N=1: all slot permutations of one epoch at a time,
    N>1: pairwise swaps of two pods' (gpu, slot) inside an epoch, in random order."""
    rng = random.Random(seed)
    best_pl, best = None, None
    log = {}
    t_end = time.time() + budget_s
    multi = any(g != 0 for pl in places for g, _ in pl)
    for name, st in starts.items():
        cur = [list(r) for r in st]
        res = simulate(pods, cur, timed, model=model)
        sims = 1
        improved = True
        while improved and time.time() < t_end:
            improved = False
            order = [e for e in range(len(pods)) if timed[e] or e >= sum(1 for t in timed if not t) - 2]
            rng.shuffle(order)
            for e in order:
                if time.time() > t_end:
                    break
                if not multi:
                    cands = [list(p) for p in itertools.permutations(cur[e])]
                else:
                    cands = []
                    ij = list(itertools.combinations(range(len(cur[e])), 2))
                    rng.shuffle(ij)
                    for i, j in ij[:48]:
                        if cur[e][i] == cur[e][j]:
                            continue
                        c = list(cur[e])
                        c[i], c[j] = c[j], c[i]
                        cands.append(c)
                for c in cands:
                    if c == cur[e]:
                        continue
                    trial = cur[:e] + [c] + cur[e + 1:]
                    r = simulate(pods, trial, timed, model=model)
                    sims += 1
                    if _key(r) > _key(res):
                        cur, res, improved = trial, r, True
        log[name] = {"slo_ok": res[0], "ms": round(res[2], 3), "sims": sims}
        if best is None or _key(res) > _key(best):
            best_pl, best = cur, res
    return best_pl, best, log


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--greedy", default="", help="a second dump of the same arrivals (e.g. --plan-bursts 0)")
    ap.add_argument("--budget-s", type=float, default=300.0)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from k8s_gpu_scheduler_amd.models.corun import CorunModel
    model = CorunModel.load()
    pods, places, timed, d = load(a.dump)
    lookahead = int(d.get("lookahead", 2))
    pol: Dict[str, List[List[Place]]] = {"planner": places, "fixed": fixed_places(places),
                                         "lpt": lpt_places(pods, places, model)}
    if a.greedy:
        gp, gpl, gt, _ = load(a.greedy)
        # the same arrivals, possibly listed in another order (the queue sorts each burst):
        # match each of this dump's pods to an identical pod of the greedy dump's epoch
        mapped = []
        for ep, gep, gpe in zip(pods, gp, gpl):
            if sorted(ep) != sorted(gep):
                raise SystemExit("--greedy dump has different arrivals")
            pool = collections.defaultdict(list)
            for x, pl in zip(gep, gpe):
                pool[x].append(pl)
            mapped.append([pool[x].pop(0) for x in ep])
        pol["greedy"] = mapped
    out: Dict[str, Any] = {"dump": a.dump, "n_gpus": d.get("n_gpus"), "seed": d.get("seed"), "lookahead": lookahead,
                           "bench_reported": d.get("sim"), "policies": {}}
    t = time.time()
    pol["myopic"] = myopic_places(pods, places, timed, model)
    myopic_s = time.time() - t
    for k, pl in pol.items():
        ok, n, ms = simulate(pods, pl, timed, lookahead, model)
        out["policies"][k] = {"slo_ok": ok, "pods": n, "slo_pct": round(100.0 * ok / n, 2), "ms": round(ms, 3),
                              "pods_per_s": round(n / ms * 1e3, 1)}
        print(k, out["policies"][k], flush=True)
    out["policies"]["myopic"]["search_s"] = round(myopic_s, 1)
    t = time.time()
    best_pl, best, log = oracle(pods, places, timed, pol, model, a.budget_s)
    ok, n, ms = best
    out["policies"]["oracle"] = {"slo_ok": ok, "pods": n, "slo_pct": round(100.0 * ok / n, 2), "ms": round(ms, 3),
                                 "pods_per_s": round(n / ms * 1e3, 1), "search_s": round(time.time() - t, 1),
                                 "from_start": log}
    print("oracle", out["policies"]["oracle"], flush=True)
    # which pods the oracle saves: per timed pod (workload, SLO / its alone rate) met by the
    # planner / by the oracle -- the pods it rescues and the ones it gives up
    o_pl, o_or = [], []
    simulate(pods, places, timed, lookahead, model, o_pl)
    simulate(pods, best_pl, timed, lookahead, model, o_or)
    saved, lost = collections.Counter(), collections.Counter()
    tight = {"saved": [], "lost": [], "both": [], "neither": []}
    for (wl, it, slo, thr_p), (_, _, _, thr_o) in zip(o_pl, o_or):
        alone = it / (model.alone_ms[model.wid(wl)] * it / 1e3)      # alone iterations / s
        k = ("both" if thr_p >= slo and thr_o >= slo else "saved" if thr_o >= slo else
             "lost" if thr_p >= slo else "neither")
        tight[k].append(round(slo / alone, 3))
        fam = wl.split("_", 1)[1].rsplit("_", 1)[0]
        if k == "saved":
            saved[fam] += 1
        elif k == "lost":
            lost[fam] += 1
    out["oracle_pods"] = {k: {"n": len(v), "slo_over_alone_rate_mean": round(sum(v) / len(v), 3) if v else None}
                          for k, v in tight.items()}
    out["oracle_pods"]["saved_by_family"] = dict(saved)
    out["oracle_pods"]["lost_by_family"] = dict(lost)
    out["oracle_places"] = best_pl
    print("oracle pods", out["oracle_pods"], flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
