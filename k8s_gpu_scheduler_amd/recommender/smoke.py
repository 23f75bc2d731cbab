"""Recommender smoke client + helpers.

Reference: `recom_client.py` calls both RPCs on localhost:50051 (and reads a file that
does not exist, reference pkg/recommender/recom_client.py:10-40); the Go
`go_client/cmd/main.go` prints `FindMaxIndForNode("A30")` = the largest value among
columns containing the node model (reference go_client/utils/utils.go:9-17).  Both are
re-created here against a live server:

  python -m k8s_gpu_scheduler_amd.recommender.smoke --addr 127.0.0.1:50051 --pod mlperf-gpu-onnx-mobilenet-1024
"""
from __future__ import annotations

import argparse
import json
from typing import Dict, List, Optional, Tuple

from .client import RecommenderClient, reply_to_map


def find_max_ind_for_node(columns: List[str], values: List[float], model: str) -> Tuple[str, float]:
    """(column, value) of the largest prediction among columns containing `model`."""
    best = ("", float("-inf"))
    for c, v in zip(columns, values):
        if model in c and v > best[1]:
            best = (c, v)
    return best


def run(addr: str, pod: str, model: str = "MI355X") -> Dict[str, object]:
    cl = RecommenderClient(addr, timeout_s=5.0)
    conf = cl.impute_configurations(pod)
    intf = cl.impute_interference(f"{pod}_{model}")
    col, val = find_max_ind_for_node(list(conf.columns), list(conf.result), model)
    cl.close()
    return {"configurations": reply_to_map(conf), "interference": reply_to_map(intf),
            "max_for_model": {"column": col, "value": val}}


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--addr", default="127.0.0.1:50051")
    ap.add_argument("--pod", default="onnx-resnet50-1024")
    ap.add_argument("--model", default="MI355X")
    a = ap.parse_args(argv)
    print(json.dumps(run(a.addr, a.pod, a.model), indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
