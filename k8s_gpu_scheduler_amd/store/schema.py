"""Redis key schema.

Reference schema: key `<nodeName>` -> JSON array of device UUIDs,
`GPU-…` or, when any MIG device exists, only the `MIG-…` ones
(reference pkg/profiler/cmd/client/client.go:37-46,70-76).  Kept verbatim; the MI355X
build adds richer side keys under a `gpusched:` prefix that the reference never reads:

  gpusched:devices:<node>      JSON list of device descriptors (index, uuid, partition, numa, cus, hbm)
  gpusched:topology:<node>     JSON link matrix (type/hops/weight) + NUMA
  gpusched:hist:<pod>          list of JSON usage samples (profiler history -> recommender resize)
  gpusched:model:<name>        versioned recommender model metadata
  gpusched:partition:<node>    requested/applied partition state
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional

from .resp import Redis, RedisNil

PREFIX = "gpusched:"


def devices_key(node: str) -> str:
    return f"{PREFIX}devices:{node}"


def topology_key(node: str) -> str:
    return f"{PREFIX}topology:{node}"


def history_key(pod: str) -> str:
    return f"{PREFIX}hist:{pod}"


def partition_key(node: str) -> str:
    return f"{PREFIX}partition:{node}"


def partition_caps_key(node: str) -> str:
    """JSON agent.devices.PartitionCaps: the modes the node's GPUs support (probed)."""
    return f"{PREFIX}partcaps:{node}"


def model_key(name: str) -> str:
    return f"{PREFIX}model:{name}"


def filter_partition_uuids(uuids: List[str]) -> List[str]:
    """If any partition ('MIG-' / AMD partition) UUID is present keep only those, like
    reference client.go:37-46 (which uses a substring test, utils.Exists)."""
    uuids = [u.strip().strip("'\"") for u in uuids if u and u.strip().strip("'\"")]
    if any("MIG" in u for u in uuids):
        return [u for u in uuids if "MIG" in u]
    if any(u.startswith("PART-") for u in uuids):
        return [u for u in uuids if u.startswith("PART-")]
    return uuids


def publish_uuids(r: Redis, node: str, uuids: List[str]) -> str:
    val = json.dumps(filter_partition_uuids(uuids), separators=(",", ":"))
    r.set(node, val)
    return val


def read_uuids(r: Redis, node: str) -> Optional[List[str]]:
    try:
        v = r.get(node)
    except RedisNil:
        return None
    try:
        out = json.loads(v)
    except json.JSONDecodeError:
        return None
    return [str(x) for x in out] if isinstance(out, list) else None


def publish_devices(r: Redis, node: str, devices: List[Dict[str, Any]]) -> None:
    r.set(devices_key(node), json.dumps(devices, separators=(",", ":")))


def read_devices(r: Redis, node: str) -> Optional[List[Dict[str, Any]]]:
    v = r.get_or(devices_key(node))
    return json.loads(v) if v else None


def append_history(r: Redis, pod: str, sample: Dict[str, Any], keep: int = 512) -> None:
    k = history_key(pod)
    r.pipeline([["RPUSH", k, json.dumps(sample, separators=(",", ":"))], ["LTRIM", k, -keep, -1]])


def read_history(r: Redis, pod: str, last: int = 512) -> List[Dict[str, Any]]:
    return [json.loads(x) for x in r.lrange(history_key(pod), -last, -1)]
