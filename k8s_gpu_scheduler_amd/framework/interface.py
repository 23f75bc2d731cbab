"""Scheduler-framework plugin API.

The reference plugs into upstream kube-scheduler v1.21's framework through Go
interfaces (`framework.ScorePlugin`, `framework.PostBindPlugin`; reference
pkg/plugins/gpu_plugin/gpu_plugins.go:43-44) -- which does not exist in this
environment (no Go), so the same extension points are re-created here with the same
semantics: codes, score range [0,100], ScoreExtensions.NormalizeScore, weights,
CycleState, Reserve/Unreserve, Permit, PreBind/Bind/PostBind.
"""
from __future__ import annotations

import enum
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

from ..api.constants import MAX_NODE_SCORE, MIN_NODE_SCORE

Obj = Dict[str, Any]


class Code(enum.IntEnum):
    SUCCESS = 0
    ERROR = 1
    UNSCHEDULABLE = 2
    UNSCHEDULABLE_AND_UNRESOLVABLE = 3
    WAIT = 4
    SKIP = 5


@dataclass
class Status:
    code: Code = Code.SUCCESS
    reasons: List[str] = field(default_factory=list)
    plugin: str = ""

    @classmethod
    def success(cls) -> "Status":
        return _SUCCESS

    @classmethod
    def error(cls, msg: str, plugin: str = "") -> "Status":
        return cls(Code.ERROR, [msg], plugin)

    @classmethod
    def unschedulable(cls, msg: str, plugin: str = "", unresolvable: bool = False) -> "Status":
        return cls(Code.UNSCHEDULABLE_AND_UNRESOLVABLE if unresolvable else Code.UNSCHEDULABLE, [msg], plugin)

    @classmethod
    def skip(cls) -> "Status":
        return cls(Code.SKIP)

    @classmethod
    def wait(cls, msg: str = "") -> "Status":
        return cls(Code.WAIT, [msg] if msg else [])

    @property
    def ok(self) -> bool:
        return self.code == Code.SUCCESS

    def is_unschedulable(self) -> bool:
        return self.code in (Code.UNSCHEDULABLE, Code.UNSCHEDULABLE_AND_UNRESOLVABLE)

    def message(self) -> str:
        return "; ".join(self.reasons)

    def __bool__(self) -> bool:  # truthy == success
        return self.ok


_SUCCESS = Status(Code.SUCCESS)


def as_status(s: Optional[Status]) -> Status:
    return _SUCCESS if s is None else s


class CycleState:
    """Per-scheduling-cycle key/value store shared by plugins.  Thread-safe without a
    lock: every operation is ONE dict operation (get/set/pop/copy), atomic under the GIL
    -- parallel Score workers (parity mode) read and write it concurrently."""

    __slots__ = ("_d", "skip_filter_plugins", "skip_score_plugins", "read", "write")

    def __init__(self) -> None:
        self._d: Dict[str, Any] = {}
        self.skip_filter_plugins: set = set()
        self.skip_score_plugins: set = set()
        # bound dict methods: read(k[, default]) / write(k, v) are the hot accessors
        self.read = self._d.get
        self.write = self._d.__setitem__

    def delete(self, k: str) -> None:
        self._d.pop(k, None)

    def clone(self) -> "CycleState":
        c = CycleState()
        c._d.update(self._d)
        return c


@dataclass
class NodeScore:
    name: str
    score: int


class Plugin:
    """Base of every plugin.  `NAME` is the registry/profile name."""
    NAME = ""

    def name(self) -> str:
        return self.NAME or type(self).__name__


class QueueSortPlugin(Plugin):
    def less(self, a: Any, b: Any) -> bool:  # a, b: QueuedPodInfo
        raise NotImplementedError


class PreFilterPlugin(Plugin):
    def pre_filter(self, state: CycleState, pod: Obj) -> Optional[Status]:
        raise NotImplementedError


class FilterPlugin(Plugin):
    def filter(self, state: CycleState, pod: Obj, node_info: Any) -> Optional[Status]:
        raise NotImplementedError


class PostFilterPlugin(Plugin):
    def post_filter(self, state: CycleState, pod: Obj, filtered: Dict[str, Status]) -> Tuple[Optional[str], Status]:
        raise NotImplementedError


class PreScorePlugin(Plugin):
    def pre_score(self, state: CycleState, pod: Obj, nodes: List[Any]) -> Optional[Status]:
        raise NotImplementedError


class ScoreExtensions:
    def normalize_score(self, state: CycleState, pod: Obj, scores: List[NodeScore]) -> Optional[Status]:
        raise NotImplementedError


class ScorePlugin(Plugin):
    def score(self, state: CycleState, pod: Obj, node_name: str) -> Tuple[int, Optional[Status]]:
        raise NotImplementedError

    def score_extensions(self) -> Optional[ScoreExtensions]:
        return None


class ReservePlugin(Plugin):
    def reserve(self, state: CycleState, pod: Obj, node_name: str) -> Optional[Status]:
        raise NotImplementedError

    def unreserve(self, state: CycleState, pod: Obj, node_name: str) -> None:
        raise NotImplementedError


class PermitPlugin(Plugin):
    def permit(self, state: CycleState, pod: Obj, node_name: str) -> Tuple[Optional[Status], float]:
        raise NotImplementedError


class PreBindPlugin(Plugin):
    def pre_bind(self, state: CycleState, pod: Obj, node_name: str) -> Optional[Status]:
        raise NotImplementedError


class BindPlugin(Plugin):
    def bind(self, state: CycleState, pod: Obj, node_name: str) -> Optional[Status]:
        raise NotImplementedError


class PostBindPlugin(Plugin):
    def post_bind(self, state: CycleState, pod: Obj, node_name: str) -> None:
        raise NotImplementedError


EXTENSION_POINTS = {
    "queueSort": QueueSortPlugin, "preFilter": PreFilterPlugin, "filter": FilterPlugin,
    "postFilter": PostFilterPlugin, "preScore": PreScorePlugin, "score": ScorePlugin,
    "reserve": ReservePlugin, "permit": PermitPlugin, "preBind": PreBindPlugin,
    "bind": BindPlugin, "postBind": PostBindPlugin,
}


def min_max_normalize(scores: List[NodeScore]) -> None:
    """Min-max rescale to [MIN_NODE_SCORE, MAX_NODE_SCORE]; all-equal -> all MIN.
    Integer arithmetic identical to reference gpu_plugins.go:816-841."""
    if not scores:
        return
    hi = max(s.score for s in scores)
    lo = min(s.score for s in scores)
    old = hi - lo
    new = MAX_NODE_SCORE - MIN_NODE_SCORE
    for s in scores:
        if old == 0:
            s.score = MIN_NODE_SCORE
        else:
            # Go int64 division truncates toward zero; operands here are >= 0.
            s.score = ((s.score - lo) * new) // old + MIN_NODE_SCORE
