"""JSON-Patch (RFC 6902), JSON Merge-Patch (RFC 7386) and selector matching.

The reference patches pods and nodes with JSON-Patch payloads built by hand
(reference pkg/resources/pods.go:63-85, pkg/resources/nodes.go:39-68); the FakeCluster
and the REST client both need a faithful implementation of the same wire semantics.
"""
from __future__ import annotations

from ..api.objects import deepcopy as _dc
import re
from typing import Any, Dict, List, Optional, Tuple


class PatchError(ValueError):
    pass


def _unescape(tok: str) -> str:
    return tok.replace("~1", "/").replace("~0", "~")


def _split_pointer(ptr: str) -> List[str]:
    if ptr == "":
        return []
    if not ptr.startswith("/"):
        raise PatchError(f"invalid JSON pointer {ptr!r}")
    return [_unescape(t) for t in ptr[1:].split("/")]


def _walk(doc: Any, toks: List[str]) -> Any:
    cur = doc
    for t in toks:
        if isinstance(cur, list):
            cur = cur[int(t)]
        elif isinstance(cur, dict):
            if t not in cur:
                raise PatchError(f"path component {t!r} not found")
            cur = cur[t]
        else:
            raise PatchError(f"cannot traverse into {type(cur).__name__}")
    return cur


def _add(doc: Any, toks: List[str], value: Any, replace: bool = False) -> Any:
    if not toks:
        return _dc(value)
    parent = _walk(doc, toks[:-1])
    last = toks[-1]
    if isinstance(parent, list):
        if last == "-":
            if replace:
                raise PatchError("replace with '-' index")
            parent.append(_dc(value))
        else:
            i = int(last)
            if replace:
                if i >= len(parent):
                    raise PatchError("replace index out of range")
                parent[i] = _dc(value)
            else:
                if i > len(parent):
                    raise PatchError("add index out of range")
                parent.insert(i, _dc(value))
    elif isinstance(parent, dict):
        if replace and last not in parent:
            raise PatchError(f"replace: key {last!r} missing")
        parent[last] = _dc(value)
    else:
        raise PatchError("parent is not a container")
    return doc


def _remove(doc: Any, toks: List[str]) -> Tuple[Any, Any]:
    if not toks:
        raise PatchError("cannot remove the root")
    parent = _walk(doc, toks[:-1])
    last = toks[-1]
    if isinstance(parent, list):
        return doc, parent.pop(int(last))
    if isinstance(parent, dict):
        if last not in parent:
            raise PatchError(f"remove: key {last!r} missing")
        return doc, parent.pop(last)
    raise PatchError("parent is not a container")


def apply_json_patch(doc: Any, ops: List[Dict[str, Any]]) -> Any:
    """Apply an RFC 6902 patch; returns a new document (input untouched)."""
    out = _dc(doc)
    for op in ops:
        kind = op.get("op")
        toks = _split_pointer(op.get("path", ""))
        if kind == "add":
            out = _add(out, toks, op.get("value"))
        elif kind == "replace":
            # The apiserver (and therefore the reference's node-label replace,
            # reference nodes.go:52-57) accepts replace on a missing map key as add.
            try:
                out = _add(out, toks, op.get("value"), replace=True)
            except PatchError:
                parent = _walk(out, toks[:-1]) if toks else None
                if isinstance(parent, dict):
                    parent[toks[-1]] = _dc(op.get("value"))
                else:
                    raise
        elif kind == "remove":
            out, _ = _remove(out, toks)
        elif kind == "test":
            if _walk(out, toks) != op.get("value"):
                raise PatchError(f"test failed at {op.get('path')}")
        elif kind == "move":
            out, v = _remove(out, _split_pointer(op["from"]))
            out = _add(out, toks, v)
        elif kind == "copy":
            v = _walk(out, _split_pointer(op["from"]))
            out = _add(out, toks, v)
        else:
            raise PatchError(f"unknown op {kind!r}")
    return out


def apply_merge_patch(doc: Any, patch: Any) -> Any:
    """RFC 7386: null deletes, dicts merge recursively, everything else replaces.
    Returns a new document (the input is copied once, then merged in place)."""
    if not isinstance(patch, dict):
        return _dc(patch)
    out = _dc(doc) if isinstance(doc, dict) else {}
    _merge_into(out, patch)
    return out


def _merge_into(out: Dict[str, Any], patch: Dict[str, Any]) -> None:
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        elif isinstance(v, dict):
            cur = out.get(k)
            if not isinstance(cur, dict):
                cur = {}
                out[k] = cur
            _merge_into(cur, v)
        else:
            out[k] = _dc(v)


# --------------------------------------------------------------------------- selectors
def _field_value(obj: Dict[str, Any], path: str) -> str:
    cur: Any = obj
    for p in path.split("."):
        if not isinstance(cur, dict):
            return ""
        cur = cur.get(p)
        if cur is None:
            return ""
    return str(cur)


def match_field_selector(obj: Dict[str, Any], selector: Optional[str]) -> bool:
    """Field selectors as the apiserver supports them: `a.b=c`, `a.b==c`, `a.b!=c`, comma-AND."""
    if not selector:
        return True
    for term in selector.split(","):
        term = term.strip()
        if not term:
            continue
        if "!=" in term:
            f, v = term.split("!=", 1)
            if _field_value(obj, f.strip()) == v.strip():
                return False
        else:
            f, v = term.split("==", 1) if "==" in term else term.split("=", 1)
            if _field_value(obj, f.strip()) != v.strip():
                return False
    return True


_SET_RE = re.compile(r"^\s*([^\s!=]+)\s+(in|notin)\s+\(([^)]*)\)\s*$")


def _split_selector_terms(sel: str) -> List[str]:
    terms, depth, cur = [], 0, []
    for ch in sel:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            terms.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    if cur:
        terms.append("".join(cur))
    return [t.strip() for t in terms if t.strip()]


def match_label_selector(lbls: Dict[str, str], selector: Any) -> bool:
    """String label selectors (`a=b,c!=d,e in (x,y),f notin (z),g,!h`) or the structured
    LabelSelector form ({matchLabels, matchExpressions})."""
    if not selector:
        return True
    lbls = lbls or {}
    if isinstance(selector, dict):
        for k, v in (selector.get("matchLabels") or {}).items():
            if lbls.get(k) != v:
                return False
        for e in selector.get("matchExpressions") or []:
            k, op, vals = e.get("key"), e.get("operator"), e.get("values") or []
            if op == "In" and lbls.get(k) not in vals:
                return False
            if op == "NotIn" and lbls.get(k) in vals:
                return False
            if op == "Exists" and k not in lbls:
                return False
            if op == "DoesNotExist" and k in lbls:
                return False
        return True
    for term in _split_selector_terms(str(selector)):
        m = _SET_RE.match(term)
        if m:
            k, op, vals = m.group(1), m.group(2), [v.strip() for v in m.group(3).split(",") if v.strip()]
            if op == "in" and lbls.get(k) not in vals:
                return False
            if op == "notin" and lbls.get(k) in vals:
                return False
        elif term.startswith("!"):
            if term[1:] in lbls:
                return False
        elif "!=" in term:
            k, v = term.split("!=", 1)
            if lbls.get(k.strip()) == v.strip():
                return False
        elif "=" in term:
            k, v = term.split("==", 1) if "==" in term else term.split("=", 1)
            if lbls.get(k.strip()) != v.strip():
                return False
        else:
            if term not in lbls:
                return False
    return True
