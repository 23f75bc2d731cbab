"""Training tables: TSV load, md5 versioning, request-index matching, model fit.

Reference: matrices are tab-separated files (named `.ods`), first column `index`
(reference pkg/recommender/recom_server.py:97-101,215-235); the version is
the file's md5 (recom_server.py:62-64); a request matches the FIRST row label that is a
substring of `request.index.replace("-", "_")` (recom_server.py:67-71,155-156).
"""
from __future__ import annotations

import hashlib
import os
import threading
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from ..models.imputers import ImputerBase, make_imputer


def file_version(path: str) -> Optional[str]:
    """md5 of the file, None if missing (the reference hashes before checking existence
    and crashes its retrain thread -- SURVEY §2.9 #12)."""
    if not path or not os.path.isfile(path):
        return None
    h = hashlib.md5()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def find_index_for_request(request: str, index: Sequence[str]) -> str:
    for ind in index:
        if ind in request:
            return ind
    return ""


@dataclass
class Table:
    index: List[str]
    columns: List[str]
    values: np.ndarray            # float64, NaN = missing

    @classmethod
    def read_tsv(cls, path: str) -> "Table":
        with open(path) as f:
            lines = [ln.rstrip("\n").rstrip("\r") for ln in f if ln.strip()]
        header = lines[0].split("\t")
        if header[0] != "index":
            raise ValueError(f"{path}: first column must be 'index' (got {header[0]!r})")
        cols = header[1:]
        idx, vals = [], []
        for ln in lines[1:]:
            parts = ln.split("\t")
            idx.append(parts[0])
            row = []
            for j in range(len(cols)):
                s = parts[j + 1].strip() if j + 1 < len(parts) else ""
                row.append(float(s) if s not in ("", "nan", "NaN", "NA") else np.nan)
            vals.append(row)
        return cls(idx, cols, np.asarray(vals, dtype=float))

    def write_tsv(self, path: str) -> None:
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write("\t".join(["index"] + list(self.columns)) + "\n")
            for i, r in zip(self.index, self.values):
                f.write("\t".join([i] + ["" if np.isnan(v) else repr(float(v)) for v in r]) + "\n")
        os.replace(tmp, path)

    def to_json(self) -> Dict[str, Any]:
        return {"index": list(self.index), "columns": list(self.columns),
                "values": [[None if np.isnan(v) else float(v) for v in r] for r in self.values]}

    @classmethod
    def from_json(cls, d: Dict[str, Any]) -> "Table":
        vals = np.asarray([[np.nan if v is None else float(v) for v in r] for r in d["values"]], dtype=float)
        return cls(list(d["index"]), list(d["columns"]), vals)

    def row(self, label: str) -> np.ndarray:
        return self.values[self.index.index(label)]

    def set(self, label: str, column: str, value: float) -> None:
        if column not in self.columns:
            self.columns.append(column)
            self.values = np.concatenate([self.values, np.full((len(self.index), 1), np.nan)], axis=1)
        if label not in self.index:
            self.index.append(label)
            self.values = np.concatenate([self.values, np.full((1, len(self.columns)), np.nan)], axis=0)
        self.values[self.index.index(label), self.columns.index(column)] = value


class TrainedTable:
    """A table + its fitted model + cached completed matrix."""

    def __init__(self, table: Table, model: ImputerBase, version: str):
        self.table, self.model, self.version = table, model, version
        self._full: Optional[np.ndarray] = None
        self._lock = threading.Lock()

    @classmethod
    def fit(cls, table: Table, kind: str = "iterative", version: str = "", **kw) -> "TrainedTable":
        return cls(table, make_imputer(kind, **kw).fit(table.values), version)

    def predict_label(self, label: str) -> np.ndarray:
        row = self.table.row(label).reshape(1, -1)
        return self.model.predict(row)[0]

    def completed(self) -> np.ndarray:
        with self._lock:
            if self._full is None:
                self._full = self.model.predict(self.table.values)
            return self._full

    def lookup(self, request_index: str) -> Dict[str, float]:
        lab = find_index_for_request(request_index.replace("-", "_"), self.table.index)
        if not lab:
            return {}
        return dict(zip(self.table.columns, (float(x) for x in self.predict_label(lab))))
