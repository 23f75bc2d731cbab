"""Summarise tools/fetch_cal.py's counter runs: per group, counted bytes per launch against the
group's compulsory bytes.  Every `p*/**/*counter_collection.csv` under <dir> is one rocprofv3
--pmc pass; each group starts after a marker dispatch (xcd_probe_kernel).  Counters reported in
KiB by rocprofv3 (FETCH_SIZE, WRITE_SIZE) are turned into bytes; others stay raw."""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

MARKER = "xcd_probe_kernel"
KIB = {"FETCH_SIZE", "WRITE_SIZE"}


def summarise(root: str) -> dict:
    groups = json.load(open(os.path.join(root, "groups.json")))["groups"]
    per = [defaultdict(float) for _ in groups]
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
        g = -1
        last = None
        for r in rows:
            did = int(r["Dispatch_Id"])
            if MARKER in r.get("Kernel_Name", ""):
                if did != last:
                    g += 1
                last = did
                continue
            if 0 <= g < len(groups):
                per[g][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for grp, c in zip(groups, per):
        d = dict(grp)
        for k, v in c.items():
            d[k] = v * 1024 if k in KIB else v
        if "FETCH_SIZE" in c:
            d["fetch_over_compulsory_read"] = round(d["FETCH_SIZE"] / grp["compulsory_read"], 4)
        if "WRITE_SIZE" in c:
            d["write_over_compulsory"] = round(d["WRITE_SIZE"] / grp["compulsory_write"], 4)
        out[grp["name"]] = d
    return out


if __name__ == "__main__":
    root = sys.argv[1]
    res = summarise(root)
    json.dump(res, open(os.path.join(root, "summary.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))
