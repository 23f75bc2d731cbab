"""Test-retest stability of the measured MI355X tables: run models.profile twice with the
same settings and report the correlation / relative spread of the two interference and
configuration matrices.  python tools/table_retest.py <iters> <repeats> <out.json>"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from k8s_gpu_scheduler_amd.models.profile import profile  # noqa: E402


def main():
    iters, repeats, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    runs = [profile(iters, repeats=repeats) for _ in range(2)]
    (n, c1, i1), (_, c2, i2) = runs
    res = {"iters": iters, "repeats": repeats}
    for name, a, b in (("configurations", c1, c2), ("interference", i1, i2)):
        a, b = a.ravel(), b.ravel()
        res[name] = {"pearson": float(np.corrcoef(a, b)[0, 1]),
                     "median_abs_rel_diff": float(np.median(np.abs(a - b) / np.maximum((a + b) / 2, 1e-9))),
                     "mean_abs_diff": float(np.mean(np.abs(a - b)))}
    print(json.dumps(res))
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
