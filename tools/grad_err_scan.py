#!/usr/bin/env python3
"""Observed gradient errors of the wide-channel GPU tests: runs tests/test_wide_gpu.py (gradient tests only)
with norm_rel_err wrapped to record every value it returns, and prints the largest per test -- the evidence
for each test's GTOL.

    python tools/grad_err_scan.py [-k expr]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import pytest  # noqa: E402

import conftest  # noqa: E402

seen = {}
_orig = conftest.norm_rel_err


def _rec(*a, **k):
    v = _orig(*a, **k)
    cur = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    seen[cur] = max(seen.get(cur, 0.0), float(np.max(v)))
    return v


class Patch:
    def pytest_collection_modifyitems(self, items):
        for it in items:
            if hasattr(it.module, "norm_rel_err"):
                it.module.norm_rel_err = _rec


if __name__ == "__main__":
    args = ["-q", "-m", "gpu", "-p", "no:cacheprovider", os.path.join(ROOT, "tests", "test_wide_gpu.py"),
            "-k", "vjp or gradient"] + sys.argv[1:]
    rc = pytest.main(args, plugins=[Patch()])
    for k, v in sorted(seen.items()):
        print(json.dumps({"test": k, "max_norm_rel_err": v}))
    sys.exit(rc)
