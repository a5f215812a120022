"""Build the reference's own Cython PDE solver into oracle/_ref/ (checker only).

TEST INFRASTRUCTURE ONLY.  Compiles /root/reference/gpsig/sigKer_fast.pyx
exactly where it lies (no source is copied into the repo) with the directives
the reference's Cython-0.29 era defaults imply under Cython 3
(``language_level=2, cpow=True``; the reference setup.py at
gpsig/setup.py:1-13 fails under Cython 3 without cpow=True).
Outputs (generated C and the extension module) go only to oracle/_ref/, which
is git-ignored.  Used by tests/golden/make_golden.py to pin oracle/pde against
the reference's own solver.

Run:  python -m oracle.build_ref
"""
from __future__ import annotations

import os
import sys
import sysconfig
import subprocess

REF_PYX = "/root/reference/gpsig/sigKer_fast.pyx"
OUT_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ref")


def build() -> str | None:
    if not os.path.exists(REF_PYX):
        return None
    os.makedirs(OUT_DIR, exist_ok=True)
    c_file = os.path.join(OUT_DIR, "sigKer_fast.c")
    ext = sysconfig.get_config_var("EXT_SUFFIX")
    so = os.path.join(OUT_DIR, "sigKer_fast" + ext)
    if os.path.exists(so) and os.path.getmtime(so) > os.path.getmtime(REF_PYX):
        return so
    subprocess.check_call([sys.executable, "-m", "cython", "-2", "-X", "cpow=True", "-X", "boundscheck=False",
                           "-X", "wraparound=False", REF_PYX, "-o", c_file])
    import numpy as np
    inc = [sysconfig.get_paths()["include"], np.get_include()]
    subprocess.check_call(["gcc", "-O2", "-fopenmp", "-fPIC", "-shared", "-ffp-contract=off"]
                          + [f"-I{p}" for p in inc] + [c_file, "-o", so])
    return so


def load():
    so = build()
    if so is None:
        return None
    sys.path.insert(0, OUT_DIR)
    try:
        import sigKer_fast  # noqa: F401
        return sigKer_fast
    finally:
        sys.path.pop(0)


if __name__ == "__main__":
    print(build())
