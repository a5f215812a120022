#!/usr/bin/env python3
"""Instruction histogram of one kernel in a hipcc --save-temps .s file (static counts; the largest
basic-block loop is reported separately).  usage: isa_stats.py file.s [symbol-substring]"""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read().split("\n")
sub = sys.argv[2] if len(sys.argv) > 2 else "sig_fo_kernel"
start = next(i for i, l in enumerate(src) if re.match(r"^_Z\S*%s\S*:" % sub, l))
end = next(i for i in range(start, len(src)) if "s_endpgm" in src[i])
body = src[start:end + 1]
# loops: a label L followed later by s_cbranch_* L
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\S+:", l)}
best = None
for i, l in enumerate(body):
    m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\S+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        span = (labels[m.group(1)], i)
        if best is None or span[1] - span[0] > best[1] - best[0]:
            best = span


def hist(lines):
    c = Counter()
    for l in lines:
        m = re.match(r"^\s+([sv]_[a-z0-9_]+)", l)
        if m:
            c[m.group(1)] += 1
    return c


for name, lines in (("kernel", body), ("loop", body[best[0]:best[1] + 1] if best else [])):
    c = hist(lines)
    v = sum(n for k, n in c.items() if k.startswith("v_"))
    s = sum(n for k, n in c.items() if k.startswith("s_"))
    print(f"== {name}: {len(lines)} lines, VALU {v}, SALU/SMEM/branch {s}, s_nop {c['s_nop']}")
    print("   " + ", ".join(f"{k} {n}" for k, n in c.most_common(40)))
