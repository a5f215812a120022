#!/bin/bash
# One GPU session: the GPU test suite (every module, no -x, so one failure does not hide the rest),
# smoke(), and the headline bench line.  Each GPU step has its own time limit; the script stops at
# the first step that faults, aborts or times out.
#   tools/gpu_suite.sh <outdir> [pytest args...]
OUT=${1:-gpurun_out/suite}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
rc() { local r=$1; if [ "$r" -eq 124 ] || [ "$r" -eq 137 ] || [ "$r" -eq 134 ] || [ "$r" -eq 139 ]; then echo "fatal rc=$r" >&2; exit "$r"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider "$@" \
  > "$OUT/pytest.log" 2>&1
r=$?; tail -5 "$OUT/pytest.log"; rc $r
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
r=$?; tail -2 "$OUT/smoke.log"; rc $r
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err"
r=$?; cat "$OUT/bench.json"; rc $r
exit 0
