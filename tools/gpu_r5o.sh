#!/bin/bash
# round 5: the whole GPU suite and smoke() on the current tree
mkdir -p gpurun_out/r5o
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5o/gpu_suite.log 2>&1
echo "suite rc=$?" >> gpurun_out/r5o/gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5o/smoke.log 2>&1
echo "smoke rc=$?" >> gpurun_out/r5o/smoke.log
