# Stall breakdown of the wide-channel Gram launch (runtime channel loop, wide.h): parked (s_waitcnt /
# barrier), issue-stalled and issuing wave-cycles, VALU activity.  One --pmc pass per channel count.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_wide
mkdir -p $O
for d in 46 126; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/d$d -o run --output-format csv -- python3 tools/bench_wide.py --d $d > $O/d$d.log 2>&1 || exit 1
  python3 tools/sq_busy.py $O/d$d "sig_fo_kernel<0" > $O/d$d.json || exit 2
done
python3 -c "
import json
for d in (46, 126):
    for r in json.load(open(f'$O/d{d}.json')):
        c = r['counters']; w = c['SQ_WAVE_CYCLES']
        print(d, r['kernel'][:48], r['dispatches'], 'valu_busy', round(r['valu_busy'], 3), 'parked', round(c['SQ_WAIT_ANY'] / w, 3), 'issue_stall', round(c['SQ_WAIT_INST_ANY'] / w, 3), 'issuing', round(c['SQ_ACTIVE_INST_ANY'] / w, 3), 'smem/valu', round(c['SQ_INSTS_SMEM'] / c['SQ_INSTS_VALU'], 4))
"
