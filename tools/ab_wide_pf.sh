# A/B of the wide-channel forward's channel-loop prefetch ring (GPSIG_WIDE_PF=U in variant libraries
# libgpsig_amd_pfU.so) against the default build: parity of the wide Gram tests under each variant,
# then K(X) times.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_wide_pf
mkdir -p $O
timeout -k 10 300 python3 -u tools/bench_wide.py --d 12 26 46 126 > $O/base.jsonl 2>&1 || exit 2
for U in 2 4; do
  V=$PWD/gpsig_amd/libgpsig_amd_pf$U.so
  GPSIG_AMD_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_wide_gpu.py -q -k "not vjp and not tvs and not kuf and not tens and not rescaled" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_pf$U.log 2>&1
  r=$?; tail -3 $O/tests_pf$U.log; [ $r -ne 0 ] && [ $r -ne 1 ] && exit $r
  GPSIG_AMD_LIB=$V timeout -k 10 300 python3 -u tools/bench_wide.py --d 12 26 46 126 > $O/pf$U.jsonl 2>&1 || exit 3
done
grep -h '^{' $O/base.jsonl $O/pf2.jsonl $O/pf4.jsonl
