# A/B of the wide-channel forward's rows per channel-loop chunk (GPSIG_WIDE_R = 4 in libgpsig_amd.so vs 8 in
# a variant library): parity of the wide tests under the variant, then K(X) times at wide channel counts.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_wide_r
mkdir -p $O
V=$PWD/gpsig_amd/libgpsig_amd_r8.so
GPSIG_AMD_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_wide_gpu.py -q -k "not vjp and not tvs and not kuf and not tens and not rescaled" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_r8.log 2>&1
r=$?; tail -3 $O/tests_r8.log; [ $r -ne 0 ] && [ $r -ne 1 ] && exit $r
timeout -k 10 300 python3 -u tools/bench_wide.py --d 46 126 > $O/r4.jsonl 2>&1 || exit 2
GPSIG_AMD_LIB=$V timeout -k 10 300 python3 -u tools/bench_wide.py --d 46 126 > $O/r8.jsonl 2>&1 || exit 3
GPSIG_FO_FIXED_MAX=0 timeout -k 10 300 python3 -u tools/bench_wide.py --d 8 16 32 > $O/r4_forced.jsonl 2>&1 || exit 4
GPSIG_FO_FIXED_MAX=0 GPSIG_AMD_LIB=$V timeout -k 10 300 python3 -u tools/bench_wide.py --d 8 16 32 > $O/r8_forced.jsonl 2>&1 || exit 5
cat $O/*.jsonl
