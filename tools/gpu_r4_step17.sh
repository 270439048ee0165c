# Round 4, step 17: the fp64 planner's batched list walks. Rescue tests, then
# the tree against the library of 0feacb9 (ab_libs/libhcpairhmm_r4b.so) at S4,
# S4-20k (warm clocks) and the 415 x 128 region call.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/s17
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "rescue or golden or use_double or stolen or small_part or s4" --timeout 300 --timeout-method thread > gpurun_out/s17/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/s17/tests.log
[ $rc -eq 0 ] || exit $rc
WL=S4 BASE=r4b WARM=300 STEPS=50 VARIANTS="new:HC_PHMM_PRIO=0" PAIRS="2000" bash tools/persist_ab.sh || exit 1
WL=S4 BASE=r4b WARM=40 STEPS=20 VARIANTS="new:HC_PHMM_PRIO=0" PAIRS="20000" bash tools/persist_ab.sh || exit 1
for rep in 1 2; do
  for b in r4b tree; do
    lib=""; [ $b = tree ] || lib=$PWD/ab_libs/libhcpairhmm_$b.so
    echo -n "region $b: "
    HC_PHMM_LIB=$lib timeout -k 10 120 python3 tools/region_ab.py 128 HC_PHMM_X=0 2>/dev/null || exit 1
  done
done
