# Round 4, step 12: stealable rescues (seg waves take deferred rescues while
# the pass drains). The new tests first, then the whole suite, then the region
# call and S2 / S4 / a 125k shard with stealing on and off.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/s12
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "stolen or small_part or golden_bit_exact" --timeout 200 --timeout-method thread > gpurun_out/s12/new_tests.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -5 gpurun_out/s12/new_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s12/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/s12/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/region_ab.py 128 HC_PHMM_STEAL=0,1 || exit 1
NO_R3=1 VARIANTS="st1:HC_PHMM_STEAL=1 st0:HC_PHMM_STEAL=0" PAIRS="125000 1000000" bash tools/persist_ab.sh || exit 1
WL=S4 NO_R3=1 VARIANTS="st1:HC_PHMM_STEAL=1 st0:HC_PHMM_STEAL=0" PAIRS="2000 20000" bash tools/persist_ab.sh || exit 1
