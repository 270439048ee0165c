# Round 4, step 10: the GPU suite at one seg wave per workgroup; the LPT tail
# length (HC_PHMM_TAIL_ROUNDS) at the shard sizes; the region call with every
# rescue in-wave (HC_PHMM_SOLO_MAX_PAIRS) and other in-wave caps.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/s10
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s10/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/s10/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
NO_R3=1 VARIANTS="t2:HC_PHMM_TAIL_ROUNDS=2 t0:HC_PHMM_TAIL_ROUNDS=0 t1:HC_PHMM_TAIL_ROUNDS=1 t3:HC_PHMM_TAIL_ROUNDS=3" PAIRS="125000 250000 1000000" bash tools/persist_ab.sh || exit 1
timeout -k 10 200 python3 tools/region_ab.py 128 HC_PHMM_SOLO_MAX_PAIRS=0,100000 || exit 1
timeout -k 10 200 python3 tools/region_ab.py 128 HC_PHMM_RESCUE_IN_WAVE_MAX=32,0,128,1000 || exit 1
