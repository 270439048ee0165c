# Round-4 closing measurements: GPU tests, the records-threshold and SW
# stripe-pipeline A/Bs, then every config's committed profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t6.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/t6.log
[ $rc -eq 0 ] || exit $rc
NO_R3=1 VARIANTS="rec_off:HC_PHMM_REC_MIN_PAIRS=100000000 rec_on:HC_PHMM_REC_MIN_PAIRS=0" PAIRS="125000 1000000" bash tools/persist_ab.sh || exit 1
NO_R3=1 WL=S1 VARIANTS="rec_off:HC_PHMM_REC_MIN_PAIRS=100000000 rec_on:HC_PHMM_REC_MIN_PAIRS=0" PAIRS="10000" bash tools/persist_ab.sh || exit 1
for v in 0 1; do
  HC_SW_SPIRAL=$v timeout -k 10 180 python3 tools/sw_timing.py W2 W3 > gpurun_out/sw_spiral_$v.json 2>&1 || exit 1
  echo "SW spiral=$v: $(grep dp_ms gpurun_out/sw_spiral_$v.json | python3 -c "import sys,json; print([(d['name'], round(d['dp_ms'],3)) for d in map(json.loads, sys.stdin)])")"
done

