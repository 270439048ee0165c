# Chained fp64 rescue: S4 at 20 000 pairs, chain tail sweep and unchained.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "rescue or golden or s4 or repeated" > gpurun_out/t_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
for v in 0:0 9:1 9:2 9:3 ; do
  ch=${v%%:*}; tl=${v##*:}
  if [ $ch = 0 ]; then export HC_PHMM_RESCUE_CHAIN=0; else unset HC_PHMM_RESCUE_CHAIN; fi
  export HC_PHMM_RESCUE_CHAIN_TAIL=$tl
  for np_ in 20000 60000; do
    timeout -k 10 120 python bench.py --workload S4 --pairs $np_ --no-cpu --no-extra --steps 10 > gpurun_out/b_${TAG}_${np_}_${ch}_${tl}.json 2>/dev/null || exit 1
  done
done
