# Chained fp64 rescue check: rescue / golden parity tests, then S4 lines
# (2 000 and 20 000 pairs), chained and unchained (HC_PHMM_RESCUE_CHAIN=0).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "rescue or golden or s4 or repeated" > gpurun_out/t_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
for np_ in 2000 20000; do
  timeout -k 10 120 python bench.py --workload S4 --pairs $np_ --no-cpu --no-extra --steps 20 > gpurun_out/b_${TAG}_S4_$np_.json 2> gpurun_out/b_${TAG}_S4_$np_.err || exit 1
  HC_PHMM_RESCUE_CHAIN=0 timeout -k 10 120 python bench.py --workload S4 --pairs $np_ --no-cpu --no-extra --steps 20 > gpurun_out/b_${TAG}_S4_${np_}_nochain.json 2> gpurun_out/b_${TAG}_S4_${np_}_nochain.err || exit 1
done
