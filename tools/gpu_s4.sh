# fp64 rescue check: parity + engine GPU tests, then S4 / S2 bench lines.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
for wl in S4 S2; do
  timeout -k 10 120 python bench.py --workload $wl --no-cpu --no-extra --steps 20 > gpurun_out/b_${TAG}_$wl.json 2> gpurun_out/b_${TAG}_$wl.err || exit 1
done
