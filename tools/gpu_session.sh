# GPU session: the whole -m gpu suite, then the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2b.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r2b.json 2> gpurun_out/bench_r2b.err
