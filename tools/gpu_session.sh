set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2a.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -eq 0 ]; then
  HC_PHMM_TRACE=1 timeout -k 10 200 python tools/e2e_timing.py > gpurun_out/e2e_trace2.log 2>&1 && HC_PHMM_TRACE=1 timeout -k 10 120 python tools/region_trace.py 128 > gpurun_out/region_trace2.log 2>&1
fi
