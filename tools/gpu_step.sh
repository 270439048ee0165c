set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region_pipeline.py -x -v -s --timeout 500 --timeout-method thread > gpurun_out/t_pipe.log 2>&1 || { tail -40 gpurun_out/t_pipe.log; exit 1; }
grep -E "sites|passed|failed" gpurun_out/t_pipe.log | tail -5
