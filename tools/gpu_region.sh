# Region call checks: engine + pipeline GPU tests, then one-region A/B timings
# (structured vs general planner, tail order) and a phase trace.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_region_pipeline.py tests/test_gpu_cpp_shim.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 200 python -u tools/region_ab.py 128 HC_PHMM_GRID_PLAN=1,0 > gpurun_out/rab_${TAG}.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u tools/region_ab.py 32 HC_PHMM_GRID_PLAN=1,0 >> gpurun_out/rab_${TAG}.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u tools/region_ab.py 128 HC_PHMM_TAIL_ROUNDS=2,0 >> gpurun_out/rab_${TAG}.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u tools/region_ab.py 128 HC_PHMM_SEG_Q=-1,0,1 >> gpurun_out/rab_${TAG}.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u tools/region_ab.py 32 HC_PHMM_SEG_Q=-1,0,1 >> gpurun_out/rab_${TAG}.jsonl 2>&1 || exit 1
HC_PHMM_TRACE=1 timeout -k 10 100 python -u tools/region_trace.py 128 > gpurun_out/rtrace_${TAG}.log 2>&1 || exit 1
