set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_inwave.log 2>&1 || { tail -30 gpurun_out/t_inwave.log; exit 1; }
tail -2 gpurun_out/t_inwave.log
timeout -k 10 300 python -u tools/sweep.py S2 S2:125000 S4 --env HC_PHMM_RESCUE_IN_WAVE=1,0 > gpurun_out/sweep_inwave.jsonl 2> gpurun_out/sweep.err || exit 1
cat gpurun_out/sweep_inwave.jsonl
