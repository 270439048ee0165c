set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_cap.log 2>&1 || { tail -30 gpurun_out/t_cap.log; exit 1; }
tail -2 gpurun_out/t_cap.log
timeout -k 10 300 python -u tools/sweep.py S1 S1w S2:10000 S4 > gpurun_out/sweep_cap.jsonl 2> gpurun_out/sweep.err || exit 1
timeout -k 10 300 python -u tools/sweep.py S2:125000 S2:10000 --env HC_PHMM_SEG_CAP=-,64,48,32 >> gpurun_out/sweep_cap.jsonl 2>> gpurun_out/sweep.err || exit 1
cat gpurun_out/sweep_cap.jsonl
