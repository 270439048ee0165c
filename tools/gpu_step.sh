set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_w2b.log 2>&1 || { tail -30 gpurun_out/t_w2b.log; exit 1; }
tail -2 gpurun_out/t_w2b.log
timeout -k 10 300 python -u tools/sweep.py S2 S2:125000 S1w:1000000 S1 S1w S4 > gpurun_out/sweep_w2b.jsonl 2>> gpurun_out/sweep.err || exit 1
cat gpurun_out/sweep_w2b.jsonl
