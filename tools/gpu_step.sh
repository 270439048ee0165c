set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/sweep.py region:415:128 region:415:32 --env HC_PHMM_SEG_CAP=-,64,48,32 > gpurun_out/sweep_region.jsonl 2> gpurun_out/sweep.err || exit 1
timeout -k 10 300 python -u tools/sweep.py region:415:128 --env HC_PHMM_TAIL_ROUNDS=0,2,4 >> gpurun_out/sweep_region.jsonl 2>> gpurun_out/sweep.err || exit 1
cat gpurun_out/sweep_region.jsonl
