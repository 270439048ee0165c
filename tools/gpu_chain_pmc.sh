# Stall counters of the fp64 rescue kernel, chained vs unchained (S4, 20 000 pairs).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-x}
export TMPDIR=/tmp
B="python3 bench.py --workload S4 --pairs 20000 --no-cpu --no-extra --steps 3 --warmup 1"
for mode in chain nochain; do
  if [ $mode = nochain ]; then export HC_PHMM_RESCUE_CHAIN=0; else unset HC_PHMM_RESCUE_CHAIN; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc_${TAG}_$mode -o run -- $B > gpurun_out/pmc_${TAG}_$mode.log 2>&1 || exit 1
done
