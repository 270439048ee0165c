# Instruction-cache counters of the fp32 seg pass at the 8-GPU shard size
# (125k pairs) and at full S2: does the shard's mid-pass issue loss follow
# instruction-cache misses (more block widths co-resident per CU pair)?
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/icache
timeout -k 5 60 rocprofv3 --list-avail > gpurun_out/icache/avail.txt 2>&1 || true
for n in 125000 1000000; do
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
      --output-format csv -d gpurun_out/icache/p_$n -o run -- \
      python3 bench.py --workload S2 --pairs $n --steps 3 --warmup 1 --no-cpu --no-extra > gpurun_out/icache/p_$n.log 2>&1 || exit 1
done
