# Instruction-cache counters and per-wave timelines of the fp32 seg pass at the
# 8-GPU shard size (125k pairs) and at full S2, persistent (P=1) and one wave
# per launched slot (P=0): does the shard's mid-pass issue loss follow
# instruction-cache misses (more block widths co-resident per CU pair)?
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/icache
timeout -k 5 60 rocprofv3 --list-avail > gpurun_out/icache/avail.txt 2>&1 || true
grep -i -E "SQC_ICACHE|SQ_IFETCH|SQ_WAIT_INST" gpurun_out/icache/avail.txt | head -20 || true
for P in 0 1; do
  for n in 125000 1000000; do
    HC_PHMM_SEG_PERSIST=$P timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_VALU SQ_WAVES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES \
        --output-format csv -d gpurun_out/icache/p_${n}_$P -o run -- \
        python3 bench.py --workload S2 --pairs $n --steps 3 --warmup 1 --no-cpu --no-extra > gpurun_out/icache/p_${n}_$P.log 2>&1 || echo "pmc $n $P failed"
  done
  HC_PHMM_SEG_PERSIST=$P timeout -k 10 120 python3 tools/timeline.py S2:125000 gpurun_out/icache/tl_125k_$P.npy > gpurun_out/icache/tl_125k_$P.json 2>&1 || exit 1
  cat gpurun_out/icache/tl_125k_$P.json
done
