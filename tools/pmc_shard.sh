# VALU instructions and issue counters of the seg kernel at S2 shard sizes
# (one PMC pass per size; compare lane-instructions per cell with full S2).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 125000 1000000; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcs_$n -o run -- python3 bench.py --workload S2 --pairs $n --steps 2 --warmup 1 --no-cpu --no-extra > gpurun_out/pmcs_$n.log 2>&1 || exit 1
done
