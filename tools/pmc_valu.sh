#!/bin/bash
# VALU utilisation / stall / clock counters for the bench workload (one group per pass).
set -e
TAG=${1:-r01}; WL=${2:-S2}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmcv_${TAG}_${WL}
mkdir -p $OUT
B="python3 bench.py --workload $WL --steps 2 --warmup 1 --no-cpu --no-extra"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_VALU --output-format csv -d $OUT/a -o run -- $B > $OUT/a.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES SQ_INST_CYCLES_VMEM_RD --output-format csv -d $OUT/b -o run -- $B > $OUT/b.log 2>&1
echo done
