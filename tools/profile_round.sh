#!/bin/bash
# Profile the bench workload on the GPU box: kernel trace + stats, then one PMC
# pass per counter group (FETCH_SIZE and WRITE_SIZE never share a pass; no
# pass exceeds the per-block counter limits of MI355X_MICROARCH.md).
#   bash tools/profile_round.sh TAG WORKLOAD
set -e
TAG=${1:-r01}
WL=${2:-S2}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}_${WL}
mkdir -p $OUT
B="python3 bench.py --workload $WL --steps 3 --warmup 1 --no-cpu --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/a -o run -- $B > $OUT/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD --output-format csv -d $OUT/b -o run -- $B > $OUT/b.log 2>&1
echo done
