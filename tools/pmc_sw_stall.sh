#!/bin/bash
# Stall breakdown of the Smith-Waterman DP kernel on W2 (one PMC pass):
# wave cycles split into active-issue / issue-stall / parked (waitcnt), VALU
# issue, LDS issue stalls and the DVFS clock.
#   bash tools/pmc_sw_stall.sh TAG [env...]
set -e
TAG=${1:-r02}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmcsw_${TAG}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/a -o run -- python3 tools/sw_timing.py W2 > $OUT/a.log 2>&1
echo done
