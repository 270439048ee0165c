#!/bin/bash
# Stall breakdown of the Smith-Waterman DP kernel on W2, two PMC passes (each
# within the SQ block's 8 slots): (a) wave cycles split into active-issue /
# issue-stall / parked (waitcnt), VALU issue, LDS issue stalls and the DVFS
# clock; (b) instruction mix: SALU, VALU, LDS, SMEM instructions and waves.
#   bash tools/pmc_sw_stall.sh TAG
set -e
TAG=${1:-r02}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmcsw_${TAG}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/a -o run -- python3 tools/sw_timing.py W2 > $OUT/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/b -o run -- python3 tools/sw_timing.py W2 > $OUT/b.log 2>&1
echo done
