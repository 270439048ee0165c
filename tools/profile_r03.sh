#!/bin/bash
# Committed profiles of one bench config at the current HEAD: a warm kernel
# trace (the first W launches of each kernel dropped from the average) and one
# PMC pass per counter group (FETCH_SIZE and WRITE_SIZE never share a pass).
# Outputs land in gpurun_out/prof3_NAME/ (merged back from the GPU box);
# r03_pmc_NAME.json and r03_NAME_kernel_stats.csv are then copied to profiles/.
#   bash tools/profile_r03.sh WORKLOAD [PAIRS]
# NAME = WORKLOAD or WORKLOAD_PAIRS (the key bench.py looks the profile up by).
set -e
#   bash tools/profile_r03.sh region NHAPS     (415 reads x NHAPS, tools/region_prof.py)
WL=$1; NP=$2; W=5
NAME=$WL${NP:+_$NP}
ARGS="--workload $WL ${NP:+--pairs $NP} --steps 20 --warmup $W"
B="python3 bench.py $ARGS --no-cpu --no-extra"
EXTRA=""
if [ "$WL" = region ]; then
    NAME=region_415x$NP
    B="python3 tools/region_prof.py $NP"
    EXTRA="--calls 35"
fi
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
if [ "$WL" = region ]; then
    CELLS=$(python3 -c "import sys; sys.path.insert(0, 'gatk-haplotypecaller-cpp17_amd'); import workloads as W; print(W.cells(W.region_flat(*W.region(415, $NP))))")
else
    CELLS=$(python3 -c "import sys; sys.path.insert(0, 'gatk-haplotypecaller-cpp17_amd'); import workloads as W; print(W.cells(W.config('$WL', ${NP:-None})))")
fi
OUT=gpurun_out/prof3_$NAME
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1
python3 tools/profile_summary.py $OUT/r03_pmc_$NAME.json --trace $OUT/trace --skip $W --cells $CELLS $EXTRA \
    fetch=$OUT/fetch write=$OUT/write sq=$OUT/sq > $OUT/summary.log
cp $OUT/trace/run_kernel_stats.csv $OUT/r03_${NAME}_kernel_stats.csv
cat $OUT/summary.log
