#!/bin/bash
# Committed profiles of one bench config at the current tree: a warm kernel
# trace (the first W launches of each kernel dropped from the average) and one
# PMC pass per counter group (FETCH_SIZE and WRITE_SIZE never share a pass).
# Outputs land in gpurun_out/prof_NAME/; ${ROUND}_pmc_NAME.json and
# ${ROUND}_NAME_kernel_stats.csv are then copied to profiles/ (ROUND: env,
# default r05).
#   bash tools/profile_cfg.sh WORKLOAD [PAIRS]     e.g. S2, S1, S4 20000
#   bash tools/profile_cfg.sh S2shard N            rank 0's shard of an N-way split
#   bash tools/profile_cfg.sh region NHAPS         (415 reads x NHAPS, tools/region_prof.py)
# NAME = WORKLOAD, WORKLOAD_PAIRS or S2shard_N (the key bench.py looks profiles up by).
set -e
WL=$1; NP=$2; W=5; ROUND=${ROUND:-r05}
NAME=$WL${NP:+_$NP}
ARGS="--workload $WL ${NP:+--pairs $NP} --steps 20 --warmup $W"
if [ "$WL" = S2shard ]; then ARGS="--workload S2 --shard-of $NP --steps 20 --warmup $W"; fi
B="python3 bench.py $ARGS --no-cpu --no-extra"
EXTRA=""
if [ "$WL" = region ]; then
    NAME=region_415x$NP
    B="python3 tools/region_prof.py $NP"
    EXTRA="--calls 35"
fi
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/prof_$NAME
rm -rf $OUT; mkdir -p $OUT
HC_BENCH_DETAIL=$PWD/$OUT/detail.json timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1
if [ "$WL" = region ]; then
    CELLS=$(python3 -c "import sys; sys.path.insert(0, 'gatk-haplotypecaller-cpp17_amd'); import workloads as W; print(W.cells(W.region_flat(*W.region(415, $NP))))")
    RC=0
else
    # cells and rescued cells of the profiled batch, from the bench run's detail record
    CELLS=$(python3 -c "import json; d=json.load(open('$OUT/detail.json')); print(d['config']['cells'])")
    RC=$(python3 -c "import json; d=json.load(open('$OUT/detail.json')); print(d['config'].get('rescued_cells') or 0)")
fi
python3 tools/profile_summary.py $OUT/${ROUND}_pmc_$NAME.json --trace $OUT/trace --skip $W --cells $CELLS --rescued-cells $RC $EXTRA \
    fetch=$OUT/fetch write=$OUT/write sq=$OUT/sq > $OUT/summary.log
cp $OUT/trace/run_kernel_stats.csv $OUT/${ROUND}_${NAME}_kernel_stats.csv
cat $OUT/summary.log
