#!/bin/bash
# Kernel trace of the small-batch configs (S1, S1w) and a width-cap sweep on S1.
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/small_trace
mkdir -p $OUT
for wl in S1 S1w; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$wl -o run -- python3 bench.py --workload $wl --no-cpu --no-extra --steps 20 > $OUT/$wl.log 2>&1
done
for cap in 16 24 32 48 64; do
  HC_PHMM_SEG_CAP=$cap timeout -k 10 120 python3 bench.py --workload S1 --no-cpu --no-extra --steps 20 > $OUT/cap_$cap.json 2>/dev/null
done
echo done
