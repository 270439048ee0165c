#!/bin/bash
# A/B: default seg kernel vs an alternative build (HC_PHMM_LIB), interleaved runs.
set -e
cd "$(dirname "$0")/.."
ALT=${1:-build_ab/libocc2.so}
for r in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu --no-extra --steps 10 > gpurun_out/ab_def_$r.json 2>/dev/null
  HC_PHMM_LIB=$ALT timeout -k 10 120 python bench.py --no-cpu --no-extra --steps 10 > gpurun_out/ab_alt_$r.json 2>/dev/null
done
HC_PHMM_TRACE=1 timeout -k 10 200 python tools/e2e_timing.py > gpurun_out/e2e.log 2>&1
echo done
