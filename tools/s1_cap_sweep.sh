# S1 / S1w fp32 kernel time under forced width caps (host planner) vs the default plan.
set -o pipefail
mkdir -p gpurun_out
for wl in S1 S1w; do
  for cap in 0 8 10 12 14 16 18 20 22; do
    HC_PHMM_SEG_CAP=$cap timeout -k 10 120 python bench.py --workload $wl --no-cpu --no-extra --steps 50 --warmup 10 > gpurun_out/s1cap_${wl}_$cap.json 2>/dev/null || exit 1
  done
done
