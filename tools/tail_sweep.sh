#!/bin/bash
# A/B of the seg-wave dispatch order (HC_PHMM_TAIL_ROUNDS: 0 = packing order,
# 2 = default, 1000 = global longest-first) at shard sizes of 1/2/4/8 GPUs.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for t in 0 2 4 1000; do
  for n in 125000 250000 1000000; do
    HC_PHMM_TAIL_ROUNDS=$t timeout -k 10 120 python bench.py --pairs $n --no-cpu --no-extra --steps 20 \
      > gpurun_out/tail_${t}_$n.json 2>/dev/null || exit 1
  done
done
