# Column-segmentation sweep on one GPU: parity of the segmented paths, then the
# 125k-pair shard (one rank's share of configs[3] at 8 GPUs) at several
# latency-cap divisors, batch sizes, and a kernel trace of the shard.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "seg or shard" > gpurun_out/seg_tests.log 2>&1 || { tail -30 gpurun_out/seg_tests.log; exit 1; }
tail -1 gpurun_out/seg_tests.log
for c in off 1 2 4 8; do
  if [ $c = off ]; then export HC_PHMM_LANE_SEG=off; else export HC_PHMM_LANE_SEG=auto HC_PHMM_SEG_CAP=$c; fi
  timeout -k 10 300 python bench.py --no-cpu --no-extra --steps 20 --pairs 125000 > gpurun_out/cap_$c.json 2>> gpurun_out/shard.err
  python -c "import json;d=json.load(open('gpurun_out/cap_$c.json'));print('cap', '$c', d['value'], d['roofline']['kernel_ms'])"
done
unset HC_PHMM_LANE_SEG HC_PHMM_SEG_CAP
for n in 250000 500000 1000000; do
  timeout -k 10 300 python bench.py --no-cpu --no-extra --steps 20 --pairs $n > gpurun_out/n_$n.json 2>> gpurun_out/shard.err
  python -c "import json;d=json.load(open('gpurun_out/n_$n.json'));print('n', $n, d['value'], d['roofline']['kernel_ms'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_shard -o shard -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-extra --steps 5 --warmup 1 --pairs 125000 > /dev/null 2>&1
