# Column segmentation vs batch size: all-segmented, auto at several divisors.
set -e
cd $GRAFT_REPO_ROOT
run() {  # tag n
  timeout -k 10 300 python bench.py --no-cpu --no-extra --steps 20 --pairs $2 > gpurun_out/sw_$1_$2.json 2>> gpurun_out/shard.err
  python -c "import json;d=json.load(open('gpurun_out/sw_$1_$2.json'));print('$1', $2, d['value'], d['roofline']['kernel_ms'])"
}
for n in 125000 250000 500000 1000000; do
  HC_PHMM_LANE_SEG=all run all $n
  HC_PHMM_SEG_CAP=8 run cap8 $n
  HC_PHMM_SEG_CAP=16 run cap16 $n
  HC_PHMM_SEG_CAP=32 run cap32 $n
done
