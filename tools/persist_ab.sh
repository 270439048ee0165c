# A/B on one box: the round-3 library (ab_libs/libhcpairhmm_r3.so, one wave per
# launched slot) against this tree's library with the persistent fp32 seg pass
# (HC_PHMM_SEG_PERSIST=1) and without it (=0), at S2 and its 1/4 and 1/8
# shards; 20 timed steps each, bench.py's HIP-event kernel time.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pab
run() {  # tag n env...
  local tag=$1 n=$2; shift 2
  env "$@" timeout -k 10 120 python3 bench.py --workload S2 --pairs $n --steps 20 --warmup 5 --no-cpu --no-extra \
      > gpurun_out/pab/b_${n}_${tag}.json 2> gpurun_out/pab/b_${n}_${tag}.err || return 1
  python3 -c "import json; d=json.load(open('gpurun_out/pab/b_${n}_${tag}.json')); print('$tag', $n, d['roofline']['kernel_ms'], d['device_pass_ms'], d['roofline']['frac'])"
}
for rep in 1 2; do
  for n in ${PAIRS:-125000 250000 1000000}; do
    run r3_$rep $n HC_PHMM_LIB=$PWD/ab_libs/libhcpairhmm_r3.so || exit 1
    run p0_$rep $n HC_PHMM_SEG_PERSIST=0 || exit 1
    run p1_$rep $n HC_PHMM_SEG_PERSIST=1 || exit 1
  done
done
