# A/B on one box: a saved library (ab_libs/libhcpairhmm_$BASE.so, default r3) against
# this tree's library under the variants in VARIANTS ("tag:ENV=V[,ENV=V]" ...;
# default: this tree's defaults only), at S2
# and its shards (PAIRS); 20 timed steps each, bench.py's HIP-event times.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pab
WL=${WL:-S2}
run() {  # tag n env...
  local tag=$1 n=$2; shift 2
  env "$@" timeout -k 10 120 python3 bench.py --workload $WL --pairs $n --steps ${STEPS:-20} --warmup ${WARM:-5} --no-cpu --no-extra \
      > gpurun_out/pab/b_${WL}_${n}_${tag}.json 2> gpurun_out/pab/b_${WL}_${n}_${tag}.err || return 1
  python3 -c "import json; d=json.load(open('gpurun_out/pab/b_${WL}_${n}_${tag}.json')); print('$WL', '$tag', $n, d['roofline']['kernel_ms'], d['kernel_ms_f64'], d['device_pass_ms'], d['roofline']['frac'])"
}
for rep in 1 2; do
  for n in ${PAIRS:-125000 250000 1000000}; do
    [ -n "$NO_R3" ] || run ${BASE:-r3}_$rep $n HC_PHMM_LIB=$PWD/ab_libs/libhcpairhmm_${BASE:-r3}.so || exit 1
    for v in ${VARIANTS:-tree:HC_PHMM_TRACE_UNSET=1}; do
      tag=${v%%:*}; envs=${v#*:}
      run ${tag}_$rep $n ${envs//,/ } || exit 1
    done
  done
done
