#!/bin/bash
# One GPU-box session: the named steps in order, each under its own time limit,
# stopping at the first failure (a fault, abort or time-out ends the call).
# Logs go to gpurun_out/$TAG/.
#
#   bash tools/gpu_run.sh TAG STEP [STEP ...]
#
# Steps:
#   tests                     the whole -m gpu suite
#   tests:EXPR                the -m gpu tests matching pytest -k EXPR
#   smoke                     __graft_entry__.smoke()
#   bench                     bench.py with its defaults (the BENCH line)
#   bench:ARGS                bench.py ARGS (commas for spaces), e.g. bench:--workload,S4,--no-cpu,--no-extra
#   profile:CFG               tools/profile_cfg.sh CFG (commas for spaces), e.g. profile:S4,20000
#   profiles                  every bench config's profile (S2 S1 S4 S4_20000 both shards, the region)
#   ab:WL:PAIRS:VARIANTS      tools/persist_ab.sh with NO_R3=1; PAIRS comma-separated, VARIANTS
#                             "tag@ENV=V,ENV=V/tag2@ENV=V" (e.g. ab:S4:2000,20000:on@HC_PHMM_X=1/off@HC_PHMM_X=0)
#   region:VARIANTS           tools/region_ab.py 128 VARIANTS (e.g. HC_PHMM_X=0,1; "X=0,1;Y=2,3": cross product)
#   timeline[:NH]             the region call's host phases and device timeline (tools/call_timeline.py)
#   e2etl                     the same for the S2 flat call (tools/e2e_timing.py)
#   py:SCRIPT[,ARGS]          python3 tools/SCRIPT ARGS ("py:SCRIPT A=1,2 B=3" when ARGS hold commas)
# A/B libraries: ab_libs/ is not pushed to the box (.gpurunignore); copy the
# builds an A/B run needs into ab_stage/ first and name them there.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for step in "$@"; do
  name=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  echo "== $step"
  case $name in
    tests)
      k=(); [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
          > $OUT/gpu_tests${arg:+_x}.log 2>&1
      rc=$?; tail -3 $OUT/gpu_tests${arg:+_x}.log ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$?; tail -2 $OUT/smoke.log ;;
    bench)
      n=$(ls $OUT | grep -c '^bench')
      HC_BENCH_DETAIL=$PWD/$OUT/bench_${n}_detail.json timeout -k 10 600 python3 bench.py ${arg//,/ } \
          > $OUT/bench_$n.json 2> $OUT/bench_$n.err
      rc=$?
      [ $rc -eq 0 ] && python3 tools/bench_brief.py $OUT/bench_${n}_detail.json && wc -c $OUT/bench_$n.json ;;
    profile)
      timeout -k 10 900 bash tools/profile_cfg.sh ${arg//,/ } > $OUT/profile_${arg//,/_}.log 2>&1
      rc=$?; tail -1 $OUT/profile_${arg//,/_}.log | cut -c1-600 ;;
    profiles)
      rc=0
      for c in S2 S1 S4 S4,20000 S2shard,8 S2shard,4 region,128; do
        timeout -k 10 900 bash tools/profile_cfg.sh ${c//,/ } > $OUT/profile_${c//,/_}.log 2>&1 || { rc=$?; break; }
        echo "$c: $(tail -1 $OUT/profile_${c//,/_}.log | cut -c1-400)"
      done ;;
    ab)
      IFS=: read -r wl pairs vars <<< "$arg"
      vv=$(echo "$vars" | tr '/' ' ' | tr '@' ':')
      WL=$wl NO_R3=1 PAIRS="${pairs//,/ }" VARIANTS="$vv" bash tools/persist_ab.sh
      rc=$? ;;
    region)
      timeout -k 10 300 python3 tools/region_ab.py 128 ${arg//;/ }
      rc=$? ;;
    timeline)
      # Region call breakdown: host phases (HC_PHMM_TRACE) and the device
      # timeline of the last calls (kernels + copies) for NH haplotypes.
      nh=${arg:-128}
      HC_PHMM_TRACE=1 timeout -k 10 120 python3 tools/region_trace.py $nh > $OUT/region_trace_$nh.log 2>&1 &&
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tl_$nh -o run \
          -- python3 tools/region_prof.py $nh > $OUT/tl_$nh.log 2>&1 &&
      python3 tools/call_timeline.py $OUT/tl_$nh --calls 3 > $OUT/call_timeline_$nh.txt
      rc=$?; tail -25 $OUT/call_timeline_$nh.txt 2>/dev/null ;;
    e2etl)
      # The S2 flat call (host buffers in, log10 out): host phases and the
      # device timeline of its last call.
      HC_PHMM_TRACE=1 REPS=4 timeout -k 10 180 python3 tools/e2e_timing.py > $OUT/e2e_trace.log 2>&1 &&
      REPS=4 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tl_e2e -o run \
          -- python3 tools/e2e_timing.py > $OUT/tl_e2e.log 2>&1 &&
      python3 tools/call_timeline.py $OUT/tl_e2e --calls 1 --gap-us 1000 > $OUT/call_timeline_e2e.txt
      rc=$?; tail -40 $OUT/call_timeline_e2e.txt 2>/dev/null ;;
    py)
      # Spaces in ARGS: taken as they are (commas kept); otherwise commas for spaces.
      case "$arg" in *" "*) a=$arg ;; *) a=${arg//,/ } ;; esac
      timeout -k 10 600 python3 tools/$a
      rc=$? ;;
    *) echo "unknown step $name"; rc=2 ;;
  esac
  echo "== $step rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
