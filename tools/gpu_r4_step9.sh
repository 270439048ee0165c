# Round 4, step 9: seg waves per workgroup (1 / 2 / 4, A/B libraries built with
# EXTRA_DEV_FLAGS=-DHC_SEG_WPB=n) at S2, a 125k shard, S1 and the 415 x 128
# region call; the tree (4) also checks the solo run's single end marker (S1).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for b in wpb1 wpb2; do
  BASE=$b VARIANTS="wpb4:HC_PHMM_PRIO=0" PAIRS="125000 1000000" bash tools/persist_ab.sh || exit 1
done
WL=S1 BASE=wpb1 VARIANTS="wpb4:HC_PHMM_PRIO=0" PAIRS="10000" bash tools/persist_ab.sh || exit 1
for rep in 1 2; do
  for b in wpb1 wpb2 tree; do
    lib=""; [ $b = tree ] || lib=$PWD/ab_libs/libhcpairhmm_$b.so
    echo -n "region $b: "
    HC_PHMM_LIB=$lib timeout -k 10 120 python3 tools/region_ab.py 128 HC_PHMM_X=0 2>/dev/null || exit 1
  done
done
