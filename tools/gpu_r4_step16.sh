# Round 4, step 16: S4 (2 000 pairs) at warm clocks (300 untimed passes),
# fp64 issue priority and wave order, fp32 priority.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
WL=S4 NO_R3=1 WARM=300 STEPS=50 VARIANTS="d:HC_PHMM_PRIO64=1 q0:HC_PHMM_PRIO64=0 o0:HC_PHMM_RESCUE_ORDER=0 p1:HC_PHMM_PRIO=1 c24:HC_PHMM_SEG_CAP=24" PAIRS="2000" bash tools/persist_ab.sh || exit 1
