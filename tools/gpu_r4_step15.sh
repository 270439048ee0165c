# Round 4, step 15: the fp32 pass's width cap (HC_PHMM_SEG_CAP, 0 = the cap
# model's choice) at S4 (few, long pairs: latency-bound) and a 125k S2 batch.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
WL=S4 NO_R3=1 VARIANTS="c0:HC_PHMM_SEG_CAP=0 c48:HC_PHMM_SEG_CAP=48 c32:HC_PHMM_SEG_CAP=32 c24:HC_PHMM_SEG_CAP=24 c16:HC_PHMM_SEG_CAP=16" PAIRS="2000 20000" bash tools/persist_ab.sh || exit 1
NO_R3=1 VARIANTS="c0:HC_PHMM_SEG_CAP=0 c64:HC_PHMM_SEG_CAP=64 c48:HC_PHMM_SEG_CAP=48 c32:HC_PHMM_SEG_CAP=32" PAIRS="125000" bash tools/persist_ab.sh || exit 1
