# Round 4, step 11: per-phase host/device trace of the 415 x 128 region call
# (HC_PHMM_TRACE=1, 35 calls; the last ones are warm).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/s11
HC_PHMM_TRACE=1 timeout -k 10 120 python3 tools/region_prof.py 128 > gpurun_out/s11/trace.log 2>&1 || exit 1
tail -60 gpurun_out/s11/trace.log
