# Round 4, step 18: SW's partial last stripe stops after n2 + r - 1 steps.
# The SW GPU tests, then W2 / W3 DP time against the library of 5b18c58
# (ab_libs/libhcpairhmm_r4c.so), two rounds.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/s18
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "sw" --timeout 300 --timeout-method thread > gpurun_out/s18/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/s18/tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for b in r4c tree; do
    lib=""; [ $b = tree ] || lib=$PWD/ab_libs/libhcpairhmm_$b.so
    echo -n "sw $b: "
    HC_PHMM_LIB=$lib timeout -k 10 200 python3 tools/sw_ab.py W2 W3 2>/dev/null || exit 1
  done
done
