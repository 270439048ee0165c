# Full GPU suite, then the persistent A/B against the round-3 library.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t2.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -5 gpurun_out/t2.log
[ $rc -eq 0 ] || exit $rc
bash tools/persist_ab.sh
