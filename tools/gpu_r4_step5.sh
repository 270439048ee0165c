set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t5.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/t5.log
[ $rc -eq 0 ] || exit $rc
NO_R3=1 VARIANTS="p0:HC_PHMM_PRIO=0" PAIRS="125000 1000000" bash tools/persist_ab.sh || exit 1
NO_R3=1 WL=S4 VARIANTS="p0:HC_PHMM_PRIO=0 q0:HC_PHMM_PRIO64=0" PAIRS="2000 20000" bash tools/persist_ab.sh || exit 1
NO_R3=1 WL=S1 VARIANTS="p0:HC_PHMM_PRIO=0" PAIRS="10000" bash tools/persist_ab.sh || exit 1
mkdir -p gpurun_out/w5
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/w5/new -o run -- python3 bench.py --workload S2 --steps 3 --warmup 1 --no-cpu --no-extra > gpurun_out/w5/new.log 2>&1 || exit 1
