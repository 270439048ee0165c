set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t3.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/t3.log
[ $rc -eq 0 ] || exit $rc
bash tools/persist_ab.sh || exit 1
mkdir -p gpurun_out/w3
for L in new r3; do
  if [ $L = r3 ]; then export HC_PHMM_LIB=$PWD/ab_libs/libhcpairhmm_r3.so; else unset HC_PHMM_LIB; fi
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/w3/$L -o run -- python3 bench.py --workload S2 --steps 3 --warmup 1 --no-cpu --no-extra > gpurun_out/w3/$L.log 2>&1 || exit 1
done
