# Round-4 closing check at HEAD: the GPU suite, smoke(), and the default bench
# line (BENCH contract: N=1 with the CPU baseline and every secondary).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/final/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit 1
tail -2 gpurun_out/final/smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/final/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['device_pass_ms'])"
