# One GPU session: the -m gpu suite, then optional extra steps given as
# arguments (each its own time-limited command). Stops at the first failure.
# usage: bash tools/gpu_check.sh TAG ["cmd1" "cmd2" ...]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$tag.log
for c in "$@"; do
    echo "== $c"
    timeout -k 10 300 bash -c "$c" || exit 1
done
