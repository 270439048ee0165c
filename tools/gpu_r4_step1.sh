set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or s1 or use_double" > gpurun_out/t1.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/t1.log
bash tools/persist_ab.sh
