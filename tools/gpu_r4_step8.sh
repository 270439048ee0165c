# Round 4, step 8: the GPU suite at the tree (solo small parts, spill-free seg
# kernel), then the tree against the library of commit 9ec30d3
# (ab_libs/libhcpairhmm_r4a.so) at S2 / a 125k shard / S1 / S1w / S4, and the
# seg kernel's WRITE_SIZE at S2.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/s8
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s8/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/s8/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
BASE=r4a VARIANTS="new:HC_PHMM_PRIO=0" PAIRS="125000 1000000" bash tools/persist_ab.sh || exit 1
for wl in S1 S1w; do
  WL=$wl BASE=r4a VARIANTS="new:HC_PHMM_PRIO=0 nosolo:HC_PHMM_SOLO_MAX_PAIRS=0" PAIRS="10000" bash tools/persist_ab.sh || exit 1
done
WL=S4 BASE=r4a VARIANTS="new:HC_PHMM_PRIO=0" PAIRS="2000" bash tools/persist_ab.sh || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/s8/write -o run -- \
    python3 bench.py --workload S2 --steps 5 --warmup 2 --no-cpu --no-extra > gpurun_out/s8/write.log 2>&1 || exit 1
python3 - <<'EOF'
import csv, glob, collections
s = collections.defaultdict(list)
for f in glob.glob("gpurun_out/s8/write/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        s[r["Kernel_Name"][:40]].append(float(r["Counter_Value"]))
for k, v in s.items():
    print("WRITE_SIZE", k, len(v), "launches, mean MB", round(sum(v) / len(v) / 1e3, 2) if v else None)
EOF
