#!/bin/bash
# Kernel averages of the S2 end-to-end call's device preparation (flat_* and
# the seg pass) under settings: one rocprofv3 kernel-trace run per setting.
#   bash tools/prep_prof.sh base "blocks2k@HC_PHMM_PREP_BLOCKS=2048" ...
# A setting is TAG or TAG@ENV=V[,ENV=V]; output gpurun_out/prep_prof/TAG/.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for v in "$@"; do
  tag=${v%%@*}; envs=""; [ "$tag" != "$v" ] && envs=${v#*@}
  out=gpurun_out/prep_prof/$tag
  rm -rf $out; mkdir -p $out
  ( for kv in ${envs//,/ }; do export "$kv"; done
    REPS=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run \
        -- python3 tools/e2e_timing.py > $out/run.log 2>&1 ) || exit $?
  st=$(find $out -name '*kernel_stats.csv' | head -1)
  echo "== $tag ($envs)"
  python3 - "$st" <<'EOF'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(flat_\w+|phmm_seg_kernel|phmm_seg64_kernel|copyBuffer|fillBufferAligned|store_to_host_kernel)", r["Name"])
    if m:
        print(f'  {m.group(1):24s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"]) / 1e3:8.1f} us')
EOF
done
