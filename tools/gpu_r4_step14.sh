# Round 4, step 14: the default bench line again (secondaries with 5 untimed + 10 timed passes).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/s14
timeout -k 10 600 python3 bench.py > gpurun_out/s14/bench.json 2> gpurun_out/s14/bench.err || exit 1
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/s14/bench.json"))
print(d["value"], d["device_pass_ms"], d["roofline"]["frac"])
for k, v in d["secondary"].items():
    print(k, {a: b for a, b in v.items() if a in ("device_pass_ms", "kernel_ms_f32", "kernel_ms_f64", "call_ms", "dp_kernel_ms", "implied_efficiency_vs_1gpu")},
          (v.get("roofline_f64") or v.get("roofline") or {}).get("frac"))
PY
