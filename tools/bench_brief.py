"""One line from a bench.py detail file (HC_BENCH_DETAIL): headline, roofline and the secondary
configs' device times (tools/gpu_run.sh prints it after each bench step)."""
import json
import sys

d = json.load(open(sys.argv[1]))
print(f"value {d['value']} {d['unit']}  ms/step {d['ms_per_step']}  frac {d['roofline']['frac']}  "
      f"fp32 {d['roofline']['kernel_ms']} ms  fp64 {d.get('kernel_ms_f64')} ms")
for k, v in (d.get("secondary") or {}).items():
    keys = ("device_pass_ms", "device_pass_ms_cold", "kernel_ms_f32", "kernel_ms_f64", "frac_f32_kernel", "call_ms",
            "call_ms_cold", "gcups")
    f64 = (v.get("roofline_f64") or {}).get("frac")
    rp = (v.get("roofline_pass") or {}).get("frac")
    print(f"  {k}: " + " ".join(f"{x}={v[x]}" for x in keys if x in v) + (f" f64frac={f64}" if f64 else "")
          + (f" passfrac={rp}" if rp else ""))
for k in ("end_to_end_gcups", "end_to_end_ms", "end_to_end_first_call_ms"):
    if k in d:
        print(f"  {k}={d[k]}")
