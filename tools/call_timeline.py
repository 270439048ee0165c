"""Device timeline of repeated calls from a rocprofv3 trace (kernel + memory
copy traces, CSV): for each of the last N calls, every kernel and copy with
its start relative to the call's first device operation, its duration, and
the idle gaps between them (verdict round 4, item 3: where a region call's
time goes outside the kernels). A call starts at a copy that follows a gap of
more than --gap-us microseconds.

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d OUT -o run -- \
        python3 tools/region_prof.py 128
    python3 tools/call_timeline.py OUT [--calls 3] [--gap-us 50]
"""
import csv
import glob
import os
import sys


def load(d):
    ev = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:60]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kind = r.get("Direction") or r.get("Operation") or "copy"
            size = r.get("Bytes") or r.get("Size") or ""
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f"C {kind} {size}"))
    ev.sort()
    return ev


def main():
    d = sys.argv[1]
    ncalls = int(sys.argv[sys.argv.index("--calls") + 1]) if "--calls" in sys.argv else 3
    gap = float(sys.argv[sys.argv.index("--gap-us") + 1]) if "--gap-us" in sys.argv else 50.0
    ev = load(d)
    starts = [0]
    for k in range(1, len(ev)):
        if (ev[k][0] - max(e[1] for e in ev[max(0, k - 8):k])) / 1e3 > gap:
            starts.append(k)
    starts.append(len(ev))
    calls = [ev[starts[i]:starts[i + 1]] for i in range(len(starts) - 1)]
    for c in calls[-ncalls:]:
        t0 = c[0][0]
        end = t0
        print(f"--- call: {len(c)} device operations, span {(max(e[1] for e in c) - t0) / 1e3:.1f} us")
        busy = 0.0
        for s, e, name in c:
            idle = max(0.0, (s - end) / 1e3)
            print(f"  +{(s - t0) / 1e3:8.1f} us  {(e - s) / 1e3:8.1f} us  (idle before {idle:6.1f})  {name}")
            busy += (e - s) / 1e3
            end = max(end, e)
        print(f"  busy {busy:.1f} us")


if __name__ == "__main__":
    main()
