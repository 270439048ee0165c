"""Kernel + memory-copy timeline from rocprofv3 CSV output (--kernel-trace
--memory-copy-trace --output-format csv): the last N events in start order,
times relative to the first event shown. usage: timeline_csv.py dir [N]"""
import csv
import glob
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 80
ev = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r.get("Stream_Id", "?"),
                   r["Kernel_Name"].replace("hcphmm::(anonymous namespace)::", "")[:48]))
for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        b = int(r.get("Bytes", 0) or 0)
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", r.get("Stream_Id", "?"),
                   f"{r['Direction']} {b / 1e6:.1f} MB"))
ev.sort()
ev = ev[-n:]
t0 = ev[0][0]
for s, e, k, st, name in ev:
    print(f"{(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f} {k} st{st:>3s} {name}")
