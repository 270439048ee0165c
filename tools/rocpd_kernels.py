"""Per-kernel summary (and optionally the dispatch timeline) from a rocprofv3
rocpd .db: usage rocpd_kernels.py file.db [--timeline N]"""
import glob
import sqlite3
import sys

f = sys.argv[1]
if not f.endswith(".db"):
    f = glob.glob(f + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(f)
rows = list(c.execute("select name, count(*), avg(duration), sum(duration), max(vgpr_count), max(accum_vgpr_count), "
                      "max(scratch_size) from kernels group by name order by sum(duration) desc"))
print(f"{'kernel':70s} {'calls':>5s} {'avg_us':>9s} {'total_us':>10s} vgpr agpr scr")
for n, k, a, s, v, ag, sc in rows:
    n = n.replace("hcphmm::(anonymous namespace)::", "")[:70]
    print(f"{n:70s} {k:5d} {a/1e3:9.1f} {s/1e3:10.1f} {v:4d} {ag:4d} {sc}")
if "--timeline" in sys.argv:
    n = int(sys.argv[sys.argv.index("--timeline") + 1])
    t = list(c.execute("select name, start, end, stream_id, grid_x from kernels order by start"))
    t0 = t[0][1]
    for name, s, e, st, g in t[-n:]:
        print(f"{(s-t0)/1e3:12.1f} {(e-t0)/1e3:12.1f} {(e-s)/1e3:9.1f} st{st} grid {g:8d} {name.replace('hcphmm::(anonymous namespace)::','')[:60]}")
