"""Per-kernel duration summary from a rocprofv3 --kernel-trace database."""
import glob
import sqlite3
import sys

db = sys.argv[1]
if not db.endswith(".db"):
    db = glob.glob(f"{db}/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
rows = list(c.execute("select name, count(*), avg(end-start), sum(end-start) from kernels group by name order by 4 desc"))
out = sys.argv[2] if len(sys.argv) > 2 else None
lines = ["Name,Calls,AverageNs,TotalNs"] + ['"%s",%d,%.1f,%d' % r for r in rows]
if out:
    open(out, "w").write("\n".join(lines) + "\n")
for r in rows:
    print(f"{r[0][:90]:90s} {r[1]:5d} {r[2] / 1000:9.1f} us {r[3] / 1e6:8.2f} ms")
