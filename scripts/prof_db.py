"""Kernel timeline / stats from a rocprofv3 rocpd database (rocprofv3 -d DIR -o NAME writes NAME_results.db).
Usage: python scripts/prof_db.py DB [--timeline N] [--csv OUT]   (stats per kernel; --csv writes them as CSV)"""
import argparse
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--timeline", type=int, default=0, help="print the last N dispatches with start gaps")
ap.add_argument("--csv", default=None)
a = ap.parse_args()
db = sqlite3.connect(a.db)
rows = db.execute("select name, start, end from kernels order by start").fetchall()
stats = {}
for name, s, e in rows:
    d = (e - s) / 1e3
    st = stats.setdefault(name, [])
    st.append(d)
out = []
for name, ds in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
    ds.sort()
    out.append((name, len(ds), sum(ds), sum(ds) / len(ds), ds[0], ds[-1]))
    print(f"{name[:70]:70s} calls {len(ds):5d} total_us {sum(ds):10.1f} avg_us {sum(ds)/len(ds):9.2f} "
          f"min {ds[0]:8.2f} max {ds[-1]:8.2f}")
if a.csv:
    with open(a.csv, "w") as f:
        f.write('"Name","Calls","TotalDurationUs","AverageUs","MinUs","MaxUs"\n')
        for r in out:
            f.write(f'"{r[0]}",{r[1]},{r[2]:.3f},{r[3]:.3f},{r[4]:.3f},{r[5]:.3f}\n')
if a.timeline:
    prev = None
    for name, s, e in rows[-a.timeline:]:
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"{name[:50]:50s} dur_us {(e - s) / 1e3:9.2f} gap_from_prev_end_us {gap:8.2f}")
        prev = e
