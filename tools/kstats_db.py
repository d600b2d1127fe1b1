"""Per-kernel duration stats from a rocprofv3 SQLite results database (tooling, not product):
python tools/kstats_db.py <results.db> [name-filter]"""
import sqlite3
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
names = {r[0]: r[1] for r in db.execute("select id, coalesce(truncated_kernel_name, kernel_name) from kernel_symbols")}
d = defaultdict(list)
for kid, s, e in db.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
    d[names.get(kid, str(kid))].append((e - s) / 1e3)
rows = sorted(((sum(v), k, len(v)) for k, v in d.items() if flt in k), reverse=True)
tot = sum(r[0] for r in rows)
print(f"{'kernel':60s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s} {'pct':>6s}")
for t, k, n in rows:
    print(f"{k[:60]:60s} {n:6d} {t:10.1f} {t / n:9.2f} {100 * t / tot:6.1f}")
