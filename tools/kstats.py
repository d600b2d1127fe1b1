"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv: tools/kstats.py DIR [N]"""
import csv, glob, sys
f = glob.glob(sys.argv[1].rstrip("/") + "/*kernel_stats.csv")[0]
rows = list(csv.DictReader(open(f)))
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    print(f"{r['Name'][:64]:64s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:10.2f}us {float(r['TotalDurationNs'])/1e6:9.3f}ms {float(r['Percentage']):6.2f}%")
