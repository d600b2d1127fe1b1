"""Per-kernel, per-dispatch mean of every counter in the rocprofv3 --pmc CSV passes
under DIR (DIR/*counter_collection.csv), as JSON: tools/pmc_csv_summary.py DIR.
FETCH_SIZE / WRITE_SIZE stay in the counter's KiB (gfx950: HBM read bytes =
2 x FETCH_SIZE, MI355X_MICROARCH.md's correction)."""
import collections
import csv
import glob
import json
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))   # (kernel, counter) -> dispatch -> value
for f in glob.glob(sys.argv[1].rstrip("/") + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"], r["Counter_Name"])][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
out = collections.defaultdict(dict)
for (k, c), d in sorted(acc.items()):
    out[k][c] = sum(d.values()) / len(d)
json.dump(out, sys.stdout, indent=1)
