"""Per-LAUNCH counter totals of the matcher's 2-NN kernels from tools/pmc_match.sh passes:
python tools/pmc_launch_json.py DIR N_LAUNCHES OUT.json   (tooling, not product)

Since r04 a two-pass launch is several dispatches per kernel (the screen in batches on two streams,
pass 2 per batch: matcher.cpp launch_two_pass_overlap), so a per-dispatch mean is no longer a
per-launch figure.  Every counter is summed over all dispatches of a kernel in the profiled run and
divided by the number of matcher launches in it (bench.py: warm-up + timed steps + the event steps
+ the PCIe-inclusive call).  FETCH_SIZE / WRITE_SIZE stay in KiB (HBM read bytes = 2 x FETCH_SIZE on
gfx950, MI355X_MICROARCH.md); bench.py's pmc_traffic reads this file's layout
({kernel: {counter: per-launch value}})."""
import collections
import csv
import glob
import json
import sys

D, n_launch, out_path = sys.argv[1].rstrip("/"), int(sys.argv[2]), sys.argv[3]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(D + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add((f, r["Dispatch_Id"]))
out = {}
for k, cs in tot.items():
    out[k] = {c: v / n_launch for c, v in cs.items()}
    out[k]["dispatches_per_launch"] = max(len(disp[(k, c)]) for c in cs) / n_launch
out["_what"] = {"launches": n_launch, "dir": D,
                "note": "counter totals per matcher launch (all dispatches of the kernel / launches)"}
json.dump(out, open(out_path, "w"), indent=1)
for k, v in out.items():
    if k.startswith("_"):
        continue
    mb = (2 * v.get("FETCH_SIZE", 0) + v.get("WRITE_SIZE", 0)) * 1024 / 1e6
    print(f"{k.split('(')[0][-48:]:48s} {v['dispatches_per_launch']:5.1f} dispatches/launch  {mb:9.1f} MB/launch")
