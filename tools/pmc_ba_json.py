"""HBM traffic per LM iteration of the BA leg from the PMC passes of tools/pmc_ba.sh:
tools/pmc_ba_json.py DIR OUT.json.  Bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB counters; gfx950
FETCH_SIZE counts half of a wide streaming read, MI355X_MICROARCH.md HBM section), summed over
every BA dispatch of the profiled `bench.py --only-ba` run (a 1-iteration warm-up run + the timed
run) and divided by its LM iterations: one per ba_gschur dispatch (an LM step) plus iteration 0
(the initial linearization) of each of the two runs."""
import collections, csv, glob, json, sys

D = sys.argv[1].rstrip("/") + "/"
per = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.Counter()
for f in sorted(glob.glob(D + "p[12]_counter_collection.csv")):
    seen = set()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        c = r["Counter_Name"]
        per[k][c] += float(r["Counter_Value"])
        if c == "FETCH_SIZE" and (r.get("Dispatch_Id"), k) not in seen:
            seen.add((r.get("Dispatch_Id"), k))
            calls[k] += 1
steps = sum(v for k, v in calls.items() if "ba_gschur" in k)
iters = steps + 2
kern = {}
total = 0.0
for k, v in per.items():
    b = 2 * v.get("FETCH_SIZE", 0) * 1024 + v.get("WRITE_SIZE", 0) * 1024
    kern[k] = {"bytes_per_iteration": b / iters, "dispatches": calls[k]}
    total += b
out = {"what": "HBM bytes per LM iteration, BA C5 (bench.py --only-ba), 2 x FETCH_SIZE + WRITE_SIZE",
       "lm_steps": steps, "iterations": iters, "bytes_per_iteration": total / iters, "kernels": kern}
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(f"{total / iters / 1e6:.1f} MB per iteration over {iters} iterations")
for k, v in sorted(kern.items(), key=lambda kv: -kv[1]["bytes_per_iteration"]):
    print(f"  {k[:50]:50s} {v['bytes_per_iteration'] / 1e6:8.1f} MB  ({v['dispatches']} dispatches)")
