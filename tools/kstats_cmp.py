"""Print the rocprofv3 kernel stats (avg us, calls) of several gpurun_out/<tag>/prof_* runs side by side."""
import csv, glob, sys
tags = sys.argv[1:]
tab = {}
for t in tags:
    f = glob.glob(f"gpurun_out/{t}/prof_*/run_kernel_stats.csv")[0]
    for r in csv.DictReader(open(f)):
        n = r["Name"].split("(")[0].replace("void ", "")[:48]
        tab.setdefault(n, {})[t] = (float(r["AverageNs"]) / 1e3, int(r["Calls"]))
for n, d in sorted(tab.items(), key=lambda kv: -max(v[0] * v[1] for v in kv[1].values())):
    print(f"{n:48s} " + " ".join(f"{d[t][0]:8.1f}us x{d[t][1]:<4d}" if t in d else f"{'-':>15s}" for t in tags))
