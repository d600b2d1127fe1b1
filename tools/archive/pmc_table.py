"""Mean counter values per kernel from a pmc_* directory: tools/pmc_table.py DIR"""
import csv, collections, glob, json, sys
D = sys.argv[1].rstrip("/") + "/"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(D + "p*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: sum(x) / len(x) for c, x in v.items()} for k, v in agg.items()}
print(json.dumps(out, indent=1))
