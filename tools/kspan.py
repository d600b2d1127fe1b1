"""Per-launch span of the 2-NN kernels from a rocprofv3 kernel trace (tooling, not product):
python tools/kspan.py <results.db | kernel_trace.csv> [sift|orb]

The matcher's two-pass launch is several dispatches on three streams (screen batches on two,
pass 2 behind events on a third: matcher.cpp launch_two_pass_overlap), so no single kernel's
average is the launch time.  A launch here = the dispatches between two `prep_` dispatches (every
bench step starts with set_images_device's prepare kernel); its span = first screen start to last
screen / subset / settle end, which is what the bench's HIP events around the launch measure
(roofline.kernel_ms_per_launch).  Prints per-launch span, summed screen time and dispatch counts."""
import csv
import sqlite3
import statistics
import sys

path = sys.argv[1]
kind = sys.argv[2] if len(sys.argv) > 2 else "sift"
rows = []   # (start_ns, end_ns, name)
if path.endswith(".db"):
    db = sqlite3.connect(path)
    names = {r[0]: r[1] for r in db.execute("select id, coalesce(truncated_kernel_name, kernel_name) from kernel_symbols")}
    rows = [(s, e, names.get(k, str(k))) for k, s, e in db.execute("select kernel_id, start, end from rocpd_kernel_dispatch")]
else:
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
pre = "sift_" if kind == "sift" else "orb_"
two_nn = ("screen16", "subset_kernel", "settle_kernel")
launches, cur = [], []
for s, e, n in rows:
    if "prep_" in n:
        if cur:
            launches.append(cur)
        cur = []
    elif pre in n and any(t in n for t in two_nn):
        cur.append((s, e, n))
if cur:
    launches.append(cur)
launches = [l for l in launches if any("screen16" in n for _, _, n in l)]
spans, screens = [], []
for l in launches:
    scr = [(s, e) for s, e, n in l if "screen16" in n]
    t0 = min(s for s, _ in scr)
    t1 = max(e for _, e, _ in l)
    spans.append((t1 - t0) / 1e6)
    screens.append(sum(e - s for s, e in scr) / 1e6)
print(f"{len(launches)} launches of the {kind} 2-NN kernels")
for i, (sp, sc, l) in enumerate(zip(spans, screens, launches)):
    print(f"  launch {i:3d}: span {sp:8.3f} ms   screen dispatches {sum('screen16' in n for _, _, n in l):3d} "
          f"(sum {sc:8.3f} ms)   dispatches {len(l)}")
if spans:
    print(f"median span {statistics.median(spans):.3f} ms, median summed screen {statistics.median(screens):.3f} ms")
