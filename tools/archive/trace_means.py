"""Per-workload mean kernel durations from a rocprofv3 kernel_trace.csv of the full bench:
tools/trace_means.py DIR > profiles/<round>_kernel_trace_means.json.  SIFT 2-NN launches are
split by workload: config 2 (50 images, grid 1225 pairs x 16 work items) and config 3 (200
images) have different grid sizes (pass 2's grid is an upper bound: 4 items per pass-1 item)."""
import collections, csv, glob, json, sys

f = glob.glob(sys.argv[1].rstrip("/") + "/*kernel_trace.csv")[0]
rows = list(csv.DictReader(open(f)))
groups = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"]
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    for key in ("sift_screen", "sift_knn2_kernel", "orb_screen", "orb_mfma", "homography_ransac_kernel", "chol_step",
                "ba_point_blocks_lds", "ba_pair_blocks", "undistort_kernel", "blur_tile_n_kernel"):
        if key in name:
            if key in ("sift_screen", "sift_knn2_kernel"):
                key += " (config 2 launches)" if grid <= 100000 * 256 else " (config 3 launches)"   # C2: 19600 screen / <= 78400 pass-2 items
            groups[key].append(dur)
out = {k: {"n": len(v), "mean_ms": sum(v) / len(v)} for k, v in groups.items()}
print(json.dumps(out, indent=1))
