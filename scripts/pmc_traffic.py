"""Write profiles/pmc_traffic.json from a `STEPS=pmc` run (gpurun_out/pmc*/): FETCH_SIZE and
WRITE_SIZE (KiB, separate passes) of the path kernel, averaged over its dispatches.
Caveats (MI355X_MICROARCH.md "HBM"): both count L2<->fabric traffic, so Infinity-Cache hits are
included (the 30.7 MB RNG table lives there); FETCH_SIZE is calibrated only for 16-B/lane streams
(the path kernel gathers dwords), so the figure is an upper-level traffic estimate."""
import csv, glob, json, os, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_traffic.json"
vals = {}
for f in glob.glob(os.path.join(root, "pmc*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "path_kernel" in r["Kernel_Name"] and r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"]) * 1024
write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"]) * 1024
rec = {"scene": "cornell", "width": 1921, "height": 1081, "passes_per_launch": 16.0,
       "fetch_bytes_per_launch": int(fetch), "write_bytes_per_launch": int(write),
       "hbm_bytes_per_launch": int(fetch + write), "dispatches": len(vals["FETCH_SIZE"]),
       "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), x1024",
       "caveat": __doc__.split("Caveats", 1)[1].strip()}
os.makedirs(os.path.dirname(out), exist_ok=True)
json.dump(rec, open(out, "w"), indent=1)
print(json.dumps(rec))
