"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-kernel, per-dispatch
HBM bytes (profiles/<round>_pmc_<config>.json), applying the gfx950 correction
of MI355X_MICROARCH.md §HBM: FETCH_SIZE reads exactly half of the bytes of
dwordx2/x4 loads -- confirmed here on k_rows_sssp, whose read volume is known
(24 B x 64 lanes x targets x groups per launch: FETCH_SIZE reports 0.50 of it).
WRITE_SIZE is exact (k_rows_sssp writes 22 B per pair: WRITE_SIZE = 1.00x)."""
import collections
import csv
import glob
import json
import os
import sys

root, out = sys.argv[1], sys.argv[2]
# optional: the bench log of the PMC pass -- its JSON line's pmc_key (config, N,
# groups per launch, build mode) is recorded, and bench.py attaches the summary
# as roofline.traffic only to a run with the same key
key = None
if len(sys.argv) > 3:
    for line in open(sys.argv[3]):
        if line.startswith("{"):
            try:
                key = json.loads(line).get("pmc_key", key)
            except ValueError:
                pass
acc = collections.defaultdict(lambda: {"fetch_kb": 0.0, "write_kb": 0.0, "dispatches": set()})
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        # "void (anonymous namespace)::k_relax<64, 8, 1>(...)" -> "k_relax"
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
        k = k[5:] if k.startswith("void ") else k
        if r["Counter_Name"] == "FETCH_SIZE":
            acc[k]["fetch_kb"] += float(r["Counter_Value"])
            acc[k]["dispatches"].add((f, r["Dispatch_Id"]))
        elif r["Counter_Name"] == "WRITE_SIZE":
            acc[k]["write_kb"] += float(r["Counter_Value"])
res = {}
for k, v in acc.items():
    nd = max(1, len(v["dispatches"]))
    res[k] = {"dispatches": nd, "fetch_bytes_raw_per_dispatch": v["fetch_kb"] * 1024 / nd,
              "fetch_bytes_per_dispatch": 2 * v["fetch_kb"] * 1024 / nd,
              "write_bytes_per_dispatch": v["write_kb"] * 1024 / nd}
    res[k]["hbm_bytes_per_dispatch"] = res[k]["fetch_bytes_per_dispatch"] + res[k]["write_bytes_per_dispatch"]
json.dump({"note": "FETCH_SIZE x2 (gfx950 correction, calibrated on k_rows_sssp); WRITE_SIZE x1",
           "pmc_key": key, "kernels": res}, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
