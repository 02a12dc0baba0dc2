"""One line per A/B run: the bench's table time, and (first pass) the rocprof
kernel stats of the same command as ms per table (STEPS + warm-up tables)."""
import csv
import glob
import json
import os
import sys

o, v, rep, tables = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
line = json.loads([x for x in open(os.path.join(o, f"b_{v}_{rep}.log")) if x.startswith("{")][-1])
msg = f"{v} rep={rep} table_s={line['full_table_time_s']} lanes={line['roofline']['relaxed_lanes_per_step']} " \
      f"derived={line['roofline']['derived_sources_per_step']} frac={line['roofline']['frac']}"
stats = glob.glob(os.path.join(o, f"kt_{v}", "**", "*kernel_stats.csv"), recursive=True)
if rep == "1" and stats:
    rows = list(csv.DictReader(open(stats[0])))
    ks = []
    for r in rows:
        name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
        name = name[5:] if name.startswith("void ") else name
        ks.append((float(r["TotalDurationNs"]) / 1e6 / tables, int(r["Calls"]), name))
    ks.sort(reverse=True)
    msg += " | " + "; ".join(f"{n.split('<')[0]} {ms:.1f}ms/{c}" for ms, c, n in ks[:8])
print(msg, flush=True)
