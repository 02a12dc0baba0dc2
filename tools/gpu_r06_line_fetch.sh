# Round 6: random 16-B reads vs 64-B / 128-B (tools/probe_line_fetch.hip): time, then
# FETCH_SIZE per kernel in its own --pmc pass.
set -e
O=gpurun_out/r06_line_fetch; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 build_ab/probe_line_fetch 128 > $O/time.json
cat $O/time.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc -o run --output-format csv -- build_ab/probe_line_fetch 128 > $O/pmc.log 2>&1
python - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r06_line_fetch/pmc/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if r["Counter_Name"] == "FETCH_SIZE":
        acc[r["Kernel_Name"][:40]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(f"{k:40s} dispatches {len(v)} FETCH_SIZE raw per dispatch {sum(v)/len(v)*1024/1e9:.3f} GB "
          f"({sum(v)/len(v)*1024/128e6:.1f} B per location)")
PY
