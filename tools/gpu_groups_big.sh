# C3 whole-table time vs 64-source blocks per build launch (beyond the auto rule), same box
set -e
O=gpurun_out/${TAG:-gbig}; mkdir -p $O
for G in ${GROUPS_LIST:-46 92 196 392 46}; do
  timeout -k 10 300 python -u bench.py --config ${CONFIG:-c3} --groups $G --no-cpu-baseline --steps 2 > $O/g$G.log 2>&1 || { tail -5 $O/g$G.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/g$G.log').read().strip().splitlines()[-1]);print('groups $G', d['value'], d['ms_per_step'], d['roofline']['launch_avg_us'], d['relax_rounds_per_step'], d['roofline']['lanes_per_group'])"
done
