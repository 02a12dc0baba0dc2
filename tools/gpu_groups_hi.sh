# groups per launch above the default cap: C3 bench steps and the C4 full table
set -e
mkdir -p gpurun_out/gh
for G in 48 64; do
  timeout -k 10 200 python -u bench.py --groups $G --no-cpu-baseline --no-profile > gpurun_out/gh/c3_$G.log 2>&1 || { tail gpurun_out/gh/c3_$G.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/gh/c3_$G.log').read().strip().splitlines()[-1]);print('C3 groups $G', d['value'], d['full_table_time_s'])"
done
for G in 64 96 128; do
  timeout -k 10 200 python -u bench.py --config c4 --full-table --groups $G > gpurun_out/gh/c4_$G.log 2>&1 || { tail gpurun_out/gh/c4_$G.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/gh/c4_$G.log').read().strip().splitlines()[-1]);print('C4 groups $G', d['value'])"
done
