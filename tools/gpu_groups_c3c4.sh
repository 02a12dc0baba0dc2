# groups-per-launch sweep on the current code: C3 bench steps and the C4 full table
set -e
mkdir -p gpurun_out/gs
for G in 16 24 32 48; do
  timeout -k 10 200 python -u bench.py --groups $G --no-cpu-baseline --no-profile > gpurun_out/gs/c3_$G.log 2>&1 || { tail gpurun_out/gs/c3_$G.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/gs/c3_$G.log').read().strip().splitlines()[-1]);print('C3 groups $G', d['value'], d['full_table_time_s'])"
done
for G in 40 60 64; do
  timeout -k 10 200 python -u bench.py --config c4 --full-table --groups $G > gpurun_out/gs/c4_$G.log 2>&1 || { tail gpurun_out/gs/c4_$G.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/gs/c4_$G.log').read().strip().splitlines()[-1]);print('C4 groups $G', d['value'])"
done
