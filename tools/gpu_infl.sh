# neighbour rows in flight per subgroup (SPE_INFL 4 / 6 / 8) on the current code: C3 steps, C4 full table
set -e
mkdir -p gpurun_out/infl
for I in 8 6 4; do
  SPE_INFL=$I timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-profile > gpurun_out/infl/c3_$I.log 2>&1 || { tail gpurun_out/infl/c3_$I.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/infl/c3_$I.log').read().strip().splitlines()[-1]);print('C3 INFL $I', d['value'])"
  SPE_INFL=$I timeout -k 10 200 python -u bench.py --config c4 --full-table > gpurun_out/infl/c4_$I.log 2>&1 || { tail gpurun_out/infl/c4_$I.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/infl/c4_$I.log').read().strip().splitlines()[-1]);print('C4 INFL $I', d['value'])"
done
