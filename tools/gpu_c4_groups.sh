# C4 one-eighth share: groups per launch sweep (the auto value caps at 16)
set -e
mkdir -p gpurun_out
for G in ${GROUPS_LIST:-16 24 32 48}; do
  timeout -k 10 300 python -u bench.py --config c4 --full-table --shares 8 --share-index 0 --groups $G > gpurun_out/c4g_$G.log 2>&1 || { tail -20 gpurun_out/c4g_$G.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/c4g_$G.log').read().strip().splitlines()[-1]);print('G=$G', d['value'], d['sources_per_s_per_gpu'])"
done
