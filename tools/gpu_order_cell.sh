# spe_order_sources: sources per Voronoi cell (SPE_ORDER_CELL) on C3 and one C4 share
set -e
mkdir -p gpurun_out
for K in ${CELLS:-16 32 64 128 512}; do
  SPE_ORDER_CELL=$K timeout -k 10 300 python -u bench.py --steps 16 --warmup 1 --no-cpu-baseline > gpurun_out/oc_c3.log 2>&1 || { tail -20 gpurun_out/oc_c3.log; exit 1; }
  SPE_ORDER_CELL=$K timeout -k 10 300 python -u bench.py --config c4 --full-table --shares 8 --share-index 0 > gpurun_out/oc_c4.log 2>&1 || { tail -20 gpurun_out/oc_c4.log; exit 1; }
  python -c "import json;a=json.loads(open('gpurun_out/oc_c3.log').read().strip().splitlines()[-1]);b=json.loads(open('gpurun_out/oc_c4.log').read().strip().splitlines()[-1]);print('cell=$K c3', a['value'], a['kernel_ms']['relax'], 'c4share', b['sources_per_s_per_gpu'])"
done
