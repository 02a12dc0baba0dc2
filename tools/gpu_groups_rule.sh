# groups per launch vs relaxation-graph size: C4 share (20k core) and C3 (50k)
set -e
mkdir -p gpurun_out
for G in 64 96; do
  timeout -k 10 300 python -u bench.py --config c4 --full-table --shares 8 --share-index 0 --groups $G > gpurun_out/c4g_$G.log 2>&1 || { tail -20 gpurun_out/c4g_$G.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/c4g_$G.log').read().strip().splitlines()[-1]);print('c4 G=$G', d['value'], d['sources_per_s_per_gpu'])"
done
for G in 16 20 24; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 1 --groups $G --blocks-per-step 48 --no-cpu-baseline > gpurun_out/c3g_$G.log 2>&1 || { tail -20 gpurun_out/c3g_$G.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/c3g_$G.log').read().strip().splitlines()[-1]);print('c3 G=$G', d['value'], d['kernel_ms']['relax'])"
done
