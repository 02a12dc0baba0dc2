# experiment: source-locality slot orders (bench.py SPE_BENCH_SLOT_ORDER) on C4 (one 1/8 share) and C3
set -e
mkdir -p gpurun_out
for O in none anchor rcm; do
  if [ $O = none ]; then unset SPE_BENCH_SLOT_ORDER; else export SPE_BENCH_SLOT_ORDER=$O; fi
  timeout -k 10 300 python -u bench.py --config c4 --full-table --shares 8 --share-index 0 > gpurun_out/so_c4_$O.log 2>&1 || { tail -20 gpurun_out/so_c4_$O.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/so_c4_$O.log').read().strip().splitlines()[-1]);print('c4 $O', d['value'], d['sources_per_s_per_gpu'])"
  timeout -k 10 300 python -u bench.py --config c3 --steps 8 --warmup 1 --no-cpu-baseline > gpurun_out/so_c3_$O.log 2>&1 || { tail -20 gpurun_out/so_c3_$O.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/so_c3_$O.log').read().strip().splitlines()[-1]);print('c3 $O', d['value'], d['kernel_ms']['relax'], d['relax_rounds_per_step'])"
done
