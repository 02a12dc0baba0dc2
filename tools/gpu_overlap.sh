# parity tests with the rows/relax overlap, then C3 / C4 with and without it (SPE_NO_OVERLAP)
set -e
mkdir -p gpurun_out/ovl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ovl/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/ovl/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/ovl/pytest_gpu.log
for V in 0 1; do
  if [ $V = 1 ]; then export SPE_NO_OVERLAP=1; fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/ovl/c3_$V.log 2>&1 || { tail gpurun_out/ovl/c3_$V.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ovl/c3_$V.log').read().strip().splitlines()[-1]);print('NO_OVERLAP=$V C3', d['value'], d['full_table_time_s'], d['kernel_ms'])"
  timeout -k 10 200 python -u bench.py --config c4 --full-table > gpurun_out/ovl/c4_$V.log 2>&1 || { tail gpurun_out/ovl/c4_$V.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ovl/c4_$V.log').read().strip().splitlines()[-1]);print('NO_OVERLAP=$V C4 full', d['value'], d['roofline']['frac'])"
done
