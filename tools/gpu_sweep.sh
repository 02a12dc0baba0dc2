set -e
mkdir -p gpurun_out
for G in 1 2 4 8 16; do
  timeout -k 10 200 python -u bench.py --steps 6 --warmup 1 --groups $G --no-cpu-baseline > gpurun_out/sweep_g$G.log 2>&1
  python -c "import json;d=json.loads(open('gpurun_out/sweep_g$G.log').read().strip().splitlines()[-1]);print('G=$G', d['value'], d['kernel_ms'], d['roofline']['launch_avg_us'], d['relax_rounds_per_step'])"
done
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 0 --groups 16 --no-cpu-baseline --no-profile > gpurun_out/pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 2 --warmup 0 --groups 16 --no-cpu-baseline --no-profile > gpurun_out/pmc2.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --groups 16 --no-cpu-baseline --no-profile > gpurun_out/kt.log 2>&1
ls -R gpurun_out | head -40
