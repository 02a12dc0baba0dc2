# Round artifacts: GPU tests, smoke, default bench (C3 full table), C5 lookups,
# rocprofv3 kernel-trace stats and FETCH/WRITE PMC passes.  Each GPU step has
# its own time limit; the chain stops at the first failure.
set -e
R=${ROUND:-r01}
O=gpurun_out/$R
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-profile > $O/pmc_fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-profile > $O/pmc_write.log 2>&1
python tools/pmc_to_json.py $O profiles/${R}_pmc_c3.json > /dev/null
timeout -k 10 300 python -u bench.py > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --no-cpu-baseline > $O/kt_bench.log 2>&1
timeout -k 10 200 python -u bench.py --config c5 --steps 10 --warmup 2 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/kt_c5 -o run --output-format csv -- python bench.py --config c5 --steps 4 --warmup 1 > $O/kt_c5.log 2>&1
echo done
