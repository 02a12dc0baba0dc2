# Round artifacts: GPU tests, smoke, default bench (C3 full table), C2 (LDS
# engine) and C5 lookups, rocprofv3 kernel-trace stats and FETCH/WRITE PMC
# passes.  Each GPU step has its own time limit; the chain stops at the first
# failure.  Copy what is judged into profiles/ afterwards (tools/collect_round.sh).
set -e
R=${ROUND:-r01}
O=gpurun_out/$R
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
for C in c3 c2 c5; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$C -o run --output-format csv -- python bench.py --config $C --steps 4 --warmup 1 --no-cpu-baseline --no-profile > $O/pmc_fetch_$C.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$C -o run --output-format csv -- python bench.py --config $C --steps 4 --warmup 1 --no-cpu-baseline --no-profile > $O/pmc_write_$C.log 2>&1
  mkdir -p $O/pmc_$C && cp -r $O/pmc_fetch_$C $O/pmc_write_$C $O/pmc_$C/
  python tools/pmc_to_json.py $O/pmc_$C profiles/${R}_pmc_$C.json > /dev/null
done
timeout -k 10 300 python -u bench.py > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt_c3 -o run --output-format csv -- python bench.py --no-cpu-baseline > $O/kt_c3.log 2>&1
timeout -k 10 300 python -u bench.py --config c2 > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt_c2 -o run --output-format csv -- python bench.py --config c2 --no-cpu-baseline > $O/kt_c2.log 2>&1
timeout -k 10 200 python -u bench.py --config c1 > $O/bench_c1.log 2>&1 || { tail -20 $O/bench_c1.log; exit 1; }
tail -1 $O/bench_c1.log
timeout -k 10 200 python -u bench.py --config c1all > $O/bench_c1all.log 2>&1 || { tail -20 $O/bench_c1all.log; exit 1; }
timeout -k 10 300 python -u bench.py --config c4 --full-table --shares 8 --share-index 0 > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log
timeout -k 10 300 python -u bench.py --config c4 --full-table > $O/bench_c4_full.log 2>&1 || { tail -20 $O/bench_c4_full.log; exit 1; }
tail -1 $O/bench_c4_full.log
timeout -k 10 200 python -u bench.py --config c4 --steps 20 --warmup 2 --no-cpu-baseline > $O/bench_c4_steps.log 2>&1 || { tail -20 $O/bench_c4_steps.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt_c4 -o run --output-format csv -- python bench.py --config c4 --steps 20 --warmup 2 --no-cpu-baseline > $O/kt_c4.log 2>&1
timeout -k 10 200 python -u bench.py --config c5 --steps 10 --warmup 2 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/kt_c5 -o run --output-format csv -- python bench.py --config c5 --steps 4 --warmup 1 > $O/kt_c5.log 2>&1
timeout -k 10 200 python -u bench.py --config c2fw > $O/bench_c2fw.log 2>&1 || { tail -20 $O/bench_c2fw.log; exit 1; }
tail -1 $O/bench_c2fw.log
timeout -k 10 300 python -u bench.py --config complete > $O/bench_complete.log 2>&1 || { tail -20 $O/bench_complete.log; exit 1; }
tail -1 $O/bench_complete.log
echo done
