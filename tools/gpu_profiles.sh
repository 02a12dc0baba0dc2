# Round profiles: rocprofv3 kernel-trace stats of the bench lines and separate
# FETCH_SIZE / WRITE_SIZE PMC passes (MI355X_MICROARCH.md HBM section), then
# the bench lines themselves (which read the PMC summaries back).
set -e
R=${ROUND:-r02}
O=gpurun_out/$R
mkdir -p $O
export TMPDIR=/tmp
for C in c3 c2 c4 c5; do
  A="--config $C --steps 1 --warmup 1 --no-cpu-baseline --no-profile"
  [ $C = c5 ] && A="--config c5 --steps 4 --warmup 1 --no-cpu-baseline"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$C -o run --output-format csv -- python bench.py $A > $O/pmc_fetch_$C.log 2>&1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$C -o run --output-format csv -- python bench.py $A > $O/pmc_write_$C.log 2>&1
  mkdir -p $O/pmc_$C && cp -r $O/pmc_fetch_$C $O/pmc_write_$C $O/pmc_$C/
  python tools/pmc_to_json.py $O/pmc_$C profiles/${R}_pmc_$C.json > /dev/null
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/kt_$C -o run --output-format csv -- python bench.py $A > $O/kt_$C.log 2>&1
done
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/kt_c2fw -o run --output-format csv -- python bench.py --config c2fw --steps 1 > $O/kt_c2fw.log 2>&1
timeout -k 10 300 python -u bench.py --config c2fw > $O/bench_c2fw.log 2>&1 || { tail -20 $O/bench_c2fw.log; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log
timeout -k 10 300 python -u bench.py --config c2 > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 1; }
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline --steps 2 > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 1; }
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 2 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
timeout -k 10 300 python -u bench.py --config c1 > $O/bench_c1.log 2>&1 || { tail -20 $O/bench_c1.log; exit 1; }
echo done
