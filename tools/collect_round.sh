# copy the judged artefacts of a tools/gpu_round.sh run into profiles/
set -e
R=${ROUND:-r01}
O=gpurun_out/$R
for C in c1 c1all c3 c2 c2fw c4 c4_full c4_steps c5 complete; do
  [ -f $O/bench_$C.log ] && cp $O/bench_$C.log profiles/${R}_bench_$C.log
  if [ -d $O/kt_$C ]; then
    f=$(find $O/kt_$C -name '*kernel_stats.csv' | head -1)
    if [ -n "$f" ]; then cp "$f" profiles/${R}_rocprof_kernel_stats_$C.csv; fi
  fi
done
[ -f gpurun_out/pmc/summary.txt ] && cp gpurun_out/pmc/summary.txt profiles/${R}_pmc_counters_c3.txt
cp $O/pytest_gpu.log profiles/${R}_pytest_gpu.log
cp $O/smoke.log profiles/${R}_smoke.log
for C in c3 c2 c5; do python tools/pmc_to_json.py $O/pmc_$C profiles/${R}_pmc_$C.json > /dev/null; done
ls -la profiles
