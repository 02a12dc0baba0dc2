# per-launch device times of one C3 whole-table build (SPE_TRACE: one "spe-trace kind ms" line per
# launch; kind 3 = the relaxation kernel, 2 = heavy, 4 = rows) and rocprofv3 kernel stats of the FW engine (C2)
set -e
O=gpurun_out/${TAG:-trace}
mkdir -p $O
export TMPDIR=/tmp
SPE_TRACE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-side > $O/c3_trace.log 2>&1 || { tail -20 $O/c3_trace.log; exit 1; }
grep -c spe-trace $O/c3_trace.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2fw -o c2fw -- python3 bench.py --config c2fw --steps 1 > $O/c2fw_prof.log 2>&1 || { tail -20 $O/c2fw_prof.log; exit 1; }
find $O/prof_c2fw -name "*kernel_stats.csv" | head -3
