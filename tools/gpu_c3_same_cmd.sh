# the C3 bench line and its rocprofv3 kernel stats from ONE process (same command),
# so the HIP-event launch average and rocprof's agree by construction
set -e
R=${ROUND:-r02}
O=gpurun_out/${R}_c3same; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python -u bench.py --no-side > $O/bench.log 2>&1
tail -1 $O/bench.log | cut -c1-400
