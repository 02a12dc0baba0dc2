# The C3 bench line and its rocprofv3 kernel stats from ONE process (the line's
# HIP-event launch averages and rocprof's must agree)
set -e
O=gpurun_out/${ROUND:-r04}; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $O/same_c3 -o run --output-format csv -- python bench.py --config c3 --steps 3 --warmup 1 --no-side --cpu-seconds 2 > $O/same_c3.log 2>&1
tail -c 300 $O/same_c3.log
