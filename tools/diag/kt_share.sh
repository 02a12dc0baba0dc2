set -e
export TMPDIR=/tmp
O=gpurun_out/kt_share; mkdir -p $O
for V in 0 1; do
SPE_EXACT_SOURCES=$V timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt_$V -o run --output-format csv -- python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-side > $O/kt_$V.log 2>&1
f=$(find $O/kt_$V -name "run_kernel_stats.csv" | head -1)
python -c "
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:9]: print(sys.argv[2], r['Name'][:70], r['Calls'], r['AverageNs'], r['TotalDurationNs'])" $f exact=$V
done
