# same-box A/B of the C3 bench: a previous commit's build checked out in _old/ vs this tree
set -e
mkdir -p gpurun_out/ab
for k in 1 2; do
  (cd _old && timeout -k 10 200 python -u bench.py --no-cpu-baseline) > gpurun_out/ab/old_$k.log 2>&1
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/ab/new_$k.log 2>&1
  for v in old new; do python -c "import json;d=json.loads(open('gpurun_out/ab/${v}_$k.log').read().strip().splitlines()[-1]);print('$v', d['value'], d['roofline']['launch_avg_us'], d['kernel_ms']['relax'], d['kernel_ms']['rows'], d['kernel_ms']['init'])"; done
done
