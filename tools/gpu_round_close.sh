# Round close-out on one GPU: the full GPU suite, then the default bench line
# (C3 plus every other config's line under side_configs).
set -e
mkdir -p gpurun_out/${ROUND:-r04}
TAG=${ROUND:-r04}_tests bash tools/gpu_tests.sh
timeout -k 10 600 python -u bench.py > gpurun_out/${ROUND:-r04}/bench_default.log 2>&1
tail -c 300 gpurun_out/${ROUND:-r04}/bench_default.log
