# Round 3 close-out: the full GPU suite, C4 / C5-on-C4 profiles, the default bench line.
set -e
mkdir -p gpurun_out/r03
TAG=r03_tests bash tools/gpu_tests.sh
CONFIGS="c4 c5_on_c4" bash tools/gpu_profiles.sh
timeout -k 10 600 python -u bench.py > gpurun_out/r03/bench_default.log 2>&1
