set -e
mkdir -p gpurun_out/r03_lean
SPE_LANES=128 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r03_lean/pytest_parity.log 2>&1 || { tail -30 gpurun_out/r03_lean/pytest_parity.log; exit 1; }
tail -1 gpurun_out/r03_lean/pytest_parity.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_bench_configs.py -k "c3 or c4" > gpurun_out/r03_lean/pytest_configs.log 2>&1 || { tail -30 gpurun_out/r03_lean/pytest_configs.log; exit 1; }
tail -1 gpurun_out/r03_lean/pytest_configs.log
TAG=r03_lean VARIANTS="base:2:0:0 tree:2:0:0 tree:2:5:7 tree:2:4:8 tree:1:0:0" bash tools/gpu_relax_ab.sh
