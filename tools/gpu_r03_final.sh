# Round 3 close-out: shared-tree parity with the shipped tile shape, the tile A/B,
# then the full GPU suite, C4 / C5-on-C4 profiles and the default bench line.
set -e
O=gpurun_out/r03_final; mkdir -p $O gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shared_trees.py tests/test_gpu_bench_configs.py -k "shared or c4" > $O/pytest_share.log 2>&1 || { tail -40 $O/pytest_share.log; exit 1; }
tail -1 $O/pytest_share.log
bash tools/gpu_share_rows_ab.sh
