# parity of the working-tree library on the batch-engine tests, then same-box A/B (tools/gpu_varab.sh)
set -e
O=gpurun_out/${TAG:-segab}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pendants.py tests/test_gpu_bench_configs.py tests/test_gpu_delta.py tests/test_gpu_source_tree.py tests/test_gpu_owner.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TAG=${TAG:-segab} bash tools/gpu_varab.sh
