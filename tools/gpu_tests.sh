# full GPU test suite (one pytest process), log under gpurun_out/$O
set -e
O=gpurun_out/${TAG:-tests}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -5 $O/pytest_gpu.log
