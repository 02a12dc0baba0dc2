set -e
O=gpurun_out/fw1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fw_engine.py tests/test_gpu_fw.py tests/test_multi_device.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py --config c2fw > $O/bench_c2fw.log 2>&1 || { tail -20 $O/bench_c2fw.log; exit 1; }
tail -1 $O/bench_c2fw.log
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
tail -c 3000 $O/bench_default.log
