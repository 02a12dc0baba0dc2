# Round 3: full-size parity incl. the whole-table checks, the multi-device split on
# one GPU, and a rehearsal of the N > 1 bench schedule on one GPU (two gloo ranks
# on device 0: never for numbers).
set -e
O=gpurun_out/r03_dist; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_bench_configs.py tests/test_multi_device.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "table_check" > $O/pytest_check.log 2>&1 || { tail -40 $O/pytest_check.log; exit 1; }
tail -2 $O/pytest_check.log
export SPE_BENCH_REHEARSE_ONE_GPU=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --no-north-star > $O/rehearse_c3_n2.log 2>&1 || { tail -40 $O/rehearse_c3_n2.log; exit 1; }
tail -1 $O/rehearse_c3_n2.log | cut -c1-1500
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config c5 --steps 3 --warmup 1 > $O/rehearse_c5_n2.log 2>&1 || { tail -40 $O/rehearse_c5_n2.log; exit 1; }
tail -1 $O/rehearse_c5_n2.log | cut -c1-800
