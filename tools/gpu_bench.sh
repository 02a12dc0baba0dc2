# bench lines of the current code: C3 default (whole table per step), C2, C4 full table, C5,
# plus the N=2 path rehearsed on one GPU (gloo; never for numbers)
set -e
O=gpurun_out/${TAG:-bench}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log
timeout -k 10 300 python -u bench.py --config c2 --cpu-seconds 6 > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline --steps 2 > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 2 --cpu-seconds 6 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log
SPE_BENCH_REHEARSE_ONE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/rehearse_n2.log 2>&1 || { tail -30 $O/rehearse_n2.log; exit 1; }
tail -1 $O/rehearse_n2.log
