# GPU parity of the in-tree build (the whole parity set incl. full-size bench configs), then
# same-box A/B of variant libraries (dirs in $VARIANTS) on C3 / C4
set -e
O=gpurun_out/${TAG:-abc}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pendants.py tests/test_gpu_bench_configs.py tests/test_gpu_delta.py tests/test_gpu_lds.py tests/test_gpu_source_tree.py tests/test_gpu_owner.py tests/test_gpu_complete.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for V in ${VARIANTS:-build_A build_B}; do
    for C in c3 c4; do
      LOG=$O/${V}_${C}_$r.log
      SPE_LIB=$PWD/$V/libspe.so timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-side --steps 2 > $LOG 2>&1 || { tail -5 $LOG; exit 1; }
      python -c "import json;d=json.loads([l for l in open('$LOG') if l.startswith('{')][-1]);print('$V $C run $r', d['value'], d['full_table_time_s'], d['kernel_ms']['relax'], d['relax_rounds_per_step'])"
    done
  done
done
