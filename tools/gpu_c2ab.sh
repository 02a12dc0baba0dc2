# LDS-engine parity, then same-box A/B of variant libraries on C2 (alternating)
set -e
O=gpurun_out/${TAG:-c2ab}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_lds.py tests/test_gpu_parity.py tests/test_gpu_source_tree.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for V in ${VARIANTS:-build_A build_B}; do
    LOG=$O/$(basename $V)_$r.log
    SPE_LIB=$PWD/$V/libspe.so timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --steps 5 > $LOG 2>&1 || { tail -5 $LOG; exit 1; }
    python -c "import json;d=json.loads([l for l in open('$LOG') if l.startswith('{')][-1]);print('$V run $r', d['value'], d['ms_per_step'], d['roofline']['launch_avg_us'])"
  done
done
