# Same-box A/B of the default lane width (64) against SPE_LANES=$L on C3 / C4, alternating,
# then the whole GPU suite under SPE_LANES=$L
set -e
O=gpurun_out/${TAG:-lanes_ab}; mkdir -p $O
L=${L:-128}
for r in 1 2 3; do
  for X in 64 $L; do
    for C in c3 c4; do
      SPE_LANES=$X timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --steps 2 > $O/${C}_L${X}_$r.log 2>&1 || { tail -5 $O/${C}_L${X}_$r.log; exit 1; }
      python -c "import json;d=json.loads(open('$O/${C}_L${X}_$r.log').read().strip().splitlines()[-1]);print('$C L=$X run $r', d['value'], d['ms_per_step'])"
    done
  done
done
SPE_LANES=$L timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_L$L.log 2>&1 || { tail -30 $O/pytest_L$L.log; exit 1; }
tail -2 $O/pytest_L$L.log
