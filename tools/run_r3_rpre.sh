#!/bin/bash
# round 3: r pass column tiles during B factorisation — FITC tests, then a same-box C4 / C5 A/B
# against the previous library (ab/libgpscore_base.so, tools/build_ref_lib.sh), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_rpre
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_fitc_grad.py -x -q --timeout 200 --timeout-method thread \
  -k "fitc or shard or c5" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for v in base cur; do
    if [ $v = base ]; then export GPSCORE_LIB=$PWD/ab/libgpscore_base.so; else unset GPSCORE_LIB; fi
    timeout -k 10 200 python -u tools/ab_bench.py --config C4 --rounds 2 --steps 5 map=0 > $O/c4_${v}_$r.txt 2>&1 || { echo "AB FAILED"; tail $O/c4_${v}_$r.txt; exit 1; }
    echo "C4 $v $r: $(grep median $O/c4_${v}_$r.txt)"
    timeout -k 10 200 python -u tools/ab_bench.py --config C5 --rounds 1 --steps 3 map=0 > $O/c5_${v}_$r.txt 2>&1 || { echo "AB FAILED"; tail $O/c5_${v}_$r.txt; exit 1; }
    echo "C5 $v $r: $(grep median $O/c5_${v}_$r.txt)"
  done
done
true
