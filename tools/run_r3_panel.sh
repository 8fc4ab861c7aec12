#!/bin/bash
# round 3: DPP-broadcast pivot panel in the leaf — leaf timing (HEAD leaf vs working leaf, same
# box), the persistent-factorisation tests, then a same-box C3 / C4 A/B against ab/libgpscore_base.so
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_panel
mkdir -p $O
for r in 1 2; do
  timeout -k 5 60 ./tools/db_base lib > $O/leaf_base_$r.txt 2>&1 || { echo "LEAF BASE FAILED"; cat $O/leaf_base_$r.txt; exit 1; }
  timeout -k 5 60 ./tools/db_cur lib > $O/leaf_cur_$r.txt 2>&1 || { echo "LEAF CUR FAILED"; cat $O/leaf_cur_$r.txt; exit 1; }
done
grep -H "us per\|max|dL|\|NaN" $O/leaf_*.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "persistent or c3_config or leaf or potrf or large_properties or golden" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in base cur; do
    if [ $v = base ]; then export GPSCORE_LIB=$PWD/ab/libgpscore_base.so; else unset GPSCORE_LIB; fi
    timeout -k 10 200 python -u tools/ab_bench.py --config C3 --rounds 1 --steps 4 map=0 > $O/c3_${v}_$r.txt 2>&1 || { echo "AB FAILED"; tail $O/c3_${v}_$r.txt; exit 1; }
    timeout -k 10 200 python -u tools/ab_bench.py --config C4 --rounds 2 --steps 5 map=0 > $O/c4_${v}_$r.txt 2>&1 || { echo "AB FAILED"; tail $O/c4_${v}_$r.txt; exit 1; }
    echo "$v $r: C3 $(grep -o 'median *[0-9.]*' $O/c3_${v}_$r.txt)  C4 $(grep -o 'median *[0-9.]*' $O/c4_${v}_$r.txt)"
  done
done
true
