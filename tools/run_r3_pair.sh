#!/bin/bash
# round 3: phase-A tile updates of the leaf in pairs — leaf timing (HEAD leaf vs working leaf, same
# box), the factorisation tests, then a same-box C3 / C4 A/B against ab/libgpscore_base.so
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_pair
mkdir -p $O
for r in 1 2; do
  for v in cur pair; do
    timeout -k 5 60 ./tools/db_$v lib > $O/leaf_${v}_$r.txt 2>&1 || { echo "LEAF $v FAILED"; cat $O/leaf_${v}_$r.txt; exit 1; }
    echo "$v $r: $(grep -E 'us per|max' $O/leaf_${v}_$r.txt | head -3 | tr '\n' ' ')"
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "persistent or c3_config or leaf or potrf or large_properties or golden or fitc" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
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
