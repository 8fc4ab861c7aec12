#!/bin/bash
# round 3: persistent-launch width (leaves CUs to the FITC test pre-pass / the T products)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_surface.py -x -v --timeout 200 --timeout-method thread -k "any_grid or persistent_factorisation_matches or surface or c3_config or large_prop" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/ab_bench.py --config C4 --rounds 3 dagwg=0 dagwg=192 dagwg=128 dagwg=96 > $O/ab_c4.txt 2>&1 || { echo "AB C4 FAILED"; tail -20 $O/ab_c4.txt; exit 1; }
cat $O/ab_c4.txt
timeout -k 10 500 python -u tools/ab_bench.py --config C3 --rounds 3 dagwg=0 dagwg=192 dagwg=128 forkmax=77 ov=0 > $O/ab_c3.txt 2>&1 || { echo "AB C3 FAILED"; tail -20 $O/ab_c3.txt; exit 1; }
cat $O/ab_c3.txt
