#!/bin/bash
# lookahead factorisation A/B (variants in $VARIANTS) + one C3 trace with $TRACE_OPTS and its fill profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/ab_bench.py --config ${CFG:-C3} --rounds 3 $VARIANTS > gpurun_out/la_ab.txt 2>&1 || { cat gpurun_out/la_ab.txt; exit 1; }
cat gpurun_out/la_ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trlb -o run \
  -- python3 tools/trace_unit.py config=${CFG:-C3} $TRACE_OPTS > gpurun_out/trlb.log 2>&1 || exit 1
python3 tools/fill_profile.py gpurun_out/trlb/run_kernel_trace.csv gram_reg 2 > gpurun_out/fill_lb.txt 2>&1
cat gpurun_out/fill_lb.txt
echo ok
