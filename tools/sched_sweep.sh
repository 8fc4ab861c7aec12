#!/bin/bash
# Headline time of the C3 unit under stream-schedule options (lookahead depth x reserved CUs).
set -e
mkdir -p gpurun_out/sched
for cfg in "2 16" "2 32" "2 64" "0 0" "2 0"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-fitc --no-cpu --lookahead $1 \
    --reserve-cus $2 > gpurun_out/sched/la$1_rc$2.json 2> gpurun_out/sched/la$1_rc$2.err
  python -c "import json; r=json.load(open('gpurun_out/sched/la$1_rc$2.json')); print('lookahead $1 reserve $2: %.2f ms/unit (accounting %.2f)' % (r['ms_per_step'], r['kernel_accounting']['ms_per_step']))"
done
