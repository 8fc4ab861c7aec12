# per-launch row-norm times, overlap off, map 5 vs the paired tiles (map 6): rocprofv3 traces
set -e
export TMPDIR=/tmp
for v in 5 6; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rowsq_prof_m$v -o run \
    -- python3 tools/ab_bench.py --config C4 --rounds 2 --steps 3 map=$v,ov=0 > gpurun_out/rowsq_prof_m$v.log 2>&1
  echo "map $v done"
done
