# kernel traces of C3 units under side-stream options: is the persistent factorisation starved by
# the side stream's T product (its WGs need whole CUs)?  ab_bench with a single variant per run.
set -e
export TMPDIR=/tmp
for v in "sprio=0,graph=1" "sprio=1,graph=1" "sprio=1,graph=0"; do
  t=$(echo $v | tr ',=' '__')
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dagtr_$t -o run \
    -- python3 tools/ab_bench.py --config C3 --rounds 1 --steps 2 $v > gpurun_out/dagtr_$t.log 2>&1
  echo "$v done"
done
