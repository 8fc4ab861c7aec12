set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in 0 1; do
  O=gpurun_out/prof_sx$v
  mkdir -p $O
  GPS_SLAB_XCD=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/fitc_unit.py > $O/trace.log 2>&1
  GPS_SLAB_XCD=$v timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fitc_fetch -o run -- python3 tools/fitc_unit.py > $O/f.log 2>&1
  GPS_SLAB_XCD=$v timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/fitc_write -o run -- python3 tools/fitc_unit.py > $O/w.log 2>&1
  python3 tools/traffic.py $O fitc_ > $O/fitc_traffic_summary.txt
  echo "sx$v done"
done
