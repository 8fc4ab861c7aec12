set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for L in ab/libgpscore_base.so scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd/gpscore/libgpscore.so; do
    GPSCORE_LIB=$PWD/$L timeout -k 10 300 python -u tools/ab_bench.py --config C2 --block es --rounds 1 --steps 3 map=0 2>&1 | sed "s|^|$(basename $L) |" || exit 1
  done
done
