set -e
export TMPDIR=/tmp
timeout -k 10 200 tbin/gemm_bench rowsq_iso > gpurun_out/rowsq_iso_r5h.txt 2>&1
echo iso done
timeout -k 10 120 tbin/gram_bench d16 > gpurun_out/gram_d16_r5h.txt 2>&1
echo gram done
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "slab_xcd" -m gpu > gpurun_out/map6_test_r5h.log 2>&1
echo test done
timeout -k 10 400 python -u tools/ab_bench.py --config C4 --rounds 5 map=0 map=6 prio=2 map=6,prio=2 > gpurun_out/map6_ab_c4_r5h.txt 2>&1
echo c4 done
timeout -k 10 400 python -u tools/ab_bench.py --config C5 --rounds 3 --steps 2 map=0 map=6 map=6,prio=2 > gpurun_out/map6_ab_c5_r5h.txt 2>&1
echo c5 done
