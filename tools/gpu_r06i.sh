set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "patchify or noise or flow_loss or rmsnorm or area or gauss" -x -v --timeout 240 --timeout-method thread > $O/ktests.log 2>&1 || { tail -40 $O/ktests.log; exit 1; }
tail -2 $O/ktests.log
for rep in 1 2; do
  timeout -k 10 200 python -u tools/hbm_kernels.py > $O/hbm_base_$rep.log 2>&1 || { tail -20 $O/hbm_base_$rep.log; exit 1; }
  timeout -k 10 200 python -u tools/hbm_kernels.py --lib rms32 > $O/hbm_rms32_$rep.log 2>&1 || { tail -20 $O/hbm_rms32_$rep.log; exit 1; }
done
tail -3 $O/hbm_base_1.log $O/hbm_rms32_1.log $O/hbm_base_2.log $O/hbm_rms32_2.log
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -2 $O/parity.log
