set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_sdxl_gpu.py tests/test_sdxl_flow_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/c5_knob_ab.py ops.GEMM_R2_128 --rounds 6 --steps 4 > $O/c5_ab.log 2>&1 || { tail -20 $O/c5_ab.log; exit 1; }
tail -1 $O/c5_ab.log
timeout -k 10 400 python -u tools/c3_knob_ab.py ops.GEMM_R2_128 --rounds 6 --steps 5 > $O/c3_ab.log 2>&1 || { tail -20 $O/c3_ab.log; exit 1; }
tail -1 $O/c3_ab.log
