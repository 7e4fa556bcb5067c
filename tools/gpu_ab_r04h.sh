set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "swiglu" > $O/swiglu_tests.log 2>&1 || { tail -20 $O/swiglu_tests.log; exit 1; }
tail -1 $O/swiglu_tests.log
VPT_DIAG=1 timeout -k 10 300 python -u tools/c3_knob_ab.py SWB_AHEAD --rounds 6 --steps 5 > $O/ab_swb.log 2>&1 || { tail -20 $O/ab_swb.log; exit 1; }
tail -3 $O/ab_swb.log
