set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "attention or qknorm or reduce" > $O/k.log 2>&1 || { tail -40 $O/k.log; exit 1; }
tail -2 $O/k.log
for K in FIXREF_ATTN_FWD FUSED_QKNORM_FWD FUSED_QKNORM_BWD; do
  timeout -k 10 300 python -u tools/c3_knob_ab.py $K --rounds 6 --steps 5 > $O/ab_$K.log 2>&1 || { tail -20 $O/ab_$K.log; exit 1; }
  tail -1 $O/ab_$K.log
done
