set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "queue_bitwise" -x -v --timeout 240 --timeout-method thread > $O/qtest.log 2>&1 || { tail -40 $O/qtest.log; exit 1; }
tail -2 $O/qtest.log
timeout -k 10 300 python -u tools/attn_queue_ab.py > $O/attn_q_ab.log 2>&1 || { tail -20 $O/attn_q_ab.log; exit 1; }
tail -1 $O/attn_q_ab.log
timeout -k 10 600 python -u tools/lib_ab.py --variants base,swbplain,resid2,swf16,epi16 --what step --rounds 6 --steps 5 > $O/step_ab.log 2>&1 || { tail -20 $O/step_ab.log; exit 1; }
tail -2 $O/step_ab.log
