set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "queue_bitwise" -x -v --timeout 240 --timeout-method thread > $O/qtest.log 2>&1 || { tail -40 $O/qtest.log; exit 1; }
tail -3 $O/qtest.log
timeout -k 10 300 python -u tools/attn_queue_ab.py > $O/attn_q_ab.log 2>&1 || { tail -20 $O/attn_q_ab.log; exit 1; }
tail -1 $O/attn_q_ab.log
timeout -k 10 300 python -u tools/lib_ab.py --variants base,swbld2,swbst16,swbboth --what swb --rounds 6 --iters 10 > $O/swb_ab.log 2>&1 || { tail -20 $O/swb_ab.log; exit 1; }
tail -1 $O/swb_ab.log
timeout -k 10 400 python -u tools/c3_knob_ab.py ATTN_BWD_QUEUE --rounds 6 --steps 5 > $O/c3_queue_ab.log 2>&1 || { tail -20 $O/c3_queue_ab.log; exit 1; }
tail -1 $O/c3_queue_ab.log
