set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 400 python -u tools/c3_knob_ab.py BWD_UNIQUE_BUFFERS --rounds 6 --steps 5 > $O/uniq_ab.log 2>&1 || { tail -20 $O/uniq_ab.log; exit 1; }
tail -3 $O/uniq_ab.log
timeout -k 10 400 python -u tools/c3_knob_ab.py BWD_UNIQUE_BUFFERS --rounds 6 --steps 5 --workload c2 > $O/uniq_ab_c2.log 2>&1 || { tail -20 $O/uniq_ab_c2.log; exit 1; }
tail -3 $O/uniq_ab_c2.log
