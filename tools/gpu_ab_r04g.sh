set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04g
mkdir -p $O
VPT_DIAG=1 timeout -k 10 200 python -u tools/attn_stage_check.py > $O/stage_check.log 2>&1 || { tail -20 $O/stage_check.log; exit 1; }
tail -1 $O/stage_check.log
VPT_DIAG=1 timeout -k 10 300 python -u tools/c3_knob_ab.py ATTN_BWD_STAGES3 --rounds 6 --steps 5 > $O/ab_stages.log 2>&1 || { tail -20 $O/ab_stages.log; exit 1; }
tail -1 $O/ab_stages.log
