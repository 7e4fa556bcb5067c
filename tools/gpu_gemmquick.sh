# Quick GEMM A/B: per-shape microbench + per-item timeline (diag lib).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-gq}
mkdir -p $O
timeout -k 10 300 python -u tools/gemm_shapes.py --rounds 2 > $O/gemm_shapes.json 2> $O/gemm_shapes.err || { tail -30 $O/gemm_shapes.err; exit 1; }
VPT_DIAG=1 timeout -k 10 120 python -u tools/gemm_timeline.py > $O/timeline.json 2> $O/timeline.err || { tail -20 $O/timeline.err; exit 1; }
echo done
