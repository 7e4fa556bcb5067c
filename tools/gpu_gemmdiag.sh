# GEMM diagnostics (diag library): square sizes vs hipBLASLt, per-item timeline, K-step stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-gemmdiag}
mkdir -p $O
export VPT_DIAG=1
timeout -k 10 240 python -u tools/gemm_square.py --rounds 2 --geos 256,128 > $O/square.json 2> $O/square.err || { tail -20 $O/square.err; exit 1; }
timeout -k 10 120 python -u tools/gemm_timeline.py > $O/timeline.json 2> $O/timeline.err || { tail -20 $O/timeline.err; exit 1; }
timeout -k 10 120 python -u tools/gemm_stamp.py > $O/stamp.json 2> $O/stamp.err || { tail -20 $O/stamp.err; exit 1; }
echo done
