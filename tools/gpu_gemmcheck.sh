# GEMM change check: GEMM + SwiGLU kernel tests, per-shape microbench, timeline, bench with breakdown.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-gemmcheck}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or swiglu or linear" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/gemm_shapes.py --rounds 3 > $O/gemm_shapes.json 2> $O/gemm_shapes.err || { tail -30 $O/gemm_shapes.err; exit 1; }
VPT_DIAG=1 timeout -k 10 120 python -u tools/gemm_timeline.py > $O/timeline.json 2> $O/timeline.err || { tail -20 $O/timeline.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --breakdown $O/breakdown.json > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
echo done
