# GEMM/SwiGLU kernel tests + parity + GEMM shape timings + bench line: bash tools/gpu_s5.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-s5a}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
VPT_DIAG=1 timeout -k 10 300 python -u tools/gemm_stagger.py --rounds 3 > $O/gemm.json 2> $O/gemm.err || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --breakdown $O/breakdown.json > $O/bench.json 2> $O/bench.err && cat $O/bench.json
