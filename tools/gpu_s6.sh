# Attention kernel tests + parity + bench line: bash tools/gpu_s6.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-s6a}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py -x -v -k "attention or parity or golden or jit or c1 or c2 or c3 or bucket" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err && cat $O/bench.json
