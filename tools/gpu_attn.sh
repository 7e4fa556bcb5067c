# attention iteration: kernel tests + microbench + bench (run via gpurun from the repo root)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-attn}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/kernel_bench.py --attn-only --rounds 3 > $O/micro.json 2> $O/micro.err && cat $O/micro.json
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && cat $O/bench.json
