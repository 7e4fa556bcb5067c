# GEMM iteration: kernel tests + sweep + microbench + full GPU suite + bench (via gpurun, repo root)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-gemm}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u tools/gemm_sweep.py > $O/sweep.json 2> $O/sweep.err && python -c "import json;d=json.load(open('$O/sweep.json'));[print(k,v['fixed_us_per_round'],v['steady_TFLOPs'],[p[2] for p in v['points']]) for k,v in d.items()]"
timeout -k 10 200 python -u tools/gemm_timeline.py > $O/tl.json 2>&1 && python -c "import json;d=json.load(open('$O/tl.json'));[print(k,v['event_us'],v['span_us'],v['item0']) for k,v in d.items()]"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && cat $O/bench.json
