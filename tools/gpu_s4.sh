# Full GPU suite + bench line with per-shape GEMM breakdown: bash tools/gpu_s4.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-s4a}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --breakdown $O/breakdown.json > $O/bench.json 2> $O/bench.err && cat $O/bench.json
