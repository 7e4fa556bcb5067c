# Round-3 GPU pass: bash tools/gpu_r03.sh TAG  -> full GPU suite, smoke, bench (each under its own limit)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -30 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
