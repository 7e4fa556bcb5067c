set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s2/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/s2/gpu_tests.log; exit 1; }
tail -5 gpurun_out/s2/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2/smoke.log 2>&1 && cat gpurun_out/s2/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/s2/bench.json 2> gpurun_out/s2/bench.err && cat gpurun_out/s2/bench.json
