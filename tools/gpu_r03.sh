# Round-3 GPU pass: bash tools/gpu_r03.sh TAG -> full GPU suite (parity stats), smoke, C3 bench, C5 bench, C2 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
rm -f $O/parity_stats.jsonl
VPT_PARITY_STATS=$O/parity_stats.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 ; rc=$?; [ $rc -le 1 ] && ! grep -q "Timeout (0:" $O/gpu_tests.log || { echo "TESTS ABORTED rc=$rc"; tail -60 $O/gpu_tests.log; exit 1; }; grep -E "^FAILED|passed|failed" $O/gpu_tests.log | tail -20
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -30 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -30 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
timeout -k 10 400 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "C5 FAILED"; tail -30 $O/bench_c5.err; exit 1; }
cut -c1-600 $O/bench_c5.json
timeout -k 10 300 python -u bench.py --workload c2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { echo "C2 FAILED"; tail -30 $O/bench_c2.err; exit 1; }
cut -c1-600 $O/bench_c2.json
