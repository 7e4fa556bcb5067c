# full GPU suite with parity stats, then c3 / c5 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
rm -f $O/parity_stats.jsonl
VPT_PARITY_STATS=$O/parity_stats.jsonl timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -30 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
timeout -k 10 400 python -u bench.py --workload c5 --steps 5 --warmup 2 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "C5 FAILED"; tail -30 $O/bench_c5.err; exit 1; }
cut -c1-600 $O/bench_c5.json
