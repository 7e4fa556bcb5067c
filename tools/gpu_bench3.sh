# bench variants: overlap on (default), off, and C2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-overlap > $O/bench_nooverlap.json 2> $O/bench2.err || { echo "BENCH2 FAILED"; tail -30 $O/bench2.err; exit 1; }
cat $O/bench_nooverlap.json
timeout -k 10 400 python -u bench.py --workload c2 > $O/bench_c2.json 2> $O/bench3.err || { echo "BENCH3 FAILED"; tail -30 $O/bench3.err; exit 1; }
cat $O/bench_c2.json
