set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03zz2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "radam or ema or lerp" -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c2 --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/c2.json 2> $GRAFT_REPO_ROOT/$O/c2.err || { echo PROF FAILED; tail -20 $GRAFT_REPO_ROOT/$O/c2.err; exit 1; }
cut -c1-300 $GRAFT_REPO_ROOT/$O/c2.json
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | head
grep -h radam $(find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv") | cut -c1-300
