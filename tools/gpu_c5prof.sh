# C5 kernel-time breakdown: rocprofv3 kernel stats of a short c5 bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-c5prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o p -- python3 $R/bench.py --workload c5 --steps 3 --warmup 1 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
cat $O/c5.json
find $O/kt -name "*kernel_stats.csv" | head -3
