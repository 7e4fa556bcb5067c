# rocprofv3 kernel stats of the C5 bench (3 timed steps + 2 warmup + 1 probe step)
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o p -- python $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 3 --warmup 2 --no-cpu-baseline > $O/ktrace.log 2>&1
tail -2 $O/ktrace.log
