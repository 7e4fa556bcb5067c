set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 300 python -u tools/c5_host_probe.py --steps 10 > $O/c5_host.log 2>&1 || { tail -20 $O/c5_host.log; exit 1; }
tail -1 $O/c5_host.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o p -- python bench.py --workload c5 --steps 6 --warmup 2 --no-cpu-baseline > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
python tools/ktrace_timeline.py $O/kt > $O/timeline.txt 2>&1 && head -30 $O/timeline.txt
