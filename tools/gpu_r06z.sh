set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06z}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sdxl_gpu.py tests/test_sdxl_flow_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --workload c5 --steps 8 --warmup 2 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o p -- python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
python tools/ktrace_summary.py $O/kt > $O/ktrace_summary.txt 2>&1; head -14 $O/ktrace_summary.txt
