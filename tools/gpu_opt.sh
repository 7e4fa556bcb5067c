# Quick A/B pass for memory-bound kernel changes: their GPU tests, then a C3 and a C2 bench (hbm_kernels report).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-opt}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "${2:-radam or rmsnorm}" -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { echo C3 FAILED; tail -20 $O/c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c2 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || { echo C2 FAILED; tail -20 $O/c2.err; exit 1; }
python -c "
import json,sys
for f in ['c3','c2']:
    d=json.loads(open('$O/'+f+'.json').read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step']); print(json.dumps(d['hbm_kernels']))
"
