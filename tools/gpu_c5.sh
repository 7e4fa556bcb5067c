# C5 (SDXL QLoRA) pass: SDXL GPU tests, then the C5 bench in each NF4 base mode (VPT_NF4_BASE)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sdxl_gpu.py tests/test_sdxl_flow_gpu.py -v --timeout 300 --timeout-method thread > $O/sdxl_tests.log 2>&1; rc=$?
[ $rc -le 1 ] && ! grep -q "Timeout (0:" $O/sdxl_tests.log || { echo "TESTS ABORTED rc=$rc"; tail -40 $O/sdxl_tests.log; exit 1; }
grep -E "^FAILED|passed|failed" $O/sdxl_tests.log | tail -12
for m in dequant resident inline; do
  VPT_NF4_BASE=$m timeout -k 10 400 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5_$m.json 2> $O/c5_$m.err || { echo "C5 $m FAILED"; tail -20 $O/c5_$m.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/c5_$m.json').read().strip().splitlines()[-1]); print('$m', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], json.dumps(d['kernels']))"
done
