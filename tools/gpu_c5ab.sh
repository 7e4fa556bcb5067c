# SDXL GPU tests + same-box C5 bench A/B of one env knob: bash tools/gpu_c5ab.sh TAG VAR  (runs VAR=1,0,1,0)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
V=$2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sdxl_gpu.py tests/test_sdxl_flow_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/sdxl_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/sdxl_tests.log; exit 1; }
tail -2 $O/sdxl_tests.log
for d in 1 0 1 0; do
  env $V=$d timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5_$V$d.json 2> $O/c5_$V$d.err || { echo "C5 FAILED"; tail -20 $O/c5_$V$d.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c5_$V$d.json')); print('$V=$d', d['value'], d['ms_per_step'])"
done
