# SDXL GPU tests, one C5 bench and its rocprof kernel stats: bash tools/gpu_c5t.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sdxl_gpu.py tests/test_sdxl_flow_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/sdxl_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/sdxl_tests.log; exit 1; }
tail -2 $O/sdxl_tests.log
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { echo "C5 FAILED"; tail -20 $O/c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['value'], d['ms_per_step'])"
bash tools/prof_c5.sh $1
