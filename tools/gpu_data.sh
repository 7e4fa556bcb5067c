set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-data}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_data_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python -u tools/data_bench.py > $O/data_bench.json 2> $O/data_bench.err && cat $O/data_bench.json
