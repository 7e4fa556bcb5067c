set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_sdxl_gpu.py tests/test_sdxl_flow_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or lora or sdxl or flow" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/c5_knob_ab.py ops.LORA_R2_128 --rounds 6 --steps 4 > $O/r2_ab.log 2>&1 || { tail -20 $O/r2_ab.log; exit 1; }
tail -1 $O/r2_ab.log
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --breakdown $O/c5_breakdown.json > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['value'], d['ms_per_step'])"
