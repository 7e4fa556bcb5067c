# C5 gate for the batched LoRA reduces: SDXL GPU tests, then bench --workload c5 batched vs unbatched
# (VPT_LORA_BATCH=0), alternating: bash tools/gpu_c5b.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-c5b}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sdxl_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline >> $O/new.jsonl 2>> $O/err.log || exit 1
  VPT_LORA_BATCH=0 timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline >> $O/old.jsonl 2>> $O/err.log || exit 1
done
python3 -c "
import json
for f in ('new','old'):
    print(f, [round(json.loads(l)['value'],2) for l in open('$O/'+f+'.jsonl')])"
