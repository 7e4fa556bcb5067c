# One round's GPU pass from the repo root (via gpurun): the GPU suite, smoke, and the bench lines
# (C3 headline, C3 with gradient checkpointing, C2, C5). Outputs under gpurun_out/<tag>/.
#   bash tools/gpu_round.sh r04a [pytest selection, default tests -m gpu]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r04}
shift
SEL=${@:-tests -m gpu}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest $SEL -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --breakdown $O/gemm_breakdown.json > $O/bench_c3.json 2> $O/bench_c3.err || { echo "C3 FAILED"; tail -30 $O/bench_c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --grad-ckpt --no-cpu-baseline > $O/bench_c3_ckpt.json 2> $O/bench_c3_ckpt.err || { echo "C3 CKPT FAILED"; tail -30 $O/bench_c3_ckpt.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c2 > $O/bench_c2.json 2> $O/bench_c2.err || { echo "C2 FAILED"; tail -30 $O/bench_c2.err; exit 1; }
timeout -k 10 400 python -u bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "C5 FAILED"; tail -30 $O/bench_c5.err; exit 1; }
python - $O <<'PY'
import json, sys
for n in ("c3", "c3_ckpt", "c2", "c5"):
    d = json.load(open(f"{sys.argv[1]}/bench_{n}.json"))
    print(n, d["value"], d["unit"], d["ms_per_step"], "ms/step", "roofline", d["roofline"]["kernel"] if "kernel" in d["roofline"] else "", d["roofline"]["frac"], "loss", d.get("final_loss"))
PY
