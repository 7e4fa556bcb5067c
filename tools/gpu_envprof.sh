# rocprof kernel stats of a bench under several values of one env knob: bash tools/gpu_envprof.sh TAG VAR v1 v2 ...
# prints the per-step totals of the kernels whose names match $MATCH (default: lora_wgrad); BENCH_ARGS (default: the
# C5 workload, 3 + 2 steps) and STEPS (launch-count divisor, default 6) select the bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
V=$2
shift 2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  export $V=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o p -- python $R/bench.py ${BENCH_ARGS:---workload c5 --steps 3 --warmup 2 --no-cpu-baseline} > $O/$v.log 2>&1 || exit 1
done
python - "$O" "${MATCH:-lora_wgrad}" "${STEPS:-6}" "$@" <<'PY'
import csv, glob, sys
o, match, steps, vals = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4:]
for v in vals:
    f = glob.glob(f"{o}/{v}/**/*kernel_stats.csv", recursive=True)[0]
    tot = 0.0
    for r in csv.DictReader(open(f)):
        if any(m in r["Name"] for m in match.split(",")):
            ms = float(r["TotalDurationNs"]) / 1e6 / steps
            tot += ms
            print(v, r["Calls"], f"{ms:.3f} ms/step", f"{float(r['AverageNs']) / 1e3:.2f} us", r["Name"][:60])
    print(v, "total", f"{tot:.3f} ms/step")
PY
