# HW queues 4 vs 8 without collectives (N = 1 line) and with them (--force-collective), interleaved x3
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06g
mkdir -p $O
run() {  # tag, args
  timeout -k 10 240 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
  python -c "import json; t=open('$O/$1.json').read(); d=json.loads(t[t.index('{'):]); print('$1', d['value'], d['ms_per_step'])"
}
for rep in 1 2 3; do
  run q4_$rep --hw-queues 4
  run q8_$rep --hw-queues 8
  run q2_$rep --hw-queues 2
  run fc_q4_$rep --force-collective --hw-queues 4
  run fc_q8_$rep --force-collective --hw-queues 8
  run fc_q2_$rep --force-collective --hw-queues 2
done
