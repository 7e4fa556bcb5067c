# N > 1 schedule with the collectives really running (bench.py --force-collective: one-rank RCCL group, every gradient
# bucket's all-reduce + bf16 wire cast and the loss all-reduce inside the timed step): overlap on / off x HW queues 8 / 4,
# interleaved twice, plus the plain N = 1 line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06f
mkdir -p $O
run() {  # tag, args
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/$1.json')); print('$1', d['value'], d['ms_per_step'], d['config']['streams'], d['config']['optimizer_overlap'])"
}
for rep in 1 2; do
  run plain_$rep
  run fc_off_q8_$rep --force-collective --overlap off --hw-queues 8
  run fc_on_q8_$rep --force-collective --overlap on --hw-queues 8
  run fc_off_q4_$rep --force-collective --overlap off --hw-queues 4
  run fc_on_q4_$rep --force-collective --overlap on --hw-queues 4
done
