# Same-box A/B of the ring GEMM grid (persistent vs one block per item) on the C3 step with the side-stream optimizer
# overlap on, alternating processes: bash tools/gpu_ring_grid_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
for i in 1 2; do
  for rg in 256 0; do
    timeout -k 10 240 python -u tools/bench_ring_grid.py $rg --overlap on --steps 30 --warmup 5 --no-cpu-baseline > $O/rg${rg}_$i.json 2> $O/rg${rg}_$i.err || { tail -20 $O/rg${rg}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'])" $O/rg${rg}_$i.json
  done
done
