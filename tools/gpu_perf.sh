# GPU perf probe: per-shape GEMM microbench at HEAD + bench with per-shape GEMM breakdown.
#   bash tools/gpu_perf.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-perf}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/gemm_shapes.py --rounds 3 > $O/gemm_shapes.json 2> $O/gemm_shapes.err || { tail -30 $O/gemm_shapes.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --breakdown $O/breakdown.json > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
echo done
