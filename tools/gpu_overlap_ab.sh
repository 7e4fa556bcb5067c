# Same-box A/B of the optimizer placement at N = 1 (one launch after the backward vs per bucket on a side stream during
# it), alternating processes: bash tools/gpu_overlap_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
for i in 1 2; do
  for ov in off on; do
    timeout -k 10 240 python -u bench.py --overlap $ov --steps 30 --warmup 5 --no-cpu-baseline > $O/ov_${ov}_$i.json 2> $O/ov_${ov}_$i.err || { tail -20 $O/ov_${ov}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'])" $O/ov_${ov}_$i.json
  done
done
