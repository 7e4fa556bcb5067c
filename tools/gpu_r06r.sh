set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06r
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c3.json')); print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['mean_launch_ms'])"
KT_SIDE=1 bash tools/round_profile.sh r06r_prof c3 || exit 1
bash tools/round_profile.sh r06r_c2_prof c2 || exit 1
bash tools/gpu_ddp_rehearsal.sh r06r_ddp || exit 1
