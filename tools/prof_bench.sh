# Round profile: bench line, kernel microbench, rocprofv3 kernel-trace stats of a short bench run.
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u $R/bench.py > $R/gpurun_out/bench_$TAG.log 2>&1
timeout -k 10 300 python -u $R/tools/kernel_bench.py --rounds 3 > $R/gpurun_out/kb_$TAG.json 2> $R/gpurun_out/kb_$TAG.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o p -- python $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof_$TAG.log 2>&1
