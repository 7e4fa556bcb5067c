# One round's measurement set on a GPU box (run via gpurun from the repo root):
#   bench line, rocprofv3 kernel-trace stats of a short bench, FETCH_SIZE and WRITE_SIZE counter passes
#   of the same command, per-op traffic summary. Outputs under gpurun_out/<tag>/.
#   bash tools/round_profile.sh r01
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
O=$R/gpurun_out/$TAG
mkdir -p $O
CMD="python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 400 python -u $R/bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o p -- $CMD > $O/ktrace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- $CMD > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o p -- $CMD > $O/pmc_write.log 2>&1
python $R/tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/ktrace $O/traffic.json > $O/traffic.log 2>&1
