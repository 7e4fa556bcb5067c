# One round's measurement set on a GPU box (run via gpurun from the repo root):
#   rocprofv3 kernel-trace stats of a short bench, FETCH_SIZE / WRITE_SIZE / MFMA-busy counter passes of the
#   same command (one counter group per pass), per-op traffic summary. Outputs under gpurun_out/<tag>/.
#   bash tools/round_profile.sh r03a [workload, default c3]
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
WL=${2:-c3}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
# per-kernel times and counters with every kernel on the step's stream (as the bench's probe pass measures them: a
# kernel sharing the chip with a concurrent one would read slow); KT_SIDE=1 adds a trace of the default (multi-stream)
# schedule for its wall time
CMD="$R/bench.py --workload $WL --steps 5 --warmup 2 --no-cpu-baseline --streams single"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o p -- python $CMD > $O/ktrace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- python $CMD > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o p -- python $CMD > $O/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_mfma -o p -- python $CMD > $O/pmc_mfma.log 2>&1
if [ "${KT_SIDE:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace_side -o p -- python $R/bench.py --workload $WL --steps 5 --warmup 2 --no-cpu-baseline > $O/ktrace_side.log 2>&1
  python $R/tools/ktrace_summary.py $O/ktrace_side > $O/ktrace_side_summary.txt 2>&1 || true
fi
python $R/tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/ktrace $O/traffic.json $O/pmc_mfma --tag $TAG > $O/traffic.log 2>&1
python $R/tools/ktrace_summary.py $O/ktrace > $O/ktrace_summary.txt 2>&1 || true
tail -5 $O/traffic.log
