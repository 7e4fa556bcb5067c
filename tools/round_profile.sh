# One round's measurement set on a GPU box (run via gpurun from the repo root):
#   rocprofv3 kernel-trace stats of a short bench, FETCH_SIZE / WRITE_SIZE / MFMA-busy counter passes of the
#   same command (one counter group per pass), per-op traffic summary. Outputs under gpurun_out/<tag>/.
#   bash tools/round_profile.sh r03a
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o p -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/ktrace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o p -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_mfma -o p -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/pmc_mfma.log 2>&1
python $R/tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/ktrace $O/traffic.json $O/pmc_mfma > $O/traffic.log 2>&1
cat $O/traffic.log | tail -5
