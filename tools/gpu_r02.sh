# Round-2 GPU session: parity suite, smoke, bench line, rocprofv3 kernel stats + PMC passes (HBM traffic,
# MFMA busy) of a short bench. Every GPU step under its own timeout, chained with &&.
#   bash tools/gpu_r02.sh TAG [skip_tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r02a}
O=gpurun_out/$TAG
mkdir -p $O
if [ "$2" != "skip_tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && cat $O/smoke.log || exit 1
fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err && cat $O/bench.json || exit 1
CMD="bench.py --steps 5 --warmup 2 --no-cpu-baseline"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/ktrace -o p -- python3 $R/$CMD > $R/$O/ktrace.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_fetch -o p -- python3 $R/$CMD > $R/$O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_write -o p -- python3 $R/$CMD > $R/$O/pmc_write.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/$O/pmc_mfma -o p -- python3 $R/$CMD > $R/$O/pmc_mfma.log 2>&1 || exit 1
python3 $R/tools/pmc_traffic.py $R/$O/pmc_fetch $R/$O/pmc_write $R/$O/ktrace $R/$O/traffic.json $R/$O/pmc_mfma > $R/$O/traffic.log 2>&1
echo done
