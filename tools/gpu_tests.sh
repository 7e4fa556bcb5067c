# Run a selection of GPU tests: bash tools/gpu_tests.sh TAG [pytest args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -5 $O/tests.log
