# Same-box, same-process A/B of engine switches at C3 (tools/c3_knob_ab.py), run via gpurun from the repo root:
#   bash tools/gpu_ab.sh TAG KNOB[,KNOB...] [diag]
# c3_knob_ab.py loads the diagnostic library itself for the knobs that are process-wide C switches.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u tools/c3_knob_ab.py $2 --rounds 6 --steps 5 > $O/ab_$2.log 2>&1 || { tail -20 $O/ab_$2.log; exit 1; }
tail -1 $O/ab_$2.log
