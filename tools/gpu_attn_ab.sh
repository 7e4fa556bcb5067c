# attention backward A/B on the GPU: build the diagnostic library there, then tools/attn_ab.py MASKS...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 300 python vision-pt_amd/vpt/_build.py --diag > $O/build.log 2>&1 || { tail -20 $O/build.log; exit 1; }
VPT_DIAG=1 timeout -k 10 300 python -u tools/attn_ab.py "$@" > $O/attn_ab.json 2> $O/attn_ab.err || { tail -20 $O/attn_ab.err; exit 1; }
cat $O/attn_ab.json
