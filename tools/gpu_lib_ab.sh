# In-process A/B of library builds (tools/lib_ab.py; variants built by vpt._build.build_variant into lib/var/), then
# optional diagnostic-switch A/Bs. bash tools/gpu_lib_ab.sh TAG VARIANTS WHAT [SETTER:VALUE [KNOB]]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 500 python -u tools/lib_ab.py --variants $2 --what $3 --rounds 6 > $O/lib_ab.log 2>&1 || { tail -30 $O/lib_ab.log; exit 1; }
tail -3 $O/lib_ab.log
if [ -n "$4" ]; then
  s=${4%%:*}; v=${4#*:}
  timeout -k 10 200 python -u tools/attn_ab.py --setter $s --value $v > $O/ab_${s}_$v.json 2> $O/ab_${s}_$v.err || { tail -20 $O/ab_${s}_$v.err; exit 1; }
  cat $O/ab_${s}_$v.json
fi
if [ -n "$5" ]; then
  timeout -k 10 300 python -u tools/c3_knob_ab.py $5 --rounds 6 --steps 5 > $O/step_$5.log 2>&1 || { tail -20 $O/step_$5.log; exit 1; }
  tail -1 $O/step_$5.log
fi
