# Attention diagnostic A/Bs (kernel level, tools/attn_ab.py) and the same knobs at the C3 step (tools/c3_knob_ab.py),
# diagnostic library. bash tools/gpu_attn_knobs.sh TAG SETTER[:VALUE][,SETTER[:VALUE]...] KNOB[,KNOB...]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
for sv in $(echo $2 | tr , ' '); do
  s=${sv%%:*}; v=${sv#*:}; [ "$v" = "$sv" ] && v=1
  timeout -k 10 200 python -u tools/attn_ab.py --setter $s --value $v > $O/ab_${s}_$v.json 2> $O/ab_${s}_$v.err || { tail -20 $O/ab_${s}_$v.err; exit 1; }
  cat $O/ab_${s}_$v.json
done
for k in $(echo $3 | tr , ' '); do
  timeout -k 10 300 python -u tools/c3_knob_ab.py $k --rounds 6 --steps 5 > $O/step_$k.log 2>&1 || { tail -20 $O/step_$k.log; exit 1; }
  tail -1 $O/step_$k.log
done
