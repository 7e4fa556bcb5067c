# kernel times of the attention backward's two block kinds as separate launches (diagnostic library)
set -e
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python vision-pt_amd/vpt/_build.py --diag > /dev/null
O=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
VPT_DIAG=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/split -o p -- python $GRAFT_REPO_ROOT/tools/attn_one.py --iters 10 --rows64 8 > $O/split.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prod -o p -- python $GRAFT_REPO_ROOT/tools/attn_one.py --iters 10 > $O/prod.log 2>&1
for d in split prod; do python3 -c "
import csv
for r in csv.DictReader(open('$O/$d/p_kernel_stats.csv')):
    print('$d', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"; done
