# XCD block-order A/B of the attention kernels (diagnostic library): event timing in one process, then FETCH_SIZE /
# WRITE_SIZE / L2 hit passes per order over tools/attn_shape_run.py --only. bash tools/gpu_attn_xcd.sh TAG
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
timeout -k 10 200 python -u $R/tools/attn_ab.py --setter vpt_attn_set_xcd_order > $O/xcd_ab.json 2> $O/xcd_ab.err
cat $O/xcd_ab.json
cd /tmp && export TMPDIR=/tmp
for x in 0 1; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch$x -o p -- python $R/tools/attn_shape_run.py --only 1 --xcd $x > $O/fetch$x.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write$x -o p -- python $R/tools/attn_shape_run.py --only 1 --xcd $x > $O/write$x.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/hit$x -o p -- python $R/tools/attn_shape_run.py --only 1 --xcd $x > $O/hit$x.log 2>&1
done
echo ok
