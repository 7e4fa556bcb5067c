# Same-box A/B of the attention kernels: production lib vs vision-pt_amd/lib/ab/$2.so, alternating processes.
#   bash tools/ab_attn.sh TAG NAME
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ab}; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 120 python -u tools/attn_one.py --time --iters 5 >> $O/new.jsonl 2>> $O/err.log || exit 1
  VPT_LIB_AB=vision-pt_amd/lib/ab/$2.so timeout -k 10 120 python -u tools/attn_one.py --time --iters 5 >> $O/old.jsonl 2>> $O/err.log || exit 1
done
echo new; cat $O/new.jsonl; echo old; cat $O/old.jsonl
