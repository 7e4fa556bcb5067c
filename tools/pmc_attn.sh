# SQ counter passes over the attention kernels (tools/attn_one.py): bash tools/pmc_attn.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-pa}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --output-format csv -d $O/p1 -o p -- python3 $R/tools/attn_one.py > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM --output-format csv -d $O/p2 -o p -- python3 $R/tools/attn_one.py > $O/p2.log 2>&1 || exit 1
echo done
