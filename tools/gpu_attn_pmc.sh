# SQ counter passes over the attention kernels at the C3 shape (tools/attn_shape_run.py), one pass per counter group
# (MI355X_MICROARCH.md rocprofv3 limits), plus a kernel-trace pass. bash tools/gpu_attn_pmc.sh TAG
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o p -- python $R/tools/attn_shape_run.py > $O/kt.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/pa -o p -- python $R/tools/attn_shape_run.py > $O/pa.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM --output-format csv -d $O/pb -o p -- python $R/tools/attn_shape_run.py > $O/pb.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_EXP SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/pc -o p -- python $R/tools/attn_shape_run.py > $O/pc.log 2>&1
echo ok
