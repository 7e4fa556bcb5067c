set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u $R/tools/gemm_square.py --rounds 3 > $R/gpurun_out/sq9.json 2> $R/gpurun_out/sq9.err
cd /tmp && export TMPDIR=/tmp
for geo in 256 2562; do
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc9_$geo -o p -- python $R/tools/gemm_one.py 8192 8192 8192 $geo 3 > $R/gpurun_out/pmc9_$geo.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc9b_$geo -o p -- python $R/tools/gemm_one.py 8192 8192 8192 $geo 3 > $R/gpurun_out/pmc9b_$geo.log 2>&1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt9 -o p -- python $R/tools/gemm_one.py 33360 2304 768 256 5 > $R/gpurun_out/kt9.log 2>&1
