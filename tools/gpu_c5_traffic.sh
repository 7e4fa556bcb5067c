# HBM traffic of the C5 (SDXL QLoRA) step's GEMM and attention kernels: a kernel-trace pass and FETCH_SIZE / WRITE_SIZE
# counter passes restricted to those kernels (--kernel-include-regex: every other dispatch of the ~4,200 per step, and
# the NF4 quantisation at init, runs without counter collection), a short bench (1 warm-up + 2 timed steps + the probe
# pass). bash tools/gpu_c5_traffic.sh TAG    -> gpurun_out/TAG/traffic_c5.json
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CMD="$R/bench.py --workload c5 --steps 2 --warmup 1"
RX='gemm_ring_kernel|gemm_r2_kernel|gemm_bf16_kernel|splitk_reduce_kernel|attn_fwd_kernel|attn_bwd'
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o p -- python3 -u $CMD > $O/ktrace.log 2>&1
echo ktrace done
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/pmc_fetch -o p -- python3 -u $CMD > $O/pmc_fetch.log 2>&1
echo fetch done
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/pmc_write -o p -- python3 -u $CMD > $O/pmc_write.log 2>&1
echo write done
python3 $R/tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/ktrace $O/traffic_c5.json --c5 --tag $1 > $O/traffic.log 2>&1
tail -30 $O/traffic.log
