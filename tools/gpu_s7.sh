# GEMM change gate: kernel + parity tests, same-box GEMM A/B vs lib/ab/$2.so, bench A/B: bash tools/gpu_s7.sh TAG NAME
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-s7}; mkdir -p $O
[ "$3" = "notest" ] || { timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }; }
[ "$3" = "notest" ] || tail -3 $O/tests.log
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/gemm_ab.py --rounds 3 >> $O/gemm_new.jsonl 2>> $O/err.log || exit 1
  VPT_LIB_AB=vision-pt_amd/lib/ab/$2.so timeout -k 10 200 python -u tools/gemm_ab.py --rounds 3 >> $O/gemm_old.jsonl 2>> $O/err.log || exit 1
done
cat $O/gemm_new.jsonl $O/gemm_old.jsonl
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_new.json 2> $O/bench.err && cat $O/bench_new.json &&
VPT_LIB_AB=vision-pt_amd/lib/ab/$2.so timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_old.json 2>> $O/bench.err && cat $O/bench_old.json
[ "$3" = "ablate" ] && VPT_DIAG=1 timeout -k 10 400 python -u tools/gemm_epi_ablate.py --rounds 4 > $O/abl.json 2>> $O/err.log && cat $O/abl.json
true
