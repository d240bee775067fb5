cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_persist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_gab.log 2>&1 || { echo "pytest rc=$?"; tail -20 gpurun_out/pt_gab.log; exit 1; }
tail -1 gpurun_out/pt_gab.log
timeout -k 10 200 python scripts/gemm_bench.py --bf16 --reps 10 > gpurun_out/gemm_gab.log 2>&1 || exit 1
tail -1 gpurun_out/gemm_gab.log
for L in g6 g12; do
  timeout -k 10 200 python scripts/gemm_bench.py --reps 10 --shapes Gx --lib scripts/ab/libsv_ge2e_$L.so > gpurun_out/gemm_gab_$L.log 2>&1 || exit 1
  tail -1 gpurun_out/gemm_gab_$L.log
done
ABLIBS="g6 g12" bash scripts/gpu_gemm_traffic.sh
