set -o pipefail
mkdir -p gpurun_out
export GEMM_EPI=res,rowvec,ln
timeout -k 10 300 python -u scripts/gemm_bench.py dma@8 > gpurun_out/gemm_new.log 2>&1 && \
LS_HIP_LIB=latentsync_amd/libls_hip_old.so timeout -k 10 300 python -u scripts/gemm_bench.py dma@8 > gpurun_out/gemm_old.log 2>&1
