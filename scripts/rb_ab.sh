# row-block residual DMA: GEMM parity tests, then same-box A/B (shipped = residual through
# LDS DMA, ab = HEAD's register residual) and the K = 640 residual switch.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rb_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rb_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in new old new640; do
    lib=latentsync_amd/libls_hip.so; [ $v = old ] && lib=latentsync_amd/libls_hip_ab.so
    e=""; [ $v = new640 ] && e="LS_GEMM_RB640_RES=1"
    env $e LS_HIP_LIB=$lib timeout -k 10 200 python -u scripts/step_ab.py 16 256 2>&1 | grep -v amdgpu.ids | sed "s/^/$v$r: /" || exit 1
  done
done
