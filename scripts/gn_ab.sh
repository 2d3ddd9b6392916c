# gn_apply rewrite: GroupNorm parity tests + same-box step A/B (shipped vs HEAD's ls_norm.hip).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py tests/test_gpu_unet.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gn_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in new old; do
    lib=latentsync_amd/libls_hip.so; [ $v = old ] && lib=latentsync_amd/libls_hip_ab.so
    LS_HIP_LIB=$lib timeout -k 10 200 python -u scripts/step_ab.py 16 256 2>&1 | grep -v amdgpu.ids | sed "s/^/$v$r: /" || exit 1
  done
done
timeout -k 10 300 python -u scripts/step_calls.py 16 256 2>&1 | grep -E "group_norm|^step|^  [a-z]" > gpurun_out/gn_calls.log; cat gpurun_out/gn_calls.log
