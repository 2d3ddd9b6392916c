set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/step_ab.py 8 > gpurun_out/step_new.log 2>&1; rc=$?; tail -1 gpurun_out/step_new.log; [ $rc -ne 0 ] && exit $rc
LS_HIP_LIB=latentsync_amd/libls_hip_old.so timeout -k 10 300 python -u scripts/step_ab.py 8 > gpurun_out/step_old.log 2>&1; rc=$?; tail -1 gpurun_out/step_old.log; exit $rc
