#!/bin/bash
# Same-box A/B of two variants, alternated (A, B, A, B) so clock / temperature drift hits
# both; every GPU step under its own time limit, the first failure ends the run.
#
#   bash scripts/ab.sh TAG VARIANT MEASURE [TESTS]
#
# VARIANT  lib          A = latentsync_amd/libls_hip.so, B = latentsync_amd/libls_hip_ab.so
#                       (build B with scripts/build_ab.sh COMMIT [file])
#          env:VAR=VAL  A = plain, B = with VAR=VAL exported (an LS_* switch)
#          lib+env:VAR=VAL  B = libls_hip_ab.so with VAR=VAL exported
# MEASURE  step[:W]     scripts/step_ab.py, one graph-replayed UNet step at W windows (default 32)
#          trace        rocprofv3 --kernel-trace of a 1-batch bench; per-kernel comparison of one
#                       mid-run step (scripts/cmp_steps.py, min over runs) -> gpurun_out/TAG_cmp.txt
#          attn:WHICH   scripts/attn_bench.py with ATTN_ONLY=WHICH (e.g. "spatial L0", cross, temporal)
# TESTS    optional pytest selector (-k expression) run first on variant A, e.g. "attention or rowblock"
set -o pipefail
tag=${1:?tag}; variant=${2:?variant}; measure=${3:-step}; tests=$4
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -k "$tests" -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${tag}_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/${tag}_tests.log; [ $rc -ne 0 ] && exit $rc
fi
run() {  # $1 = A|B, $2 = round
  local envs=()
  case $variant in
    lib) [ "$1" = B ] && envs+=(LS_HIP_LIB=latentsync_amd/libls_hip_ab.so) ;;
    lib+env:*) [ "$1" = B ] && envs+=(LS_HIP_LIB=latentsync_amd/libls_hip_ab.so "${variant#lib+env:}") ;;
    env:*) [ "$1" = B ] && envs+=("${variant#env:}") ;;
    *) echo "unknown variant $variant"; return 2 ;;
  esac
  case $measure in
    step*) local w=${measure#step}; w=${w#:}
      env "${envs[@]}" timeout -k 10 300 python -u scripts/step_ab.py ${w:-32} 256 2>&1 | grep -v amdgpu.ids | sed "s/^/$1$2 /" ;;
    attn:*) env "${envs[@]}" NO_SDPA=1 WINDOWS=32 ATTN_ONLY="${measure#attn:}" timeout -k 10 200 \
      python -u scripts/attn_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$1$2 /" ;;
    trace) env "${envs[@]}" timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${tag}_$1$2 -o run -- \
      python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-single-window --no-whisper \
      > gpurun_out/${tag}_$1$2.log 2>&1; local r=$?; echo "$1$2 rc=$r"; return $r ;;
    *) echo "unknown measure $measure"; return 2 ;;
  esac
}
for r in 1 2 3; do  # three alternated rounds: single-run A/Bs sit inside the +-1 % run-to-run spread
  for v in A B; do
    run $v $r || exit 1
  done
done
if [ "$measure" = trace ]; then
  python3 scripts/cmp_steps.py "gpurun_out/${tag}_A*" "gpurun_out/${tag}_B*" 20 > gpurun_out/${tag}_cmp.txt
  rc=$?; cat gpurun_out/${tag}_cmp.txt
  rm -rf gpurun_out/${tag}_A? gpurun_out/${tag}_B?  # traces stay on the box (the copy-back cap)
  exit $rc
fi
