set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/step_calls.py 8 256 encode > gpurun_out/p20_enc.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/step_calls.py 8 256 decode > gpurun_out/p20_dec.log 2>&1
