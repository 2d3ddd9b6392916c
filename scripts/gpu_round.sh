set -o pipefail
bash scripts/gpu_full.sh r1d && bash scripts/pmc_pass.sh r1d
