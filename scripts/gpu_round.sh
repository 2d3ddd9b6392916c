# Round-end GPU evidence: gpu tests -> bench -> rocprofv3 kernel stats -> two PMC passes.
# usage: bash scripts/gpu_round.sh TAG
set -o pipefail
tag=${1:-r1e}
bash scripts/gpu_full.sh $tag && bash scripts/pmc_pass.sh $tag
