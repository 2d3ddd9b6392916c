#!/bin/bash
# PMC HBM traffic of the conv family on the current tree (two passes), then the bench with
# the regenerated traffic figure, a kernel trace (step / phase breakdowns) and the
# headline-depth parity tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04n}
bash scripts/pmc_pass.sh ${T} 48 || exit 1
cp gpurun_out/${T}_traffic.json profiles/pmc_traffic.json
head -12 gpurun_out/${T}_per_kernel.txt
TAG=${T} bash scripts/r04g.sh
