#!/bin/bash
# Round-end evidence in one GPU call: C3 steady-state kernel trace + PMC
# traffic passes, the default bench line (with the CPU baseline), and the C5
# steady-state kernel trace.  Output under gpurun_out/<tag>_C3, <tag>_C5, <tag>.
#   tools/gpu_final.sh <tag> [pmc|sq|all]   (PMC passes of the C3 profile, default pmc)
set -euo pipefail
tag=$1
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$root/gpurun_out/$tag"
cd "$root"
bash tools/gpu_steady_profile.sh "${tag}_C3" C3 "${2:-pmc}"
cd "$root"
timeout -k 10 400 python bench.py > "gpurun_out/$tag/bench.json" 2> "gpurun_out/$tag/bench.err"
bash tools/gpu_steady_profile.sh "${tag}_C5" C5
echo "final $tag done"
