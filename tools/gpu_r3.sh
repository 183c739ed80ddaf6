#!/bin/bash
# One GPU call of round 3: the whole -m gpu suite, the default bench line,
# then the C3 steady-state profile (kernel trace + optional PMC passes).
#   tools/gpu_r3.sh <tag> [pmc|sq|all|none] [pytest -k expr|ALL|SKIP]
# Every GPU step runs under its own time limit; the chain stops at the first
# failure (set -e).  Output under gpurun_out/<tag>*.
set -euo pipefail
tag=$1
pmc=${2:-pmc}
kexpr=${3:-ALL}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd "$root"
if [ "$kexpr" != "SKIP" ]; then
  K=()
  [ "$kexpr" != "ALL" ] && K=(-k "$kexpr")
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread "${K[@]}" \
    > "$out/tests.log" 2>&1
fi
timeout -k 10 500 python bench.py > "$out/bench.json" 2> "$out/bench.err"
if [ "$pmc" != "skip" ]; then
  bash tools/gpu_steady_profile.sh "${tag}_C3" C3 "$([ "$pmc" = none ] && echo "" || echo "$pmc")"
fi
echo "gpu_r3 $tag done"
