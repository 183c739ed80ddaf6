#!/bin/bash
# Quick round-3 check: selected parity tests, the default bench line, the C3
# steady-state kernel trace.  tools/gpu_quick3.sh <tag> "<pytest -k expr>"
set -euo pipefail
tag=$1
kexpr=$2
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd "$root"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread -k "$kexpr" > "$out/tests.log" 2>&1
timeout -k 10 400 python bench.py --no-cpu-baseline > "$out/bench.json" 2> "$out/bench.err"
bash tools/gpu_steady_profile.sh "${tag}_C3" C3
echo "quick3 $tag done"
