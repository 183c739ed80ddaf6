#!/bin/bash
set -euo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r3i
mkdir -p "$out"
cd "$root"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread \
  -k "dense or global_tile or benchmark_workload or threshold or poisoned or resort or graph or default_box" > "$out/tests.log" 2>&1
bash tools/gpu_ab3.sh r3i_ab "- dni r3f st" C3 2
