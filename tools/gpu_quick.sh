#!/bin/bash
# Quick GPU check: selected parity tests, kernel trace of the bench, bench line.
#   tools/gpu_quick.sh <tag> "<pytest -k expr>"
# Output under gpurun_out/<tag>/; each GPU step has its own time limit and
# the chain stops at the first failure.
set -euo pipefail
tag=$1
kexpr=$2
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd "$root"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$kexpr" > "$out/tests.log" 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 "$root/bench.py" --no-cpu-baseline --steps 30 --warmup 10 > "$out/trace.log" 2>&1
cd "$root"
python3 tools/step_timeline.py "$(find "$out/trace" -name '*kernel_trace.csv' -print -quit)" 3 > "$out/timeline.txt"
timeout -k 10 200 python bench.py --no-cpu-baseline > "$out/bench.log" 2>&1
echo "gpu_quick $tag done"
