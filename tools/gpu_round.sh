#!/bin/bash
# One GPU call: parity tests, bench line, kernel-trace profile of the bench.
#   tools/gpu_round.sh <tag> [pytest -k expr]
# Output under gpurun_out/<tag>/.  Each GPU step has its own time limit and
# the chain stops at the first failure.
set -euo pipefail
tag=$1
kexpr=${2:-}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd "$root"
if [ -n "$kexpr" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$kexpr" > "$out/tests.log" 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1
fi
timeout -k 10 300 python bench.py > "$out/bench.log" 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 "$root/bench.py" --no-cpu-baseline --steps 30 --warmup 10 > "$out/trace.log" 2>&1
python3 "$root/tools/prof_summary.py" "$(find "$out/trace" -name '*kernel_trace.csv' -print -quit)" 10 > "$out/summary.txt"
python3 "$root/tools/step_timeline.py" "$(find "$out/trace" -name '*kernel_trace.csv' -print -quit)" 3 > "$out/timeline.txt"
echo "gpu_round $tag done"
