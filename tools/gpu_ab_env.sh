#!/bin/bash
# Parity subset, then the default bench under several engine env settings
# (A/B of runtime knobs, same library).
#   tools/gpu_ab_env.sh <tag> "<pytest -k expr>" "ENV=1 ENV2=x" "ENV=2" ...
# An empty -k expression skips the tests.  Bench lines: gpurun_out/<tag>/bench_<i>.json
set -euo pipefail
tag=$1
kexpr=$2
shift 2
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd "$root"
if [ -n "$kexpr" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$kexpr" \
    > "$out/tests.log" 2>&1
fi
i=0
for e in "$@"; do
  echo "$e" > "$out/bench_$i.env"
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --profile > "$out/bench_$i.json" 2> "$out/bench_$i.err"
  i=$((i + 1))
done
echo "gpu_ab_env $tag done"
