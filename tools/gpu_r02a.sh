#!/bin/bash
# Round-2 checks: new parity tests (replay, replicas, C2 long, steady-state
# windows), then bench lines (C3 default with evolution, C5).
set -euo pipefail
tag=${1:-r02a}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd "$root"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "replay or two_gpu or c2_long or chunked or default_box" > "$out/tests_new.log" 2>&1
timeout -k 10 500 python -u -m pytest tests/test_gpu_steady.py -x -v -s --timeout 600 --timeout-method thread \
  > "$out/tests_steady.log" 2>&1
timeout -k 10 300 python bench.py --profile > "$out/bench_C3.json" 2> "$out/bench_C3.err"
timeout -k 10 400 python bench.py --workload C5 --steps 20 --warmup 5 --no-cpu-baseline --profile \
  > "$out/bench_C5.json" 2> "$out/bench_C5.err"
echo "gpu_r02a done"
