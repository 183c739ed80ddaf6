#!/bin/bash
# probe: side-stream complexes (parity + bench), tile-scan stage timings
set -euo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/probe1
mkdir -p "$out"
cd "$root"
KMC_SIDE=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "dense_reactions or larger_box or C3" > "$out/tests_side.log" 2>&1
KMC_SIDE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --profile > "$out/bench_side.json" 2> "$out/bench_side.err"
timeout -k 10 200 python bench.py --no-cpu-baseline --profile > "$out/bench_base.json" 2> "$out/bench_base.err"
for st in 1 2 3; do
  KMC_DEBUG_SCAN_STAGE=$st timeout -k 10 200 python bench.py --no-cpu-baseline --profile --steps 100 > "$out/stage$st.json" 2> "$out/stage$st.err"
done
echo probe1 done
