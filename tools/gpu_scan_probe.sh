#!/bin/bash
# Timing probe of the two tile scans at a steady state: evolve + save, then
# short runs from that state with the scans stopped after stage 1 (staging),
# 2 (pair lists), 3 (pair checks, no flush) and complete (0).  Results of the
# stopped runs are invalid; only the per-kernel times matter.
#   tools/gpu_scan_probe.sh <tag> [workload]
set -euo pipefail
tag=$1
wl=${2:-C3}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
state=/tmp/kmc_probe_$wl.kmc
cd "$root"
timeout -k 10 400 python bench.py --workload $wl --steps 10 --warmup 0 --no-cpu-baseline --no-fresh-window \
  --save-state $state > "$out/evolve.json" 2> "$out/evolve.err"
for st in ${STAGES:-1 2 3 0}; do
  KMC_DEBUG_SCAN_STAGE=$st timeout -k 10 200 python bench.py --workload $wl --load-state $state --steps 40 \
    --warmup 105 --no-cpu-baseline --profile > "$out/stage$st.json" 2> "$out/stage$st.err" || true
done
rm -f $state
echo "scan probe $tag done"
