#!/bin/bash
# Pair-scan phase costs from one saved steady state: the same short window
# with the scan stopped after staging (KMC_DEBUG_SCAN_STAGE=1), before the
# list flush (3) and complete (0); per-kernel HIP-event breakdown on stderr.
# Timing only: stages 1 and 3 drop the scan's output (the trajectory is not
# the reference's).   tools/gpu_stage_probe.sh <tag> [workload]
set -euo pipefail
tag=$1
wl=${2:-C3}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd "$root"
state=/tmp/kmc_probe_$wl.kmc
timeout -k 10 500 python bench.py --workload $wl --steps 10 --warmup 0 --no-cpu-baseline --no-fresh-window \
  --save-state $state > "$out/evolve.json" 2> "$out/evolve.err"
for st in 0 1 3 0; do
  KMC_DEBUG_SCAN_STAGE=$st timeout -k 10 200 python bench.py --workload $wl --load-state $state --steps 10 --warmup 10 \
    --no-cpu-baseline --profile > "$out/stage$st.json" 2>> "$out/stage$st.err"
done
rm -f $state
echo "stage probe $tag done"
