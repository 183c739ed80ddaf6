#!/bin/bash
# Phase shares of the tile scans (diagnostic -DKMC_STAMPS build from
# tools/build_variants.py stamps=-DKMC_STAMPS): evolve + save, then a short run
# from the saved state that prints the accumulated per-phase cycles.
#   tools/gpu_stamps.sh <tag> [workload]
set -euo pipefail
tag=$1
wl=${2:-C3}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
state=/tmp/kmc_stamps_$wl.kmc
cd "$root"
timeout -k 10 400 python bench.py --workload $wl --steps 10 --warmup 0 --no-cpu-baseline --no-fresh-window \
  --save-state $state > "$out/evolve.json" 2> "$out/evolve.err"
KMC_DEBUG_COUNTS=1 KMC_DIAG=1 KMC_LIB_PATH=$root/ab_variants/libkmc_stamps.so timeout -k 10 200 \
  python bench.py --workload $wl --load-state $state --steps 20 --warmup 0 --no-cpu-baseline \
  > "$out/stamps.json" 2> "$out/stamps.err"
rm -f $state
echo "stamps $tag done"
