#!/bin/bash
# A/B timing from one saved steady state: evolve the workload once (in-tree
# library), then every variant runs a short bench from that exact state with
# the per-kernel breakdown (HIP events, every kernel bracketed in the warm-up).
#   tools/gpu_ab3.sh <tag> "v1 v2 ..." [workload] [rounds]
# "-" = in-tree, vK = ab_variants/libkmc_vK.so, a suffix @T sets KMC_TILE=T;
# each variant is run `rounds` times interleaved.  Output
# gpurun_out/<tag>/NN_<v>.json / .err
set -euo pipefail
tag=$1
vs=$2
wl=${3:-C3}
rounds=${4:-2}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd "$root"
state=/tmp/kmc_ab_$wl.kmc
timeout -k 10 500 python bench.py --workload $wl --steps 10 --warmup 0 --no-cpu-baseline --no-fresh-window \
  --save-state $state > "$out/evolve.json" 2> "$out/evolve.err"
i=0
for r in $(seq 1 $rounds); do
  for vt in $vs; do
    i=$((i + 1))
    v=${vt%%@*}
    t=""
    [ "$v" != "$vt" ] && t=${vt##*@}
    export KMC_TILE=$t
    n=$(printf "%02d_%s" $i "${vt//@/_t}")
    if [ "$v" = "-" ]; then
      timeout -k 10 200 python bench.py --workload $wl --load-state $state --steps 100 --warmup 30 --no-cpu-baseline \
        --profile > "$out/$n.json" 2> "$out/$n.err"
    else
      KMC_DEBUG_COUNTS=$([ "$v" = st ] && echo 1 || echo 0) KMC_DIAG=1 KMC_LIB_PATH=$root/ab_variants/libkmc_$v.so \
        timeout -k 10 200 python bench.py --workload $wl --load-state $state --steps 100 --warmup 30 \
        --no-cpu-baseline --profile > "$out/$n.json" 2> "$out/$n.err"
    fi
  done
done
rm -f $state
echo "gpu_ab3 $tag done"
