#!/bin/bash
# Kernel traces of short C3 / C5 benches for the re-sort's cost
# (tools/resort_cost.py sums one re-sort's kernels): the in-tree build ("new")
# and, when given, a variant library ("old", e.g. a build before a re-sort change).
#   bash tools/resort_prof.sh <tag> [old_lib.so]
set -e
o=gpurun_out/${1:-resort}
old=${2:-}
mkdir -p $o
for w in C3 C5; do
  for v in new old; do
    if [ $v = old ]; then
      [ -n "$old" ] || continue
      export KMC_DIAG=1 KMC_LIB_PATH=$old
    else
      unset KMC_DIAG KMC_LIB_PATH
    fi
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $o/${w}_$v -o run -- \
      python3 -u bench.py --workload $w --evolve 300 --steps 200 --warmup 5 --no-cpu-baseline --no-fresh-window > $o/${w}_$v.log 2>&1
  done
done
