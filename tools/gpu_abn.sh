#!/bin/bash
# Interleaved A/B benches after a parity subset on the in-tree library.
#   tools/gpu_abn.sh <tag> "<pytest -k expr>" "v1 v2 ..."   ("-" = in-tree; vK = ab_variants/libkmc_vK.so;
#   v@TILE sets KMC_TILE, a trailing +g sets KMC_GRAPH=1).  Outputs gpurun_out/<tag>/NN_<v>.json with the per-kernel breakdown on stderr.
set -euo pipefail
tag=$1
kexpr=$2
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd "$root"
if [ -n "$kexpr" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$kexpr" > "$out/tests.log" 2>&1
fi
i=0
for vt in $3; do
  i=$((i + 1))
  g=""
  x=$vt
  if [ "${x%+g}" != "$x" ]; then g=1; x=${x%+g}; fi
  v=${x%%@*}
  t=""
  [ "$v" != "$x" ] && t=${x##*@}
  n=$(printf "%02d_%s" $i "${vt//@/_t}")
  export KMC_GRAPH=$g
  if [ "$v" = "-" ]; then
    KMC_TILE=$t timeout -k 10 200 python bench.py --no-cpu-baseline --profile > "$out/$n.json" 2> "$out/$n.err"
  else
    KMC_TILE=$t KMC_DIAG=1 KMC_LIB_PATH=$root/ab_variants/libkmc_$v.so \
      timeout -k 10 200 python bench.py --no-cpu-baseline --profile > "$out/$n.json" 2> "$out/$n.err"
  fi
done
echo "gpu_abn $tag done"
