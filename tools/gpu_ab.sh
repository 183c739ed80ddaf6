#!/bin/bash
# A/B timing of library variants (tools/build_variants.py) after a parity
# subset on the default library.
#   tools/gpu_ab.sh <tag> "<pytest -k expr>" variant1 variant2 ...
set -euo pipefail
tag=$1
kexpr=$2
shift 2
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd "$root"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$kexpr" > "$out/tests.log" 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline > "$out/bench_base.json" 2> "$out/bench_base.err"
for v in "$@"; do
  KMC_DIAG=1 KMC_LIB_PATH=$root/ab_variants/libkmc_$v.so \
    timeout -k 10 200 python bench.py --no-cpu-baseline > "$out/bench_$v.json" 2> "$out/bench_$v.err"
done
timeout -k 10 200 python bench.py --no-cpu-baseline > "$out/bench_base2.json" 2> "$out/bench_base2.err"
echo "gpu_ab $tag done"
