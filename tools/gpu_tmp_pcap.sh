set -euo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r02y
mkdir -p "$out"
state=/tmp/kmc_probe_C3.kmc
cd "$root"
timeout -k 10 400 python bench.py --workload C3 --steps 10 --warmup 0 --no-cpu-baseline --no-fresh-window \
  --save-state $state > "$out/evolve.json" 2> "$out/evolve.err"
for v in base p4096 p1024 base p4096; do
  if [ $v = base ]; then e=""; else e="KMC_DIAG=1 KMC_LIB_PATH=$root/ab_variants/libkmc_$v.so"; fi
  env $e timeout -k 10 200 python bench.py --workload C3 --load-state $state --steps 100 \
    --warmup 105 --no-cpu-baseline --profile > "$out/$v.json" 2>> "$out/$v.err"
done
rm -f $state
echo done
