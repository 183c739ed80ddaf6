set -euo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r02x
mkdir -p "$out"
state=/tmp/kmc_probe_C3.kmc
cd "$root"
timeout -k 10 400 python bench.py --workload C3 --steps 10 --warmup 0 --no-cpu-baseline --no-fresh-window \
  --save-state $state > "$out/evolve.json" 2> "$out/evolve.err"
for st in 1 5 4 2 0; do
  KMC_DEBUG_SCAN_STAGE=$st timeout -k 10 200 python bench.py --workload C3 --load-state $state --steps 40 \
    --warmup 105 --no-cpu-baseline --profile > "$out/stage$st.json" 2> "$out/stage$st.err"
done
for t in 10 11 12 14; do
  KMC_TILE=$t timeout -k 10 200 python bench.py --workload C3 --load-state $state --steps 40 \
    --warmup 105 --no-cpu-baseline --profile > "$out/tile$t.json" 2> "$out/tile$t.err"
done
rm -f $state
echo done
