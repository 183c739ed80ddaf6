#!/bin/bash
# Steady-state profile: evolve the workload (untimed, not traced) and save the
# exact state, then trace a bench run that starts from that state.
#   tools/gpu_steady_profile.sh <tag> [workload] [pmc|sq|all]
# pmc: FETCH_SIZE / WRITE_SIZE passes (traffic.json); sq: SQ + TCC passes
# Output: gpurun_out/<tag>/{evolve.json,trace/,summary.txt,timeline.txt,bench.json}
set -euo pipefail
tag=$1
wl=${2:-C3}
pmc=${3:-}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
state=/tmp/kmc_steady_$wl.kmc
cd "$root"
timeout -k 10 400 python bench.py --workload $wl --steps 10 --warmup 0 --no-cpu-baseline --no-fresh-window \
  --save-state $state > "$out/evolve.json" 2> "$out/evolve.err"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 "$root/bench.py" --workload $wl --load-state $state --steps 30 --warmup 105 --no-cpu-baseline \
  > "$out/bench.json" 2> "$out/trace.err"
python3 "$root/tools/prof_summary.py" "$(find "$out/trace" -name '*kernel_trace.csv' -print -quit)" 5 > "$out/summary.txt"
python3 "$root/tools/step_timeline.py" "$(find "$out/trace" -name '*kernel_trace.csv' -print -quit)" 3 > "$out/timeline.txt"
if [ "$pmc" = "pmc" ] || [ "$pmc" = "all" ]; then
  for p in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $p --output-format csv -d "$out/$p" -o run -- \
      python3 "$root/bench.py" --workload $wl --load-state $state --steps 30 --warmup 105 --no-cpu-baseline \
      > "$out/$p.log" 2>&1
  done
  python3 "$root/tools/pmc_traffic.py" "$(find "$out/FETCH_SIZE" -name '*counter_collection.csv' -print -quit)" \
    "$(find "$out/WRITE_SIZE" -name '*counter_collection.csv' -print -quit)" "$out/traffic.json"
fi
if [ "$pmc" = "sq" ] || [ "$pmc" = "all" ]; then
  run_pmc() {  # name, counters...
    local name=$1
    shift
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$out/$name" -o run -- \
      python3 "$root/bench.py" --workload $wl --load-state $state --steps 30 --warmup 105 --no-cpu-baseline \
      > "$out/$name.log" 2>&1
  }
  run_pmc sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES
  run_pmc tcc TCC_HIT_sum TCC_MISS_sum
  echo "k_bfs k_complex k_complex_heavy k_propose_free k_pair_scan k_rec_scatter k_rej_commit" | \
    python3 "$root/tools/pmc_summary.py" $(find "$out/sq" "$out/tcc" -name '*counter_collection.csv') > "$out/pmc_summary.txt"
fi
rm -f $state
echo "steady profile $tag done"
