#!/bin/bash
# Steady-state profile: evolve the workload (untimed, not traced) and save the
# exact state, then trace a bench run that starts from that state.  The engine
# re-sorts right after the first loaded step (kmc_set_state), so the traced
# window is in the grouped slot layout of the steady state; the warm-up (12
# steps) passes that re-sort and the timed 60 steps hold no periodic one.
#   tools/gpu_steady_profile.sh <tag> [workload] [pmc|sq|all]
# pmc: FETCH_SIZE / WRITE_SIZE passes (traffic.json); sq: SQ / LDS passes
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
timeout -k 10 500 python bench.py --workload $wl --steps 10 --warmup 0 --no-cpu-baseline --no-fresh-window \
  --save-state $state > "$out/evolve.json" 2> "$out/evolve.err"
cd /tmp
export TMPDIR=/tmp
BENCH=(python3 "$root/bench.py" --workload $wl --load-state $state --steps 60 --warmup 12 --no-cpu-baseline)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  "${BENCH[@]}" > "$out/bench.json" 2> "$out/trace.err"
python3 "$root/tools/prof_summary.py" "$(find "$out/trace" -name '*kernel_trace.csv' -print -quit)" 3 > "$out/summary.txt"
python3 "$root/tools/step_timeline.py" "$(find "$out/trace" -name '*kernel_trace.csv' -print -quit)" 3 > "$out/timeline.txt"
run_pmc() {  # name, counters...
  local name=$1
  shift
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$out/$name" -o run -- \
    "${BENCH[@]}" > "$out/$name.log" 2>&1
}
if [ "$pmc" = "pmc" ] || [ "$pmc" = "all" ]; then
  run_pmc FETCH_SIZE FETCH_SIZE
  run_pmc WRITE_SIZE WRITE_SIZE
  python3 "$root/tools/pmc_traffic.py" "$(find "$out/FETCH_SIZE" -name '*counter_collection.csv' -print -quit)" \
    "$(find "$out/WRITE_SIZE" -name '*counter_collection.csv' -print -quit)" "$out/traffic.json"
fi
if [ "$pmc" = "sq" ] || [ "$pmc" = "all" ]; then
  run_pmc sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES
  run_pmc sq2 SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES
  run_pmc tcc TCC_HIT_sum TCC_MISS_sum
  echo "k_bfs k_propose_free k_move_members k_cx_check k_complex_heavy k_rec_scatter k_pair_scan k_col_exact k_col_resolve k_commit_rxn k_match k_diss_observe" | \
    python3 "$root/tools/pmc_summary.py" $(find "$out/sq1" "$out/sq2" "$out/tcc" -name '*counter_collection.csv') > "$out/pmc_summary.txt"
fi
rm -f $state
echo "steady profile $tag done"
