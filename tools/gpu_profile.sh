#!/bin/bash
# Profile bench.py on the GPU box: kernel trace, then PMC passes (each its own
# rocprofv3 run, counters only with --kernel-trace; see MI355X_MICROARCH.md).
#   tools/gpu_profile.sh <tag> [bench args...]
# Output: gpurun_out/<tag>/{trace,fetch,write,sq,tcc}/ and <tag>/summary.txt
set -euo pipefail
tag=$1
shift
args=("$@")
[ ${#args[@]} -eq 0 ] && args=(--no-cpu-baseline --steps 30 --warmup 10)
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd /tmp
export TMPDIR=/tmp
run() {  # name, extra rocprof args...
  local name=$1
  shift
  timeout -k 10 240 rocprofv3 "$@" -d "$out/$name" -o run -- python3 "$root/bench.py" "${args[@]}" \
    >"$out/$name.log" 2>&1
}
run trace --kernel-trace --stats --output-format csv
run fetch --kernel-trace --pmc FETCH_SIZE --output-format csv
run write --kernel-trace --pmc WRITE_SIZE --output-format csv
run sq --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv
python3 "$root/tools/pmc_traffic.py" "$(find "$out/fetch" -name '*counter_collection.csv' -print -quit)" \
  "$(find "$out/write" -name '*counter_collection.csv' -print -quit)" "$out/traffic.json"
run tcc --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv
run sq2 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv || true
{
  echo "== kernel trace (mean us per launch)"
  python3 "$root/tools/prof_summary.py" "$(find "$out/trace" -name "*kernel_trace.csv" -print -quit)" 10
  for p in fetch write sq tcc sq2; do
    echo "== $p"
    python3 "$root/tools/pmc_summary.py" $(find "$out/$p" -name '*counter_collection.csv') </dev/null
  done
} >"$out/summary.txt" 2>&1
grep -h '^{' "$out/trace.log" >"$out/bench.json" || true
echo "profile $tag done"
