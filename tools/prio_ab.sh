#!/bin/bash
# A/B of the complex stream's priority (KMC_CX_STREAM_PRIO) from one evolved
# state per workload: alternating bench runs, then one traced run with the
# priority on (step timeline).
#   tools/prio_ab.sh <tag> [workload] [KMC_CX_STREAM]
set -euo pipefail
tag=$1
wl=${2:-C5}
cx=${3:-}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
state=/tmp/kmc_prio_$wl.kmc
cd "$root"
[ -n "$cx" ] && export KMC_CX_STREAM=$cx
timeout -k 10 500 python bench.py --workload $wl --steps 10 --warmup 0 --no-cpu-baseline --no-fresh-window \
  --save-state $state > "$out/evolve.json" 2> "$out/evolve.err"
for round in 0 1; do
  for p in 1 0; do
    KMC_CX_STREAM_PRIO=$p timeout -k 10 200 python bench.py --workload $wl --load-state $state --steps 60 --warmup 12 \
      --no-cpu-baseline > "$out/prio${p}_$round.json" 2> "$out/prio${p}_$round.err"
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" \
      "$out/prio${p}_$round.json" "prio=$p round $round" | tee -a "$out/ab.log"
  done
done
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 "$root/bench.py" --workload $wl --load-state $state --steps 60 --warmup 12 --no-cpu-baseline \
  > "$out/bench.json" 2> "$out/trace.err"
python3 "$root/tools/prof_summary.py" "$(find "$out/trace" -name '*kernel_trace.csv' -print -quit)" 3 > "$out/summary.txt"
python3 "$root/tools/step_timeline.py" "$(find "$out/trace" -name '*kernel_trace.csv' -print -quit)" 3 > "$out/timeline.txt"
rm -f $state
echo "prio ab $tag done"
