#!/bin/bash
# A/B of engine environment settings from one evolved state: alternating bench
# runs (two rounds), each variant a label and its settings, then one traced
# run of the first variant (kernel summary and step timeline).
#   tools/env_ab.sh <tag> <workload> <label>=<VAR=V[,VAR=V]> ...
# e.g. tools/env_ab.sh r6q C3 off=KMC_CX_STREAM=0 m3=KMC_CX_STREAM=3
set -euo pipefail
tag=$1
wl=$2
shift 2
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/$tag
mkdir -p "$out"
state=/tmp/kmc_ab_$wl.kmc
cd "$root"
timeout -k 10 500 python bench.py --workload $wl --steps 10 --warmup 0 --no-cpu-baseline --no-fresh-window \
  --save-state $state > "$out/evolve.json" 2> "$out/evolve.err"
for round in 0 1; do
  for v in "$@"; do
    label=${v%%=*}
    envs=${v#*=}
    timeout -k 10 200 env ${envs//,/ } python bench.py --workload $wl --load-state $state --steps 60 --warmup 12 \
      --no-cpu-baseline > "$out/${label}_$round.json" 2> "$out/${label}_$round.err"
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" \
      "$out/${label}_$round.json" "$label ($envs) round $round" | tee -a "$out/ab.log"
  done
done
first=$1
fenv=${first#*=}
export ${fenv//,/ }
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 "$root/bench.py" --workload $wl --load-state $state --steps 60 --warmup 12 --no-cpu-baseline \
  > "$out/bench.json" 2> "$out/trace.err"
python3 "$root/tools/prof_summary.py" "$(find "$out/trace" -name '*kernel_trace.csv' -print -quit)" 3 > "$out/summary.txt"
python3 "$root/tools/step_timeline.py" "$(find "$out/trace" -name '*kernel_trace.csv' -print -quit)" 3 > "$out/timeline.txt"
rm -f $state
echo "env ab $tag done"
