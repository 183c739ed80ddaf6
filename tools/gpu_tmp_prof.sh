set -euo pipefail
root=$(pwd)
bash tools/gpu_steady_profile.sh r02i C3 pmc
out=$root/gpurun_out/r02i_fresh; mkdir -p $out
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 "$root/bench.py" --evolve 0 --no-fresh-window --steps 30 --warmup 5 --no-cpu-baseline > "$out/bench.json" 2> "$out/trace.err"
python3 "$root/tools/prof_summary.py" "$(find "$out/trace" -name '*kernel_trace.csv' -print -quit)" 5 > "$out/summary.txt"
for p in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $p --output-format csv -d "$out/$p" -o run -- python3 "$root/bench.py" --evolve 0 --no-fresh-window --steps 30 --warmup 5 --no-cpu-baseline > "$out/$p.log" 2>&1
done
python3 "$root/tools/pmc_traffic.py" "$(find "$out/FETCH_SIZE" -name '*counter_collection.csv' -print -quit)" "$(find "$out/WRITE_SIZE" -name '*counter_collection.csv' -print -quit)" "$out/traffic.json"
echo done
