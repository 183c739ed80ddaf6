set -euo pipefail
bash tools/gpu_ab_env.sh r02z "test" "KMC_CX_MODE=1"
timeout -k 10 500 python bench.py --workload C5 --steps 20 --warmup 5 --no-cpu-baseline --no-fresh-window --profile > gpurun_out/r02z/c5.json 2> gpurun_out/r02z/c5.err
echo done
