set -euo pipefail
out=gpurun_out/r02o; mkdir -p $out
bash tools/gpu_ab_env.sh r02o "dense_reactions or C3-8 or steady_state or poisoned or default_box or replay" "KMC_CX_MODE=1" "KMC_CX_MODE=4"
KMC_DIAG=1 KMC_LIB_PATH=$PWD/ab_variants/libkmc_stamps.so KMC_DEBUG_COUNTS=1 KMC_CX_MODE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-fresh-window --steps 20 --warmup 0 > $out/b.json 2> $out/b.err
echo done
