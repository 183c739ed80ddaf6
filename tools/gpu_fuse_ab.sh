set -euo pipefail
o=gpurun_out/fuse; mkdir -p $o
V=$PWD/kmc-with-a-diffusion-reaction-algorithm_amd/lib/variants/libkmc_fuse.so
KMC_LIB_PATH=$V timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dense or C3-8 or poisoned or larger or default_box" > $o/tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline > $o/base.json 2>/dev/null
KMC_LIB_PATH=$V timeout -k 10 200 python bench.py --no-cpu-baseline > $o/fuse.json 2>/dev/null
timeout -k 10 200 python bench.py --no-cpu-baseline > $o/base2.json 2>/dev/null
KMC_LIB_PATH=$V timeout -k 10 200 python bench.py --no-cpu-baseline > $o/fuse2.json 2>/dev/null
echo done
