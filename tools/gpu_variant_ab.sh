set -euo pipefail
# A/B of one library variant (tools/build_variants.py): parity subset on the
# variant, then bench base / variant / base / variant.  tools/gpu_variant_ab.sh <variant>
VAR=${1:-fuse}; o=gpurun_out/ab_$VAR; mkdir -p $o
V=$PWD/ab_variants/libkmc_$VAR.so
KMC_DIAG=1 KMC_LIB_PATH=$V timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dense or C3-8 or poisoned or larger or default_box" > $o/tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline > $o/base.json 2>/dev/null
KMC_DIAG=1 KMC_LIB_PATH=$V timeout -k 10 200 python bench.py --no-cpu-baseline > $o/var.json 2>/dev/null
timeout -k 10 200 python bench.py --no-cpu-baseline > $o/base2.json 2>/dev/null
KMC_DIAG=1 KMC_LIB_PATH=$V timeout -k 10 200 python bench.py --no-cpu-baseline > $o/var2.json 2>/dev/null
echo done
