set -e
o=gpurun_out/${1:-r6p}
mkdir -p $o
for w in C3 C5; do
  for v in new old; do
    if [ $v = old ]; then export KMC_DIAG=1 KMC_LIB_PATH=ab_variants/libkmc_subc3.so; else unset KMC_DIAG KMC_LIB_PATH; fi
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $o/${w}_$v -o run -- \
      python3 -u bench.py --workload $w --evolve 300 --steps 200 --warmup 5 --no-cpu-baseline --no-fresh-window > $o/${w}_$v.log 2>&1
  done
done
