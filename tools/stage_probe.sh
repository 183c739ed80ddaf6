# timing probe (debug): tile scans stopped after stage 1 (load), 2 (items), 3 (scan, no flush)
set -e
for st in 2 3 0; do
  KMC_DEBUG_SCAN_STAGE=$st timeout -k 10 200 python bench.py --no-cpu-baseline --profile --steps 100 > gpurun_out/stage$st.json 2> gpurun_out/stage$st.err
done
