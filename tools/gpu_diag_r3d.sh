#!/bin/bash
# Round-3 diagnostic call: the C3 evolution with the one-lane complex
# alignment and with the wave one (same bond counts expected), then the
# steady-state parity windows.
set -euo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r3d}
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd "$root"
KMC_CX_SERIAL=1 timeout -k 10 150 python -u tools/diag_evolve.py C3 10000 1000 > "$out/serial.log" 2>&1
timeout -k 10 150 python -u tools/diag_evolve.py C3 10000 1000 > "$out/wave.log" 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_steady.py -x -v -s --timeout 600 --timeout-method thread > "$out/steady.log" 2>&1
echo "diag done"
