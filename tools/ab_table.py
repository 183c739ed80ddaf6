"""Table of an A/B directory of round 4's first session (made by the former tools/gpu_ab3.sh; tools/pmc_ab.py prints its own): ms/step (steady, fresh) and
per-launch kernel means (µs) from each bench's --profile breakdown."""
import glob
import json
import sys

KS = ["k_cx_kill", "k_classify", "k_propose", "k_propose_free", "k_complex_heavy", "k_scan", "k_rec_scatter",
      "k_pair_scan", "k_col_exact", "k_col_rounds", "k_commit_rxn", "k_match", "k_diss_observe"]
print("variant".ljust(16), "ms/step fresh  " + " ".join(k[2:][:9].rjust(9) for k in KS))
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        print(f, "no result")
        continue
    b = {}
    for line in open(f[:-5] + ".err"):
        if line.startswith("{"):
            b = json.loads(line).get("per_launch_ms", b)
    if f.endswith("evolve.json"):
        continue
    print(f.split("/")[-1][:-5].ljust(16), f"{d['ms_per_step']:.4f} {d['config'].get('ms_per_step_fresh') or 0:.4f}",
          " ".join(f"{b.get(k, 0) * 1e3:9.1f}" for k in KS))
