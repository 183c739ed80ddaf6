"""C5 steady-state window against the keyed oracle (evidence run, not part of
the GPU test suite: the CPU oracle takes ~40 s per step at 1e7 particles).

The GPU evolves C5 (1e7 particles, reference physics) for EVOLVE steps, the
exact state it reached is handed to the cell-list oracle, and WINDOW more
steps are compared bit for bit (every bond.dat record, full-state hash) —
tests/test_gpu_steady.py's procedure at the largest benchmark size.
  python -u tools/c5_window.py [evolve] [window]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))  # oracle/oracle.py, as tests/conftest.py does
from _kmc import O, engine, workloads  # noqa: E402


def main():
    evolve = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    window = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    p = workloads.params("C5", seed=3)
    sim = engine.Simulation(p)
    sim.set_state(engine.host_init_random(p))
    t = time.time()
    done = 0
    while done < evolve:
        k = min(2000, evolve - done)
        ob = sim.step(k)
        done += k
        print(f"evolved {done}/{evolve}: bond_num {int(ob[-1]['bond_num'])} ({time.time() - t:.0f}s)", flush=True)
    st = sim.get_state()
    obs, hashes = [], []
    for _ in range(window):  # one step at a time: every step's full-state hash
        obs.append(sim.step(1)[0])
        hashes.append(engine.state_hash(p, sim.get_state()))
    h = hashes[-1]
    sim.close()
    o = O.Oracle(p, nbmode=O.NB_CELLS)
    o.set_state(st)
    print(f"oracle loaded ({time.time() - t:.0f}s)", flush=True)
    ok = True
    for s in range(window):
        obs_o, hs_o = o.step(1)
        same = obs[s] == obs_o[0]
        hsame = hashes[s] == int(hs_o[0])
        ok &= bool(same) and hsame
        print(f"step {evolve + s + 1}: {'equal' if same else 'DIFFERENT'} bond.dat record {obs[s]} "
              f"(every field), state hash gpu {hashes[s]:x} oracle {int(hs_o[0]):x}: "
              f"{'equal' if hsame else 'DIFFERENT'} ({time.time() - t:.0f}s)", flush=True)
    hs = o.hash()
    print(f"state hash gpu {h:x} oracle {hs:x}: {'equal' if h == hs else 'DIFFERENT'}", flush=True)
    print("window events", o.stats(), flush=True)
    sys.exit(0 if ok and h == hs else 1)


if __name__ == "__main__":
    main()
