"""The CPU oracle (stream-RNG mode) against the REFERENCE's own golden traces.

tests/golden/ holds what the unmodified main.cpp computed (built and run by
tests/golden/make_golden.py through oracle/ref_interpose.cpp): per-step
hashes of the full state, bond counters, cluster statistics and RNG stream
positions, exact state dumps, and the position.cpt / bond.dat files the
reference wrote.  The oracle must reproduce them bit for bit; this is what
pins the oracle (and, through it, the GPU engine) to the reference.
"""
import gzip
import os
import shutil

import numpy as np
import pytest

from _kmc import GOLDEN, O, capi, engine, golden, scenarios, state_from_dump

SC = scenarios()


def _params(name):
    sc = SC[name]
    return capi.default_params(n_a=sc["n_a"], n_b=sc["n_b"], **sc["params"])


def _rows(g):
    return {int(s): i for i, s in enumerate(g["step"])}


def _check_rows(g, obs, hashes, first_step):
    """Compare oracle per-step output with every golden row in range."""
    idx = _rows(g)
    checked = 0
    for k in range(len(obs)):
        s = first_step + k
        if s not in idx:
            continue
        i = idx[s]
        assert int(hashes[k]) == int(g["hash"][i]), f"state hash differs at step {s}"
        o = obs[k]
        assert (o["bond_num_rl"], o["bond_num_mono_cis"], o["bond_num_cis"], o["bond_num"]) == (
            g["rl"][i], g["mono"][i], g["cis"][i], g["bond"][i]), f"bond counters differ at step {s}"
        assert o["cluster_size"] == g["cluster_size"][i], f"cluster_size differs at step {s}"
        assert o["protein_num_in_max_complex"] == g["maxc"][i]
        assert (o["tot_proteins_in_cluster"], o["tot_cluster_num"]) == (g["tot_prot"][i], g["tot_clu"][i])
        checked += 1
    return checked


def test_placement_matches_reference():
    """main.cpp:281-447 placement draws + geometry, step-0 state hash."""
    for name in ("default", "dense"):
        g = golden(name)
        o = O.Oracle(_params(name), rng_mode=O.RNG_STREAM, stream_t0=SC[name]["t0"])
        o.init_placement()
        assert g["step"][0] == 0
        assert o.hash() == int(g["hash"][0])
        assert o.stream_position == (int(g["clock"][0]), int(g["rand_calls"][0]))


def test_default_first_600_steps():
    g = golden("default")
    o = O.Oracle(_params("default"), rng_mode=O.RNG_STREAM, stream_t0=SC["default"]["t0"])
    o.init_placement()
    obs, h = o.step(600)
    assert _check_rows(g, obs, h, 1) == 600


@pytest.mark.parametrize("start,n", [(0, 400), (8000, 500), (15000, 300)])
def test_dense_windows(start, n):
    """Dense scenario: all reactions, complexes, multi-ligand alignment."""
    name = "dense"
    g = golden(name)
    p = _params(name)
    o = O.Oracle(p, rng_mode=O.RNG_STREAM, stream_t0=SC[name]["t0"])
    if start == 0:
        o.init_placement()
    else:
        st = state_from_dump(g[f"state_{start}"], p.n_a, p.n_b)
        i = _rows(g)[start]
        assert engine.state_hash(p, st) == int(g["hash"][i])
        o.set_state(st)
        o.set_stream(int(g["clock"][i]), int(g["rand_calls"][i]))
    obs, h = o.step(n)
    assert _check_rows(g, obs, h, start + 1) == n
    end = _rows(g)[start + n]
    assert o.stream_position == (int(g["clock"][end]), int(g["rand_calls"][end]))


def test_dense_window_covers_every_code_path():
    g = golden("dense")
    p = _params("dense")
    st = state_from_dump(g["state_8000"], p.n_a, p.n_b)
    i = _rows(g)[8000]
    o = O.Oracle(p, rng_mode=O.RNG_STREAM)
    o.set_state(st)
    o.set_stream(int(g["clock"][i]), int(g["rand_calls"][i]))
    o.step(500, want_hashes=False)
    ev = o.stats()
    for k in ("free_a", "dimer", "free_b", "complex", "multi", "reject", "rl", "snap_bond", "snap_cis"):
        assert ev[k] > 0, k


def test_resume_from_reference_checkpoint(tmp_path):
    """position.cpt written by the reference at step 5000 → continue."""
    p = _params("resume")
    g = golden("resume")
    cpt = tmp_path / "position.cpt"
    with gzip.open(os.path.join(GOLDEN, "dense_5000.cpt.gz"), "rb") as f:
        cpt.write_bytes(f.read())
    st = engine.host_load_cpt(p, str(cpt))
    assert st.step == 5000
    i = _rows(g)[5000]
    assert engine.state_hash(p, st) == int(g["hash"][i]), "cpt reader differs from main.cpp:226-270"
    o = O.Oracle(p, rng_mode=O.RNG_STREAM, stream_t0=SC["resume"]["t0"])
    o.set_state(st)
    obs, h = o.step(300)
    assert _check_rows(g, obs, h, 5001) == 300


@pytest.mark.parametrize("name,step", [("dense", 15000), ("dense", 20000), ("resume", 10000)])
def test_cpt_writer_matches_reference_bytes(tmp_path, name, step):
    p = _params(name)
    g = golden(name)
    st = state_from_dump(g[f"state_{step}"], p.n_a, p.n_b)
    out = tmp_path / "position.cpt"
    engine.host_write_cpt(p, st, str(out))
    with gzip.open(os.path.join(GOLDEN, f"{name}_{step}.cpt.gz"), "rb") as f:
        ref = f.read()
    assert out.read_bytes() == ref


@pytest.mark.parametrize("name", ["dense", "resume"])
def test_bond_dat_lines_match_reference(name):
    p = _params(name)
    g = golden(name)
    idx = _rows(g)
    lines = open(os.path.join(GOLDEN, f"{name}_bond.dat")).read().splitlines(keepends=True)
    assert lines
    for line in lines:
        step = int(round(float(line.split()[0]) / p.time_step))
        i = idx[step]
        rec = np.zeros(1, dtype=capi.OBS_DTYPE)[0]
        rec["step"], rec["t"] = step, step * p.time_step
        rec["bond_num_rl"], rec["bond_num_mono_cis"] = g["rl"][i], g["mono"][i]
        rec["bond_num_cis"], rec["bond_num"] = g["cis"][i], g["bond"][i]
        rec["cluster_size"], rec["protein_num_in_max_complex"] = g["cluster_size"][i], g["maxc"][i]
        assert engine.bond_line(p, rec) == line


@pytest.mark.skipif(not os.path.exists("/root/reference/main.cpp"), reason="reference source not present")
def test_reference_O0_equals_O2_with_portable_libm(tmp_path):
    """With libm interposed, -O0 and -O2 builds of main.cpp agree (they do not
    with glibc's sincos fusion — SURVEY.md §0.2 fact 5)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.dirname(O.REF_BIN) + "/..", "ref"], check=True)
    traces = []
    for exe in ("kmc_ref", "kmc_ref_O0"):
        d = tmp_path / exe
        d.mkdir()
        env = dict(os.environ, KMC_REF_T0="31337", KMC_REF_TRACE=str(d / "t.txt"), KMC_REF_SET="simu_step=60")
        subprocess.run([os.path.join(os.path.dirname(O.REF_BIN), exe)], cwd=d, env=env, check=True,
                       stdout=subprocess.DEVNULL)
        traces.append((d / "t.txt").read_text())
    assert traces[0] == traces[1]
