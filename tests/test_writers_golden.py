"""The trajectory / log writers against the files the REFERENCE wrote.

tests/golden/<scenario>_{test.gro,cluster.log,parameter.log}.gz are the
unmodified main.cpp's own outputs (tests/golden/make_golden.py).  They are
regenerated here from the reference's exact state dumps:

  test.gro     main.cpp:2258-2287 — one frame per output step, from the state
               after that step (dumps at s, or the dump at s-1 advanced one
               step by the stream-mode oracle)
  cluster.log  main.cpp:2291-2305 — one block per output step, the BFS rows of
               that step after the multi-ligand shuffles (dump at s-1 + one
               oracle step in stream mode, the reference's own RNG stream)
  parameter.log main.cpp:178-205

and must be byte-identical to the reference's files.
"""
import gzip
import os

import pytest

from _kmc import GOLDEN, O, capi, engine, golden, scenarios, state_from_dump

SC = scenarios()
OUT_STEPS = {"dense": [5000, 10000, 15000, 20000], "resume": [10000]}


def _params(name):
    sc = SC[name]
    return capi.default_params(n_a=sc["n_a"], n_b=sc["n_b"], **sc["params"])


def _ref(name, fn):
    return gzip.open(os.path.join(GOLDEN, f"{name}_{fn}.gz")).read()


def _step_from_dump(name, s):
    """Stream-mode oracle at the reference's state of step s-1, advanced to s."""
    g = golden(name)
    p = _params(name)
    row = {int(x): i for i, x in enumerate(g["step"])}[s - 1]
    o = O.Oracle(p, rng_mode=O.RNG_STREAM)
    o.set_state(state_from_dump(g[f"state_{s - 1}"], p.n_a, p.n_b))
    o.set_stream(int(g["clock"][row]), int(g["rand_calls"][row]))
    o.step(1, want_hashes=False)
    assert o.hash() == int(g["hash"][{int(x): i for i, x in enumerate(g["step"])}[s]])
    return o


@pytest.mark.parametrize("name", ["dense", "resume"])
def test_test_gro_matches_reference_bytes(tmp_path, name):
    p = _params(name)
    g = golden(name)
    out = tmp_path / "test.gro"
    for s in OUT_STEPS[name]:
        key = f"state_{s}"
        st = state_from_dump(g[key], p.n_a, p.n_b) if key in g else _step_from_dump(name, s).get_state()
        engine.append_gro(p, st, str(out))
    assert out.read_bytes() == _ref(name, "test.gro")


@pytest.mark.parametrize("name", ["dense", "resume"])
def test_cluster_log_matches_reference_bytes(tmp_path, name):
    p = _params(name)
    out = tmp_path / "cluster.log"
    for s in OUT_STEPS[name]:
        row, mem = _step_from_dump(name, s).clusters()
        engine.append_cluster_log(p, s, row, mem, str(out))
    ref = _ref(name, "cluster.log")
    assert out.read_bytes() == ref
    assert ref.count(b"\n") > 4 * len(OUT_STEPS[name])


@pytest.mark.parametrize("name", ["dense", "resume"])
def test_parameter_log_matches_reference_bytes(tmp_path, name):
    out = tmp_path / "parameter.log"
    engine.write_parameter_log(_params(name), str(out))
    assert out.read_bytes() == _ref(name, "parameter.log")
