"""Host side of libkmc without a GPU: the library loads, exports every
declared symbol, struct layouts match the header, formats and validation."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from _kmc import DENSE, O, REPO, capi, engine, params

HEADER = os.path.join(REPO, "include", "kmc.h")


def test_library_builds_and_exports_header_symbols():
    build = __import__("_kmc").build
    lib = build.build()
    text = open(HEADER).read()
    names = set(re.findall(r"^\s*(?:const\s+)?[\w]+\**\s+\**(kmc_\w+)\s*\(", text, flags=re.M))
    assert len(names) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (kmc_\w+)$", out, flags=re.M))
    missing = names - exported
    assert not missing, f"declared in include/kmc.h but not exported: {missing}"
    engine.load_library()


def test_ctypes_layouts_match_header(tmp_path):
    src = tmp_path / "abi.c"
    fields = {
        "kmc_params": [f for f, _ in capi.Params._fields_],
        "kmc_obs": [f for f, _ in capi.Obs._fields_],
        "kmc_state_view": [f for f, _ in capi.StateView._fields_],
    }
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for st, fs in fields.items():
        lines.append(f'printf("{st} %zu\\n", sizeof({st}));')
        for f in fs:
            lines.append(f'printf("{st}.{f} %zu\\n", offsetof({st}, {f}));')
    lines.append("return 0;}")
    src.write_text("\n".join(lines))
    exe = tmp_path / "abi"
    subprocess.run(["gcc", "-O0", "-o", str(exe), str(src)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True).stdout.splitlines())
    for st, cls in (("kmc_params", capi.Params), ("kmc_obs", capi.Obs), ("kmc_state_view", capi.StateView)):
        assert int(got[st]) == C.sizeof(cls)
        for f, _ in cls._fields_:
            assert int(got[f"{st}.{f}"]) == getattr(cls, f).offset, f"{st}.{f}"


def test_params_default_match_reference_globals():
    L = engine.load_library()
    p = capi.Params()
    L.kmc_params_default(C.byref(p))
    q = capi.default_params()
    for f, _ in capi.Params._fields_:
        assert getattr(p, f) == getattr(q, f), f


def test_cpt_roundtrip_is_3_decimal(tmp_path):
    p = params(seed=4, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    o.step(200, want_hashes=False)
    st = o.get_state()
    path = str(tmp_path / "position.cpt")
    engine.host_write_cpt(p, st, path)
    back = engine.host_load_cpt(p, path)
    assert np.array_equal(back.a_int, st.a_int) and np.array_equal(back.b_int, st.b_int)
    assert np.array_equal(back.counters, st.counters) and back.step == st.step
    assert np.max(np.abs(back.ra - st.ra)) <= 0.0005 + 1e-9
    engine.host_write_cpt(p, back, path + "2")
    assert open(path, "rb").read() == open(path + "2", "rb").read()
    lines = open(path).read().splitlines()
    assert len(lines) == p.n_a * 17 + p.n_b * 12 + 6


def test_cpt_reader_rejects_truncated_file(tmp_path):
    p = params()
    st = engine.host_init_random(p)
    path = tmp_path / "position.cpt"
    engine.host_write_cpt(p, st, str(path))
    path.write_bytes(path.read_bytes()[: len(path.read_bytes()) // 2])
    with pytest.raises(engine.KmcError) as e:
        engine.host_load_cpt(p, str(path))
    assert e.value.code == -3
    with pytest.raises(engine.KmcError) as e:
        engine.host_load_cpt(p, str(tmp_path / "missing.cpt"))
    assert e.value.code == -2


def test_validate_rejects_inconsistent_links():
    p = params(seed=8, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    o.step(3000, want_hashes=False)
    st = o.get_state()
    assert engine.host_validate(p, st) == 0
    bound = np.flatnonzero(st.a_int[0] == 1)
    assert bound.size > 0
    bad = st.copy()
    bad.a_int[2, bound[0]] = 0  # status says bound, link says not
    assert engine.host_validate(p, bad) == -4
    bad = st.copy()
    bad.ra[3, 0] += 5.0  # receptor domain 2 off the [1][1] axis
    assert engine.host_validate(p, bad) == -8


def test_bond_line_format():
    p = params()
    rec = np.zeros(1, dtype=capi.OBS_DTYPE)[0]
    rec["t"], rec["bond_num_rl"], rec["bond_num_mono_cis"] = 50000.0, 38, 2
    rec["bond_num_cis"], rec["bond_num"], rec["cluster_size"], rec["protein_num_in_max_complex"] = 0, 40, 2.652, 4
    assert engine.bond_line(p, rec) == "      50000.000   38    2         0        40     2.652         4\n"


def test_exact_state_roundtrip_and_resume_on_oracle(tmp_path):
    # KMCSTAT1 keeps every bit; resuming the keyed oracle from it continues the
    # trajectory exactly (the 3-decimal position.cpt cannot, main.cpp:2208)
    p = params(seed=6, **DENSE)
    o = O.Oracle(p)
    o.init_placement()
    o.step(300, want_hashes=False)
    st = o.get_state()
    path = str(tmp_path / "state.kmc")
    engine.host_save_state(p, st, path)
    back = engine.host_load_state(p, path)
    for name in ("ra", "rb", "a_int", "b_int", "counters"):
        assert np.array_equal(getattr(back, name), getattr(st, name)), name
    assert back.step == st.step
    o.step(300, want_hashes=False)
    o2 = O.Oracle(p)
    o2.set_state(back)
    o2.step(300, want_hashes=False)
    assert o2.hash() == o.hash()


def test_exact_state_refuses_other_trajectory_and_corruption(tmp_path):
    p = params(seed=7)
    st = engine.host_init_random(p)
    path = tmp_path / "state.kmc"
    engine.host_save_state(p, st, str(path))
    other = params(seed=8)
    with pytest.raises(engine.KmcError) as e:
        engine.host_load_state(other, str(path))
    assert e.value.code == capi.ERR_ARG
    raw = bytearray(path.read_bytes())
    raw[200] ^= 1
    path.write_bytes(bytes(raw))
    with pytest.raises(engine.KmcError) as e:
        engine.host_load_state(p, str(path))
    assert e.value.code == capi.ERR_FORMAT
    path.write_bytes(bytes(raw[: len(raw) // 2]))
    with pytest.raises(engine.KmcError) as e:
        engine.host_load_state(p, str(path))
    assert e.value.code == capi.ERR_FORMAT
