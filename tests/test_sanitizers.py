"""Host code under AddressSanitizer + UBSan: the oracle and
libkmc's host side (kmc_io.cpp: the position.cpt tokenizer, the KMCSTAT1
reader, the writers, the placement generator) built by `make -C oracle asan`
and driven by oracle/asan_driver.cpp over the reference-written checkpoints,
their truncations and corruptions, a dense oracle run with exact-state round
trips, and refused foreign / corrupt KMCSTAT1 files."""
import gzip
import os
import subprocess

from _kmc import GOLDEN, REPO


def test_host_code_clean_under_asan_ubsan(tmp_path):
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "asan"], check=True)
    cpts = []
    for name in ("dense_5000", "dense_20000"):
        p = tmp_path / f"{name}.cpt"
        p.write_bytes(gzip.open(os.path.join(GOLDEN, name + ".cpt.gz")).read())
        cpts.append(str(p))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(REPO, "oracle", "_build", "asan_driver"), str(tmp_path), *cpts],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "asan_driver ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
