"""N1 acceptance (BASELINE north_star: "src/hempc.c links unchanged and the
cstr-hempc test runs as-is"): HECTR's own sources, compiled where they lie
under /root/reference with the reference's flags (Makefile:21) against this
repository's include/gpqhe.h, libpmu/pmu.h and the harness LAPACKE subset,
linked with the reference's line (tests/Makefile:25, -lgcrypt dropped: MPI
comes from gpqhe.h), then `test-hectr cstr-hempc` run unchanged.

Here (CPU container) the binary runs on the CPU oracle (config 1 plumbing:
HECTR's own n=4096 / q=2^109 and N=2^13, L=4 through the GPQHE_LOGN /
GPQHE_NLIMBS override); tests/test_gpu_hectr_caller.py runs the same binary
on the MI355X library.  Nothing from the reference is copied into the repo:
the build outputs go to oracle/_ref/ (git-ignored).
"""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
OUT = os.path.join(ROOT, "oracle", "_ref")
DT = np.dtype([("k", "<u4"), ("x", "<f8", 3), ("u", "<f8", 2)])  # tests/hectr.c:812-817

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")),
                                reason="reference sources not present (GPU box)")


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "harness"), "hectr", f"REF={REF}"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout + r.stderr


def test_reference_sources_compile_unchanged(built):
    """-Wall -Wextra -Wpedantic: no diagnostic points into this repository's
    headers (the reference's own warnings, e.g. mpc.c's missing <stdlib.h>,
    are its own)."""
    diags = open(os.path.join(OUT, "libhectr.warnings")).read() + open(os.path.join(OUT, "test-hectr.warnings")).read()
    ours = [l for l in diags.splitlines() if re.search(r"(gpqhe\.h|pmu\.h|lapacke\.h|lapacke_subset)", l)]
    assert not ours, "\n".join(ours)
    for f in ("libhectr.so", "test-hectr"):
        assert os.path.exists(os.path.join(OUT, f))


def _nm(path, flag):
    r = subprocess.run(["nm", "-D", flag, path], capture_output=True, text=True, check=True)
    return {l.split()[-1] for l in r.stdout.splitlines() if l.strip()}


def test_every_gpqhe_symbol_resolves(built):
    want = set()
    for f in ("libhectr.so", "test-hectr"):
        want |= {s for s in _nm(os.path.join(OUT, f), "--undefined-only") if re.match(r"(he_|hectx_|gpqhe_)", s)}
    assert {"hectx_init", "he_gemv", "he_enc_pk", "he_dcd", "gpqhe_mpi_lshift"} <= want
    for lib in (os.path.join(ROOT, "hectr_amd", "lib", "libgpqhe.so"), os.path.join(ROOT, "oracle", "libgpqhe_oracle.so")):
        have = _nm(lib, "--defined-only")
        assert want <= have, f"{lib} lacks {sorted(want - have)}"


def run_cstr_hempc(libdir, tmp_path, env_extra=None, timeout=600):
    """./test-hectr cstr-hempc in a scratch directory (it writes
    results/cstr-hempc.bin relative to the working directory); returns the
    41 records and the harness's own closed-loop time (ms, pmu.h)."""
    (tmp_path / "results").mkdir(parents=True, exist_ok=True)
    env = dict(os.environ, LD_LIBRARY_PATH=libdir, GPQHE_SEED="5")
    env.update(env_extra or {})
    r = subprocess.run([os.path.join(OUT, "test-hectr"), "cstr-hempc"], cwd=tmp_path, env=env, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    m = re.search(r"closed-loop simulate\s+([0-9.]+) ms", r.stdout + r.stderr)
    rec = np.fromfile(tmp_path / "results" / "cstr-hempc.bin", dtype=DT)
    return rec, float(m.group(1)) if m else None


def compare_to_mpc(rec):
    ref = np.fromfile(os.path.join(ROOT, "tests", "golden", "cstr-mpc.bin"), dtype=DT)
    assert len(rec) == len(ref) == 41
    assert np.array_equal(rec["k"], ref["k"])
    return max(np.max(np.abs(rec["x"] - ref["x"]) / np.abs(ref["x"])),
               np.max(np.abs(rec["u"] - ref["u"]) / np.abs(ref["u"])))


@pytest.mark.parametrize("env", [{}, {"GPQHE_LOGN": "13", "GPQHE_NLIMBS": "4"}], ids=["ref_n4096", "config1_n8192_l4"])
def test_cstr_hempc_unchanged_on_cpu_oracle(built, tmp_path, env):
    """The unchanged harness's encrypted loop over the CPU oracle matches the
    reference's plaintext run (tests/results/cstr-mpc.bin) within 1e-6
    relative (north_star tolerance; the reference's own hempc-vs-mpc gap is
    1.15e-11)."""
    rec, _ = run_cstr_hempc(os.path.join(OUT, "cpu"), tmp_path, env)
    assert compare_to_mpc(rec) < 1e-6
