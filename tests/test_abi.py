"""The C ABI boundary (include/gpqhe.h): every declared function is exported
by both libgpqhe.so (product) and the oracle, the header compiles as pure C
under HECTR's warning flags (reference Makefile:21) and is include-guarded
(tests/hectr.c:22-23 includes it twice), object sizes are complete, and the
product library refuses to run without a GPU (no CPU fallback).  CPU only:
no compute calls on the product library."""
import ctypes
import os
import re
import subprocess
import sys

import pytest

from hectr_amd import gpqhe

ROOT = gpqhe.ROOT
HEADER = ROOT / "include" / "gpqhe.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"#define[^\n]*(\\\n[^\n]*)*", "", text)
    names = set(re.findall(r"\b([a-z_][a-z0-9_]*)\s*\(", text))
    keywords = {"sizeof", "if", "for", "while", "return"}
    return sorted(n for n in names - keywords if n.startswith(("he_", "hectx_", "poly_", "gpqhe_")))


def exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", str(lib)], capture_output=True, text=True, check=True)
    return {line.split()[-1] for line in out.stdout.splitlines()}


def test_binding_covers_header():
    assert set(declared_functions()) == set(gpqhe.EXPORTED)


@pytest.mark.parametrize("lib", [gpqhe.PRODUCT_LIB, gpqhe.ORACLE_LIB])
def test_library_exports_every_symbol(lib):
    assert lib.exists(), f"{lib} not built (run __graft_entry__.build())"
    missing = set(declared_functions()) - exported(lib)
    assert not missing, missing


def test_product_loads_and_links_hip():
    lib = ctypes.CDLL(str(gpqhe.PRODUCT_LIB), mode=ctypes.RTLD_LOCAL)
    assert hasattr(lib, "he_gemv")
    ldd = subprocess.run(["ldd", str(gpqhe.PRODUCT_LIB)], capture_output=True, text=True).stdout
    assert "libamdhip64" in ldd


def test_header_is_pure_c_and_guarded(tmp_path):
    src = tmp_path / "t.c"
    src.write_text(
        '#include "gpqhe.h"\n#include "gpqhe.h"\n'
        "_Static_assert(sizeof(he_ct_t) == 48, \"ct\");\n"
        "int main(void) { MPI q = mpi_set_ui(NULL, 1); mpi_lshift(q, q, 109);\n"
        "  he_ct_t ct; he_evk_t rk[16]; (void)ct; (void)rk; mpi_release(q); return 0; }\n")
    cmd = ["gcc", "-std=c11", "-Wall", "-Wextra", "-Wpedantic", "-Wshadow", "-Werror", "-I", str(ROOT / "include"),
           "-c", str(src), "-o", str(tmp_path / "t.o")]
    subprocess.run(cmd, check=True)
    # the forwarding header at HECTR's include path resolves to the same ABI
    src2 = tmp_path / "u.c"
    src2.write_text('#include "../GPQHE/src/gpqhe.h"\nint main(void){ return (int)sizeof(poly_mpi_t) - 48; }\n')
    # (HECTR's src/hectr.h:35 includes it relative to a sibling directory)
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", str(ROOT / "libpmu"), "-c", str(src2), "-o",
                    str(tmp_path / "u.o")], check=True)


def test_pmu_header_compiles(tmp_path):
    src = tmp_path / "p.c"
    src.write_text('#include "pmu.h"\nint main(void){ TEST_BEGIN(); int s = 0;\n'
                   'TEST_DO("x");{ s += 1; }TEST_DONE(); TEST_END(); return s - 1; }\n')
    subprocess.run(["gcc", "-std=gnu11", "-Wall", "-Wextra", "-Werror", "-I", str(ROOT / "libpmu"), str(src), "-o",
                    str(tmp_path / "p")], check=True)
    assert subprocess.run([str(tmp_path / "p")], capture_output=True).returncode == 0


def test_product_refuses_without_gpu():
    """On a host with no HIP device the product aborts with a message instead
    of silently computing on the CPU (skipped where a GPU is visible)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible here")
    code = ("import sys; sys.path.insert(0, %r); from hectr_amd.gpqhe import Engine; "
            "e = Engine.product(); e.init(12, 109, 16, 50)" % str(ROOT))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "no HIP device" in r.stderr
