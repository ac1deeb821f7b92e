#!/bin/bash
# Writes tests/golden/cstr-mpc-100.bin: the reference's own plaintext CSTR-MPC
# loop (ctr_simulate, /root/reference/src/ctr.c:363-443) at N = 100 steps
# (horizon 10, src/ctr.c:376), run through harness/cstr_run.c on HECTR's
# unchanged sources built against SciPy's bundled OpenBLAS LAPACKE
# (`make -C harness ref-openblas`) -- independent of this
# repository's LAPACKE subset and CKKS engine.  Build container only (needs
# /root/reference); the GPU box reads the committed fixture.
#
# Check first that the same build reproduces the reference's committed
# 40-step run (tests/golden/cstr-mpc.bin, written by tests/hectr.c:751-756).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -C "$ROOT/harness" ref-openblas >/dev/null
EXE="$ROOT/oracle/_ref/openblas/cstr-run"
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
"$EXE" mpc 40 "$TMP/mpc40.bin" > "$TMP/log40" 2>&1
python3 - "$TMP/mpc40.bin" "$ROOT/tests/golden/cstr-mpc.bin" <<'PY'
import sys
import numpy as np
DT = np.dtype([("k", "<u4"), ("x", "<f8", 3), ("u", "<f8", 2)])
a, b = np.fromfile(sys.argv[1], dtype=DT), np.fromfile(sys.argv[2], dtype=DT)
rel = max(np.max(np.abs(a["x"] - b["x"]) / np.abs(b["x"])), np.max(np.abs(a["u"] - b["u"]) / np.abs(b["u"])))
assert len(a) == len(b) == 41 and rel < 1e-9, rel
print(f"40-step run vs the reference's cstr-mpc.bin: max rel {rel:.2e}")
PY
"$EXE" mpc 100 "$ROOT/tests/golden/cstr-mpc-100.bin" > "$TMP/log100" 2>&1
echo "wrote tests/golden/cstr-mpc-100.bin ($(stat -c %s "$ROOT/tests/golden/cstr-mpc-100.bin") bytes)"
