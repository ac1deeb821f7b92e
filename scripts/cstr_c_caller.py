"""Closed-loop time of HECTR's unchanged C harness (test-hectr cstr-hempc,
40 steps, its own pmu timer) on the product library, with the deferral
switches given as KEY=VALUE arguments; repeated runs, median reported."""
import os
import statistics
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_hectr_caller import ROOT, run_cstr_hempc  # noqa: E402

env = dict(a.split("=", 1) for a in sys.argv[1:])
reps = int(env.pop("REPS", "5"))
ms = []
for i in range(reps):
    with tempfile.TemporaryDirectory() as d:
        _, t = run_cstr_hempc(os.path.join(ROOT, "hectr_amd", "lib"), Path(d), env, timeout=120)
        ms.append(t)
print(f"test-hectr cstr-hempc {env or 'default'}: closed loop {statistics.median(ms):.2f} ms / 40 steps "
      f"(runs {', '.join(f'{m:.2f}' for m in ms)})")
