set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5r
timeout -k 10 800 python -u -m pytest tests/test_gpu_dist.py -x -v -m gpu --timeout 780 --timeout-method thread > gpurun_out/r5r/pytest.log 2>&1 || { tail -40 gpurun_out/r5r/pytest.log; exit 1; }
tail -3 gpurun_out/r5r/pytest.log
timeout -k 10 600 python bench.py --no-cpu --no-cstr --no-ntt > gpurun_out/r5r/bench.log 2>&1 || { tail -30 gpurun_out/r5r/bench.log; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r5r/bench.log") if l.startswith('{"metric"')][-1])
h = d["config5"]["hempc_gemv"]
print("headline", round(d["value"]), "c5", round(d["config5"]["value"]), "c5 hempc gemv", round(h["value"]), "gemv/s", round(h["us_per_gemv_per_gpu"], 1), "us")
for k, v in h["kernels"].items():
    print("  ", k, round(v["avg_us"], 1), round(v["us_per_gemv"], 2))
PY
