#!/bin/bash
# Round-5 gemv on mixed prime sets: the rotation / gemv parity tests, the
# generic-path and windowed-path timings at the 60-bit set, the bench's gemv
# leg, and a kernel trace of the pipelined stream arrangement (overlap).
#   RUN=name bash scripts/gpu_r5b.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5b}
mkdir -p $OUT
K=${TESTS_K:-"evaluation or gemv or rot"}
timeout -k 10 900 python -u -m pytest tests/test_gpu_rotations.py tests/test_gpu_parity.py -x -v -m gpu -k "$K" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
if [ -z "$NO_TIME" ]; then
  GPQHE_GEMV_WIN=0 timeout -k 10 300 python scripts/gemv_time.py --set bench_d2 --count 8 > $OUT/gemv_generic_d2.json 2>&1 || { cat $OUT/gemv_generic_d2.json; exit 1; }
  timeout -k 10 300 python scripts/gemv_time.py --set bench_d2 --count 64 > $OUT/gemv_win_d2.json 2>&1 || { cat $OUT/gemv_win_d2.json; exit 1; }
  tail -1 $OUT/gemv_generic_d2.json | cut -c1-300; tail -1 $OUT/gemv_win_d2.json | cut -c1-300
fi
timeout -k 10 600 python bench.py --no-cpu --no-cstr --no-ntt --no-c5 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
python - $OUT/bench.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
print("headline", round(d["value"]), "60-bit", round(d.get("value_60bit", 0)))
g = d.get("gemv", {})
print("gemv", round(g.get("value", 0)), "us/gemv", round(g.get("us_per_gemv_per_gpu", 0), 2), "rot us", round(g.get("rot_batch", {}).get("us_per_rotation_per_gpu", 0), 2))
a = g.get("alt_primes", {})
print("gemv 60-bit", round(a.get("value", 0)), "us/gemv", round(a.get("us_per_gemv_per_gpu", 0), 2), "rot us", round(a.get("rot_batch", {}).get("us_per_rotation_per_gpu", 0), 2))
for k, v in a.get("kernels", {}).items():
    print(f"   {k:28s} {v['launches']:4d} x {v['avg_us']:8.1f} us  {v['us_per_gemv']:6.2f} us/gemv")
for k, v in g.get("kernels", {}).items():
    print(f" 51 {k:28s} {v['launches']:4d} x {v['avg_us']:8.1f} us  {v['us_per_gemv']:6.2f} us/gemv")
PY
if [ -n "$PIPE_KT" ]; then
  B="python bench.py --steps 10 --warmup 2 --no-cpu --no-cstr --no-ntt --no-c5 --no-gemv --alt-bits 0"
  GPQHE_SPLIT_PIPE=4 timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/kt_pipe4 -o kt_pipe4 --output-format csv -- $B > $OUT/kt_pipe4.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/kt_pipe0 -o kt_pipe0 --output-format csv -- $B > $OUT/kt_pipe0.log 2>&1 || exit 1
fi
