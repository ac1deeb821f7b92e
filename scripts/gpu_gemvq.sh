set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gemvq
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_cstr.py tests/test_gpu_hectr_caller.py tests/test_gpu_parity.py -k "gemv or cstr or hectr or caller" > gpurun_out/gemvq/tests.log 2>&1 || { tail -30 gpurun_out/gemvq/tests.log; exit 1; }
tail -3 gpurun_out/gemvq/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" && \
timeout -k 10 200 python scripts/cstr_prof.py 300 > gpurun_out/gemvq/on.log 2>&1 && \
GPQHE_DEFER_GEMV=0 timeout -k 10 200 python scripts/cstr_prof.py 300 > gpurun_out/gemvq/off.log 2>&1 && \
timeout -k 10 200 python scripts/cstr_prof.py 300 > gpurun_out/gemvq/on2.log 2>&1 && \
head -1 gpurun_out/gemvq/on.log gpurun_out/gemvq/off.log gpurun_out/gemvq/on2.log
