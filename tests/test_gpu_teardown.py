"""Engine teardown on MI355X: hectx_exit releases every HIP object the
engine created (the second sub-chunk stream of he_mul_rescale_batch and its
fork / join events, the decode and profiling events, the context's own
stream), so nothing is left for the runtime's or a profiler's exit handlers
(round 5 recorded a SIGSEGV in __cxa_finalize after a two-stream run under
rocprofv3).  A child process runs the two-stream headline op, hectx_exit, a
second context on one stream, hectx_exit, and must exit with status 0; the
two contexts' outputs (same keys, same inputs) must be equal."""
import pytest

from tests.test_gpu_gemv_shapes import run_worker

pytestmark = pytest.mark.gpu


def test_two_stream_teardown_clean_exit():
    assert run_worker("teardown", {}) == {"equal": True}
