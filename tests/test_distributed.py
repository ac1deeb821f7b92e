"""N > 1 path of bench.py on the CPU: two ranks (gloo) shard a global batch of
ciphertext pairs, each with a replica of the context and relinearization key
(same seed), multiply their shard with the oracle engine, and rank 0 checks
that the gathered shards equal a single-process run of the whole batch and
that the max-over-ranks reduction is what `value` uses."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

PARAMS = dict(logn=10, nlimbs=3, nspecial=1, dnum=3, slots=8, q0_bits=50, qi_bits=40, p_bits=55, seed=77)
GLOBAL = 7  # pairs (uneven split on purpose)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run_batch(first, count):
    from hectr_amd import dist
    from hectr_amd.gpqhe import Engine
    e = Engine.oracle()
    e.init_params(**PARAMS)
    pk, sk, rlk = e.pk(), e.sk(), e.evk()
    e.keypair(pk, sk)
    e.genrlk(rlk, sk)
    L, n = e.L, e.n
    a = np.zeros(max(count, 1) * 2 * L * n, dtype=np.uint64)
    b = np.zeros_like(a)
    out = np.zeros(max(count, 1) * 2 * (L - 1) * n, dtype=np.uint64)
    dist.fill_pairs(e.lib, a.ctypes.data, b.ctypes.data, first, count, L, n)
    if count:
        e.lib.he_mul_rescale_batch(out.ctypes.data, a.ctypes.data, b.ctypes.data, count, L, ctypes.byref(rlk))
    e.exit()
    return out[:count * 2 * (L - 1) * n]


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    os.environ["OMP_NUM_THREADS"] = "1"
    from hectr_amd import dist
    try:
        r, w, _ = dist.init("gloo")
        first, stop = dist.shard(GLOBAL, r, w)
        out = _run_batch(first, stop - first)
        t = dist.max_over_ranks(float(r + 1))
        parts = dist.gather(out)
        dist.barrier()
        if r == 0:
            q.put((np.concatenate(parts), t))
        import torch.distributed as td
        td.destroy_process_group()
    except Exception as exc:  # pragma: no cover - surfaced to the parent
        q.put(exc)
        raise


def test_shard_bounds():
    from hectr_amd.dist import shard
    for count in (0, 1, 7, 256):
        for world in (1, 2, 3, 8):
            spans = [shard(count, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == count
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def test_two_rank_gloo_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
    if isinstance(res, Exception):
        raise res
    gathered, tmax = res
    assert tmax == 2.0
    single = _run_batch(0, GLOBAL)
    assert np.array_equal(gathered, single)


def test_bench_self_launch_two_ranks():
    """bench.py --gpus 2 without torchrun starts its own two rank processes
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), which meet over gloo, run the
    barrier and the max-over-ranks reduction the timed region uses, and rank 0
    prints one JSON line with n_gpus = 2."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["HECTR_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--launch-check"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    assert lines[0]["n_gpus"] == 2 and lines[0]["max_over_ranks"] == 2.0


def test_bench_self_launch_eight_ranks():
    """The driver's 8-GPU command shape without the engine: bench.py --gpus 8
    starts eight rank processes that meet over gloo (rendezvous on
    127.0.0.1), run the barrier and the max-over-ranks reduction, and rank 0
    prints one line with n_gpus = 8 and the largest rank's value."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["HECTR_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8", "--launch-check"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    assert lines[0]["n_gpus"] == 8 and lines[0]["max_over_ranks"] == 8.0


def test_bench_rejects_world_mismatch():
    """Under an external launcher, --gpus must equal WORLD_SIZE (a scale run
    must never silently time fewer ranks than it reports)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
