"""The N > 1 path on the product library: bench.py
--gpus 2 starts its own two rank processes before anything touches the GPU,
both on the one visible MI355X (gloo for the collectives: RCCL needs distinct
devices), each multiplies its shard of one global batch at the headline shape
(N=2^16, L=8, dnum=2, K=4) under one key (both ranks' key replicas come from
the same seed), and rank 0 compares the gathered shards word for word with a
single context's run of the whole global batch (bench.py --check-shards)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("streams", [1, 2])
def test_bench_two_ranks_shards_bit_exact(streams):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["HECTR_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch", "3", "--steps", "2", "--warmup",
           "1", "--streams", str(streams), "--no-cpu", "--no-cstr", "--no-ntt", "--no-c5", "--no-gemv", "--alt-bits", "0",
           "--check-shards"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 2 and d["config"]["batch_per_gpu"] == 3
    chk = d["shard_check"]
    assert chk["pairs"] == 6 and chk["ranks"] == 2
    assert chk["bit_exact"], chk


def test_bench_two_ranks_c5_and_gemv_shards_bit_exact():
    """The config-5 leg (N=2^17, L=12, dnum=3: 3 pairs per rank, split 1 + 2
    over the two sub-chunk streams), the gemv leg (he_gemv_batch at the
    headline shape with HECTR's 16 slots, 3 ciphertexts per rank) and config
    5 as a hempc batch (he_gemv_batch at N=2^17, L=12, 2 per rank) at two
    ranks: each leg's gathered output shards equal one context's run of its
    whole global batch, and the line reports every rank's time."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["HECTR_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch", "3", "--steps", "2", "--warmup",
           "1", "--no-cpu", "--no-cstr", "--no-ntt", "--alt-bits", "0", "--c5-batch", "3", "--gemv-batch", "3",
           "--c5-gemv-batch", "2", "--check-shards"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    d = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][0]
    assert d["shard_check"]["bit_exact"], d["shard_check"]
    assert len(d["rank_times_s"]) == 2
    c5, g = d["config5"], d["gemv"]
    assert c5["shard_check"] == {"pairs": 6, "ranks": 2, "bit_exact": True, "differing_pairs": []}, c5["shard_check"]
    assert g["shard_check"] == {"cts": 6, "ranks": 2, "bit_exact": True, "differing_cts": []}, g["shard_check"]
    assert len(c5["rank_times_s"]) == 2 and len(g["rank_times_s"]) == 2
    h = c5["hempc_gemv"]  # config 5 as a hempc batch: he_gemv_batch at N=2^17, L=12
    assert h["shard_check"] == {"cts": 4, "ranks": 2, "bit_exact": True, "differing_cts": []}, h["shard_check"]
    assert len(h["rank_times_s"]) == 2


def test_bench_two_ranks_default_legs():
    """The driver's N > 1 command shape with every leg bench.py runs there at
    its defaults (the 60-bit alternates of the headline, config 5 and the gemv
    leg included; NTT, CSTR and the CPU baseline are N = 1 only), small
    batches: one JSON line carrying each leg's value and both ranks' times."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["HECTR_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch", "3", "--steps", "2", "--warmup",
           "1", "--c5-batch", "2", "--gemv-batch", "3", "--c5-gemv-batch", "2"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["value_60bit"] > 0
    assert d["config5"]["value"] > 0 and d["config5"]["value_60bit"] > 0 and d["config5"]["hempc_gemv"]["value"] > 0
    g = d["gemv"]
    assert g["value"] > 0 and g["alt_primes"]["value"] > 0 and len(g["rank_times_s"]) == 2


@pytest.mark.timeout(900)
def test_bench_eight_ranks_shards_bit_exact():
    """Rehearsal of the driver's 8-GPU command shape on the one GPU of the test
    box: bench.py --gpus 8 starts eight rank processes (gloo for the
    collectives; every rank on device LOCAL_RANK mod device_count), each runs
    the headline, config 5, the gemv leg and config 5 as a hempc batch on its
    one-item shard (the headline's single pair takes the one-stream path),
    and rank 0 compares every leg's gathered shards with one context's run of
    the 8-item global batch.  The line carries eight rank times per leg."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["HECTR_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--batch", "1", "--steps", "2", "--warmup",
           "1", "--no-cpu", "--no-cstr", "--no-ntt", "--alt-bits", "0", "--c5-batch", "1", "--gemv-batch", "1",
           "--c5-gemv-batch", "1", "--check-shards"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=840, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 8 and len(d["rank_times_s"]) == 8
    assert d["shard_check"]["pairs"] == 8 and d["shard_check"]["bit_exact"], d["shard_check"]
    c5, g = d["config5"], d["gemv"]
    assert c5["shard_check"] == {"pairs": 8, "ranks": 8, "bit_exact": True, "differing_pairs": []}, c5["shard_check"]
    assert g["shard_check"] == {"cts": 8, "ranks": 8, "bit_exact": True, "differing_cts": []}, g["shard_check"]
    h = c5["hempc_gemv"]
    assert h["shard_check"] == {"cts": 8, "ranks": 8, "bit_exact": True, "differing_cts": []}, h["shard_check"]
    assert len(c5["rank_times_s"]) == 8 and len(g["rank_times_s"]) == 8 and len(h["rank_times_s"]) == 8
