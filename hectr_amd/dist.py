"""Ciphertext-batch sharding across GPUs.

One process per GPU (torch.distributed; backend "nccl" = RCCL on ROCm, "gloo"
for CPU tests).  Ciphertexts are independent, so there is no data-path
collective: every rank holds a replica of the context and keys generated from
one seed (bench.py KEY_SEED), so all ranks work under one key, and processes
the pairs whose global index falls in its shard (fill_pairs: pair g from seeds
of g alone).  bench.py --check-shards gathers the product's output shards and
compares them with one context's run of the whole global batch
(tests/test_gpu_dist.py).  Collectives
carry only the barrier, the max-over-ranks time and (tests) result gathers.
"""
from __future__ import annotations

import os

import numpy as np


def env():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str):
    import torch.distributed as dist
    rank, world, local = env()
    if world > 1 and not dist.is_initialized():
        kw = {}
        if backend == "nccl":
            import torch
            kw["device_id"] = torch.device("cuda", local % max(1, torch.cuda.device_count()))
        import datetime
        # bounded rendezvous / collectives: a rank that never arrives ends the
        # job instead of hanging it (bench.py's launcher also polls its ranks)
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=300), **kw)
    return rank, world, local


def barrier():
    import torch.distributed as dist
    if dist.is_initialized():
        dist.barrier()


def max_over_ranks(x: float, device="cpu") -> float:
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_values(x: float, device="cpu") -> list:
    """Every rank's value of x, in rank order (one all_gather)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return [x]
    t = torch.tensor([x], dtype=torch.float64, device=device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [float(p.item()) for p in parts]


def shard(count: int, rank: int, world: int):
    """Contiguous shard [start, stop) of `count` global items for `rank`."""
    base, extra = divmod(count, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def fill_pairs(lib, a_ptr, b_ptr, first: int, count: int, nlimbs: int, n: int, seed: int = 1000):
    """Inputs of global pairs [first, first + count): pair g is generated from
    seeds (seed + 2g, seed + 2g + 1), so any sharding of a global batch sees
    the same ciphertexts.  Pointers address [count][2][nlimbs][n] words."""
    words = 2 * nlimbs * n
    for i in range(count):
        g = first + i
        lib.poly_fill_uniform(a_ptr + 8 * i * words, 2, nlimbs, seed + 2 * g)
        lib.poly_fill_uniform(b_ptr + 8 * i * words, 2, nlimbs, seed + 2 * g + 1)


def gather(arr: np.ndarray):
    """Rank 0 receives every rank's array (CPU tensors, gloo)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return [arr]
    t = torch.from_numpy(arr.view(np.int64).copy())
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(dist.get_world_size())]
    dist.all_gather(sizes, torch.tensor([t.numel()], dtype=torch.int64))
    sizes = [int(s.item()) for s in sizes]
    big = max(sizes)
    padded = torch.zeros(big, dtype=torch.int64)
    padded[:t.numel()] = t
    out = [torch.zeros(big, dtype=torch.int64) for _ in sizes]
    dist.all_gather(out, padded)
    return [o[:k].numpy().view(arr.dtype) for o, k in zip(out, sizes)]
