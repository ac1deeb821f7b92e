#!/usr/bin/env python3
"""bench.py - headline benchmark of the MI355X CKKS engine.

Metric (BASELINE.json): ct x ct + relinearization (+ rescale) per second at
N = 2^16, L = 8 RNS primes (configs[2]: batch = 256 ciphertext pairs per GPU,
one step = one batch through he_mul_rescale_batch).  Inputs are synthetic
random-residue ciphertexts already resident in HBM (poly_fill_uniform,
splitmix64 streams); the relinearization key is a real key (he_genrlk).

Multi-GPU: one process per GPU (torch.distributed, RCCL), each rank
multiplies its own batch (independent ciphertexts: no data-path
collective); the collective is only the barrier / max-time reduction.
`value` = pairs processed by all ranks / max rank time ("scaling": "weak").

Also reported on rank 0:
  roofline      - for the dominant kernel, algorithmic bytes per launch /
                  its average launch duration (HIP events on the engine
                  stream, same shapes as inside the step), vs 8 TB/s;
  cpu_baseline  - the CPU restatement (oracle/, "port") timed on this host
                  on a bounded sample of the same op;
  op_roofline   - the whole op against its algorithmic bytes (24.4 MB/op).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--logn", type=int, default=16)
    ap.add_argument("--nlimbs", type=int, default=8)
    ap.add_argument("--dnum", type=int, default=2,
                    help="key-switch digits (2: fastest measured at L=8, see DESIGN.md; L: one limb per digit)")
    ap.add_argument("--nspecial", type=int, default=0, help="special primes K (default: enough for P > digit)")
    ap.add_argument("--p-bits", type=int, default=51, help="special prime size in bits")
    ap.add_argument("--q0-bits", type=int, default=51, help="first prime size in bits")
    ap.add_argument("--alt-bits", type=int, default=60,
                    help="also time q0/special primes of this size (conventional CKKS sizes; 0: skip)")
    ap.add_argument("--no-cstr", action="store_true", help="skip the encrypted CSTR loop (config 4)")
    ap.add_argument("--cstr-steps", type=int, default=100)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-ntt", action="store_true", help="skip the NTT roundtrip leg (config 2)")
    ap.add_argument("--ntt-polys", type=int, default=1024)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample duration")
    return ap.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    from hectr_amd import dist as hdist
    from hectr_amd.gpqhe import Engine

    rank, world, local = hdist.env()
    # one process per GPU; the modulus only matters for rehearsals with more
    # ranks than GPUs (HECTR_DIST_BACKEND=gloo: RCCL needs distinct devices)
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    backend = os.environ.get("HECTR_DIST_BACKEND", "nccl")
    hdist.init(backend)
    red_dev = "cuda" if backend == "nccl" else "cpu"
    barrier = hdist.barrier

    L, logn, B = args.nlimbs, args.logn, args.batch
    n = 1 << logn
    dnum = args.dnum or L
    K = args.nspecial or special_primes(L, dnum, q0_bits=args.q0_bits, p_bits=args.p_bits)
    eng = Engine.product()
    eng.init_params(logn=logn, nlimbs=L, dnum=dnum, nspecial=K, slots=64, q0_bits=args.q0_bits, qi_bits=50,
                    p_bits=args.p_bits, seed=1000 + rank)
    stream = torch.cuda.Stream()
    eng.lib.gpqhe_set_stream(ctypes.c_void_p(stream.cuda_stream))
    pk, sk, rlk = eng.pk(), eng.sk(), eng.evk()
    eng.keypair(pk, sk)
    eng.genrlk(rlk, sk)
    in_words, out_words = 2 * L * n, 2 * (L - 1) * n
    a = torch.empty(B * in_words, dtype=torch.int64, device="cuda")
    b = torch.empty_like(a)
    out = torch.empty(B * out_words, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    # global pairs [rank B, (rank + 1) B): each rank multiplies its own shard
    hdist.fill_pairs(eng.lib, a.data_ptr(), b.data_ptr(), rank * B, B, L, n)
    eng.sync()

    def step():
        eng.lib.he_mul_rescale_batch(out.data_ptr(), a.data_ptr(), b.data_ptr(), B, L, ctypes.byref(rlk))

    for _ in range(args.warmup):
        step()
    eng.sync()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    eng.sync()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    ev_s = ev0.elapsed_time(ev1) / 1e3
    elapsed = hdist.max_over_ranks(elapsed, device=red_dev)
    ops = world * B * args.steps
    value = ops / elapsed
    ms_per_step = 1e3 * elapsed / args.steps

    # algorithmic bytes per op: 2 ct in, 1 ct out at L-1, rlk amortised over the batch
    evk_bytes = 2 * eng.info.dnum * (L + K) * n * 8
    alg_bytes = (2 * in_words + out_words) * 8 + evk_bytes / B

    # instrumented pass (same steps): per-kernel device time from HIP events on
    # the engine stream, algorithmic bytes per launch from the library
    eng.prof_enable(True)
    ti0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.sync()
    ti1 = time.perf_counter()
    stats = eng.prof_collect()
    eng.prof_enable(False)

    result = None
    if rank == 0:
        dom_name = max(stats, key=lambda k: stats[k][1])
        launches, tot_us, nbytes = stats[dom_name]
        achieved = nbytes / tot_us / 1e3  # GB/s
        workload = (f"ct x ct mult + relin + rescale, N=2^{logn}, L={L}, K={K}, dnum={eng.info.dnum}, "
                    f"primes {args.q0_bits}/50/{args.p_bits} bits, batch={B} pairs per GPU")
        traffic, src = pmc_traffic(dom_name, workload, tot_us / launches)
        dom = {"bound": "hbm", "kernel": dom_name, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
               "avg_launch_us": tot_us / launches, "alg_bytes_per_launch": nbytes / launches,
               "share_of_step": tot_us / (1e6 * (ti1 - ti0))}
        kernels = {k: {"launches": v[0], "avg_us": v[1] / v[0], "share": v[1] / (1e6 * (ti1 - ti0)),
                       "GBs": v[2] / v[1] / 1e3} for k, v in sorted(stats.items(), key=lambda kv: -kv[1][1])}
        result = {
            "metric": "ct×ct+relin/sec at N=2^16, L=8 RNS primes; encrypted CSTR-MPC steps/sec",
            "value": value,
            "unit": "ct-mult/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic random-residue ciphertexts (splitmix64), real relinearization key",
            "config": {"workload": workload,
                       "batch_per_gpu": B, "logn": logn, "nlimbs": L, "nspecial": K,
                       "dnum": eng.info.dnum, "prime_bits": {"q0": args.q0_bits, "qi": 50, "p": args.p_bits},
                       "parallelism": f"batch-sharded x{world}"},
            "event_s_rank0": ev_s,
            "op_roofline": {"alg_bytes_per_op": alg_bytes,
                            "achieved_GBs": alg_bytes * value / world / 1e9,
                            "frac": alg_bytes * value / world / 1e9 / HBM_PEAK_GBS},
            "roofline": dom,
            "kernels": kernels,
            "instrumented_ms_per_step": 1e3 * (ti1 - ti0) / args.steps,
        }
    if rank == 0 and not args.no_ntt:
        result["ntt_roundtrip"] = ntt_roundtrip(eng, stream, logn, L, args.ntt_polys)
    if rank == 0 and world == 1 and args.alt_bits and args.alt_bits != args.q0_bits:
        eng.exit()
        result["alt_primes"] = alt_rate(args, stream, L, logn, B, dnum)
    barrier()
    if rank == 0 and not args.no_cstr:
        eng.exit()
        result["cstr"] = cstr_loop(args.cstr_steps)
    if rank == 0 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(args, logn, L, dnum)
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()
    return result


def pmc_traffic(kernel, workload, avg_us):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/*_pmc.json, written by scripts/prof_summary.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this same workload, with
    the gfx950 FETCH_SIZE x2 correction).  A profile whose mean launch time is
    not within 0.7-1.4x of this run's (`avg_us`) was taken with another chunk
    size, so its bytes per launch do not apply and it is skipped.  (None, None)
    when no profile of this workload exists: PMC counters cannot be read from
    inside the timed run."""
    import glob
    import re
    def order(f):  # profiles/r<round>_v<version>_pmc.json, newest first
        m = re.search(r"r(\d+)_v(\d+)_pmc", os.path.basename(f))
        return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")), key=order, reverse=True)
    for f in files:
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("meta", {}).get("bench_workload") != workload:
            continue
        base, _, tag = kernel.partition("<")
        flag = {"fwd>": "false>", "inv>": "true>"}.get(tag)
        for name, e in d.get("kernels", {}).items():
            if name.split("<")[0] != base or "hbm_bytes" not in e:
                continue
            if flag and not name.endswith(flag):
                continue
            if not 0.7 <= e.get("mean_us", avg_us) / avg_us <= 1.4:
                continue
            return e["hbm_bytes"], os.path.relpath(f, ROOT) + ":" + name
    return None, None


def alt_rate(args, stream, L, logn, B, dnum):
    """The same op and batch with q0 and the special primes at args.alt_bits
    (60: the conventional CKKS sizes).  Limbs of 51 bits and more take the
    64-bit integer butterflies instead of the FP64 ones."""
    from hectr_amd.gpqhe import Engine
    bits = args.alt_bits
    K = special_primes(L, dnum, q0_bits=bits, p_bits=bits)
    eng = Engine.product()
    eng.init_params(logn=logn, nlimbs=L, dnum=dnum, nspecial=K, slots=64, q0_bits=bits, qi_bits=50, p_bits=bits,
                    seed=1000)
    eng.lib.gpqhe_set_stream(ctypes.c_void_p(stream.cuda_stream))
    pk, sk, rlk = eng.pk(), eng.sk(), eng.evk()
    eng.keypair(pk, sk)
    eng.genrlk(rlk, sk)
    import torch
    n = 1 << logn
    a = torch.empty(B * 2 * L * n, dtype=torch.int64, device="cuda")
    b = torch.empty_like(a)
    out = torch.empty(B * 2 * (L - 1) * n, dtype=torch.int64, device="cuda")
    from hectr_amd import dist as hdist
    hdist.fill_pairs(eng.lib, a.data_ptr(), b.data_ptr(), 0, B, L, n)
    for _ in range(max(1, args.warmup)):
        eng.lib.he_mul_rescale_batch(out.data_ptr(), a.data_ptr(), b.data_ptr(), B, L, ctypes.byref(rlk))
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.lib.he_mul_rescale_batch(out.data_ptr(), a.data_ptr(), b.data_ptr(), B, L, ctypes.byref(rlk))
    eng.sync()
    dt = time.perf_counter() - t0
    eng.exit()
    return {"q0_bits": bits, "qi_bits": 50, "p_bits": bits, "nspecial": K, "value": B * args.steps / dt,
            "unit": "ct-mult/s", "steps": args.steps}


def ntt_roundtrip(eng, stream, logn, L, polys, reps=3):
    """Config 2: forward + inverse NTT of `polys` polynomials x L limbs at
    N=2^logn resident in HBM (poly_ntt_batch / poly_intt_batch), timed with
    HIP events on the engine stream; algorithmic bytes = read + write of every
    limb per transform (twiddles amortised), i.e. 16 n L bytes per poly."""
    import torch
    n = 1 << logn
    buf = torch.empty(polys * L * n, dtype=torch.int64, device="cuda")
    eng.lib.poly_fill_uniform(buf.data_ptr(), polys, L, 0x48454354520001)
    eng.lib.poly_ntt_batch(buf.data_ptr(), polys, L)
    eng.lib.poly_intt_batch(buf.data_ptr(), polys, L)
    eng.sync()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(reps):
        eng.lib.poly_ntt_batch(buf.data_ptr(), polys, L)
        eng.lib.poly_intt_batch(buf.data_ptr(), polys, L)
    ev1.record(stream)
    eng.sync()
    dt = ev0.elapsed_time(ev1) / 1e3 / reps
    alg = 2.0 * 2 * 8 * n * L * polys  # two transforms, each reads + writes every limb once
    del buf
    return {"polys": polys, "nlimbs": L, "logn": logn, "roundtrip_ms": 1e3 * dt, "polys_per_s": polys / dt,
            "alg_GBs": alg / dt / 1e9, "frac_of_8TBs": alg / dt / 8e12}


def special_primes(L, dnum, q0_bits=60, qi_bits=50, p_bits=60):
    """Smallest K with P = prod(p_i) above the largest digit modulus (hybrid
    key switching needs P > Q_j for its noise bound)."""
    alpha = -(-L // dnum)
    digit_bits = q0_bits + (alpha - 1) * qi_bits
    return max(1, -(-digit_bits // p_bits))


def cstr_loop(steps):
    """Config 4: the encrypted CSTR-MPC closed loop on cuda:0 (HECTR's
    hectx_init(12, 2^109, slots, 2^50); horizon = steps/10, slots from
    src/ctr.c:510-511), steps/s end to end (plaintext plant + encrypted
    regulator, keygen excluded) and its deviation from the plaintext loop."""
    import numpy as np

    from hectr_amd.cstr import CstrProblem, EncryptedRegulator
    from hectr_amd.gpqhe import Engine
    pb = CstrProblem(steps)
    xp, up = pb.simulate(pb.regulator_plain)
    eng = Engine.product()
    reg = EncryptedRegulator(eng, pb, seed=5)
    t0 = time.perf_counter()
    x, u = pb.simulate(reg)
    dt = time.perf_counter() - t0
    reg.close()
    eng.exit()
    rel = float(max(np.max(np.abs(x - xp) / np.abs(xp)), np.max(np.abs(u - up) / np.abs(up))))
    return {"steps": steps, "horizon": pb.horizon, "slots": pb.slots, "steps_per_s": steps / dt,
            "regulator_ms_median": 1e3 * float(np.median(reg.timings)), "keygen_s": reg.keygen_s,
            "max_rel_dev_vs_plaintext": rel}


def cpu_baseline(args, logn, L, dnum):
    """Oracle (CPU restatement, -O3, OpenMP over the batch) on a bounded
    sample of the same op; threads = OMP_NUM_THREADS (16 on the GPU box)."""
    import numpy as np

    from hectr_amd.gpqhe import Engine
    threads = int(os.environ.get("OMP_NUM_THREADS", str(min(16, os.cpu_count() or 1))))
    ora = Engine.oracle()
    ora.init_params(logn=logn, nlimbs=L, dnum=dnum, slots=64, q0_bits=args.q0_bits, qi_bits=50, p_bits=args.p_bits,
                    seed=7, nspecial=args.nspecial or special_primes(L, dnum, q0_bits=args.q0_bits,
                                                                     p_bits=args.p_bits))
    pk, sk, rlk = ora.pk(), ora.sk(), ora.evk()
    ora.keypair(pk, sk)
    ora.genrlk(rlk, sk)
    n = 1 << logn
    cnt = 4 * threads  # a fixed set of pairs, multiplied repeatedly for ~cpu_seconds
    a = np.zeros(cnt * 2 * L * n, dtype=np.uint64)
    b = np.zeros_like(a)
    out = np.zeros(cnt * 2 * (L - 1) * n, dtype=np.uint64)
    ora.lib.poly_fill_uniform(a.ctypes.data, 2 * cnt, L, 11)
    ora.lib.poly_fill_uniform(b.ctypes.data, 2 * cnt, L, 12)
    done, t0 = 0, time.perf_counter()
    while True:
        ora.lib.he_mul_rescale_batch(out.ctypes.data, a.ctypes.data, b.ctypes.data, cnt, L, ctypes.byref(rlk))
        done += cnt
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds:
            break
    ora.exit()
    cnt = done
    return {"value": cnt / dt, "unit": "ct-mult/s", "cores": threads, "kind": "port",
            "sample": f"{cnt} ct x ct+relin+rescale ops at N=2^{logn}, L={L}, dnum={dnum} "
                      f"({4 * threads} distinct pairs, OpenMP over the batch, {dt:.1f} s)"}


if __name__ == "__main__":
    main()
