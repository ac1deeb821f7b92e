#!/usr/bin/env python3
"""bench.py - headline benchmark of the MI355X CKKS engine.

Metric (BASELINE.json): ct x ct + relinearization (+ rescale) per second at
N = 2^16, L = 8 RNS primes (configs[2]: batch = 256 ciphertext pairs per GPU,
one step = one batch through he_mul_rescale_batch, run as two 128-pair
sub-chunks on two HIP streams, gpqhe_set_streams).  Inputs are synthetic
random-residue ciphertexts already resident in HBM (poly_fill_uniform,
splitmix64 streams); the relinearization key is a real key (he_genrlk).

Multi-GPU: one process per GPU, each rank multiplies its own
shard of one global batch (independent ciphertexts: no data-path collective;
RCCL carries only the barrier and the max-time reduction) under one key: every
rank's context and relinearization key replica come from the same seed
(KEY_SEED), and pair g of the global batch is generated from seeds of g alone
(dist.fill_pairs).  `--check-shards` gathers the output shards and compares
them with one rank's run of the whole global batch.  `value` = pairs processed by all
ranks / max rank time ("scaling": "weak").  Under torchrun the ranks come from
the environment; `--gpus N` without torchrun starts the N rank processes
itself, before anything touches the GPU.

Also reported (rank 0):
  roofline      - the dominant kernel: SURVEY 8(d)'s algorithmic bytes per op
                  (2 ct in, 1 ct out at L-1, key / batch) x the pairs one launch
                  processes, / its average launch time (HIP events on the
                  engine stream), vs 8 TB/s; the kernel's own streamed bytes
                  and the PMC traffic of the pipeline beside it;
  op_roofline   - the whole op against its algorithmic bytes;
  value_60bit   - the same op with the conventional 60-bit q0 / special primes;
  config5       - n=2^17, L=12 (dnum 3, K 4), per GPU and aggregate, at the
                  headline's prime sizes and at the 60-bit ones;
  ntt_roundtrip - config 2 (1024 polys, forward + inverse, identity checked);
  cstr          - config 4, the encrypted CSTR-MPC loop;
  cpu_baseline  - the CPU restatement (oracle/, "port") on this host.
"""
import argparse
import ctypes
import glob
import json
import os
import re
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# one key for all ranks: the context / key replicas of every rank share these
# seeds (the headline and 60-bit legs, and config 5)
KEY_SEED, C5_KEY_SEED, GEMV_KEY_SEED, C5_GEMV_KEY_SEED = 1000, 2000, 3000, 4000
# kernels of the fused he_mul_rescale_batch pipeline (n = 2^16: one launch each per chunk)
PIPELINE = ("d2_rows_kernel", "ks_cols4_kernel", "ksq_kernel<drop>", "dn_cols_kernel", "ksq_kernel<keep>")


def parse(argv=None):
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
    ap.add_argument("--no-c5", action="store_true", help="skip the config 5 leg (n=2^17, L=12)")
    ap.add_argument("--c5-batch", type=int, default=64)
    ap.add_argument("--no-gemv", action="store_true", help="skip the he_gemv_batch / he_rot_batch leg")
    ap.add_argument("--gemv-batch", type=int, default=256)
    ap.add_argument("--c5-gemv-batch", type=int, default=64,
                    help="config 5 as a hempc batch: he_gemv_batch ciphertexts per GPU at N=2^17, L=12 (0: skip)")
    ap.add_argument("--gemv-slots", type=int, default=16, help="slots (HECTR's own: 16) = gemv diagonals")
    ap.add_argument("--ntt-polys", type=int, default=1024)
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline sample duration per thread count")
    ap.add_argument("--streams", type=int, default=2,
                    help="sub-chunks of a batch on their own HIP streams (gpqhe_set_streams: 1 or 2)")
    ap.add_argument("--launch-check", action="store_true",
                    help="run only the multi-process launch / rendezvous / reduction path (no engine, no GPU)")
    ap.add_argument("--check-shards", action="store_true",
                    help="after the timed steps, gather every rank's output shard and compare it bit for bit "
                         "with one rank's run of the whole global batch (rank 0)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# Launch: torchrun, or N rank processes started here
# ---------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """Start n fresh rank processes of this script (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* set) and wait for them.  The parent never touches the
    GPU, so no process that initialised it is ever replaced.  Returns the
    first non-zero exit code (0 when all ranks succeeded)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # poll: a rank that dies early would leave the others blocked in the
    # rendezvous or a collective, so the first failure ends them all
    while True:
        codes = [p.poll() for p in procs]
        bad = next((c for c in codes if c not in (None, 0)), None)
        if bad is not None:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            return bad
        if all(c == 0 for c in codes):
            return 0
        time.sleep(0.2)


def launch_check(args):
    """The N > 1 harness without the engine: rendezvous, barrier, the
    max-over-ranks reduction bench.py times with, and rank 0's JSON line."""
    from hectr_amd import dist as hdist
    rank, world, _ = hdist.env()
    backend = os.environ.get("HECTR_DIST_BACKEND", "nccl")
    hdist.init(backend)
    hdist.barrier()
    t = hdist.max_over_ranks(float(rank + 1))
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "requested": args.gpus, "max_over_ranks": t}))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


# ---------------------------------------------------------------------------
# Timed legs
# ---------------------------------------------------------------------------
def special_primes(L, dnum, q0_bits=60, qi_bits=50, p_bits=60):
    """Smallest K with P = prod(p_i) above the largest digit modulus (hybrid
    key switching needs P > Q_j for its noise bound)."""
    alpha = -(-L // dnum)
    digit_bits = q0_bits + (alpha - 1) * qi_bits
    return max(1, -(-digit_bits // p_bits))


def alg_bytes_per_op(n, L, K, dnum, batch):
    """read 2 ct (2 L limbs each), write 1 ct at L-1, the
    relinearization key (2 dnum (L+K) limbs) amortised over the batch."""
    return (2 * 2 * L + 2 * (L - 1)) * n * 8 + 2 * dnum * (L + K) * n * 8 / batch


class MulBatch:
    """One engine context + resident inputs for he_mul_rescale_batch."""

    def __init__(self, stream, logn, L, dnum, q0_bits, p_bits, nspecial, batch, first, seed):
        import torch
        from hectr_amd import dist as hdist
        from hectr_amd.gpqhe import Engine
        self.K = nspecial or special_primes(L, dnum, q0_bits=q0_bits, p_bits=p_bits)
        self.eng = Engine.product()
        self.eng.init_params(logn=logn, nlimbs=L, dnum=dnum, nspecial=self.K, slots=64, q0_bits=q0_bits,
                             qi_bits=50, p_bits=p_bits, seed=seed)
        self.eng.lib.gpqhe_set_stream(ctypes.c_void_p(stream.cuda_stream))
        self.pk, self.sk, self.rlk = self.eng.pk(), self.eng.sk(), self.eng.evk()
        self.eng.keypair(self.pk, self.sk)
        self.eng.genrlk(self.rlk, self.sk)
        n = 1 << logn
        self.n, self.L, self.B, self.dnum = n, L, batch, self.eng.info.dnum
        self.a = torch.empty(batch * 2 * L * n, dtype=torch.int64, device="cuda")
        self.b = torch.empty_like(self.a)
        self.out = torch.empty(batch * 2 * (L - 1) * n, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        # global pairs [first, first + batch): each rank multiplies its own shard
        hdist.fill_pairs(self.eng.lib, self.a.data_ptr(), self.b.data_ptr(), first, batch, L, n)
        self.eng.sync()

    def step(self):
        self.eng.lib.he_mul_rescale_batch(self.out.data_ptr(), self.a.data_ptr(), self.b.data_ptr(), self.B, self.L,
                                          ctypes.byref(self.rlk))

    def alg_bytes(self):
        return alg_bytes_per_op(self.n, self.L, self.K, self.dnum, self.B)

    def close(self):
        del self.a, self.b, self.out
        self.eng.exit()


class GemvBatch:
    """he_gemv_batch / he_rot_batch: HECTR's encrypted matrix-vector step
    (reference src/hempc.c:257-259, `slots` rotation keys from src/ctr.c:521,
    526-532) over a batch of independent ciphertexts sharing the matrix and the
    keys (north_star: the hempc ciphertext batch).  Ciphertext g of the global
    batch comes from seed + g alone (any sharding sees the same inputs); M is a
    dense random complex slots x slots matrix (every diagonal non-zero)."""

    def __init__(self, stream, logn, L, dnum, q0_bits, p_bits, nspecial, slots, batch, first, seed):
        import numpy as np
        import torch
        from hectr_amd.gpqhe import Engine
        self.K = nspecial or special_primes(L, dnum, q0_bits=q0_bits, p_bits=p_bits)
        self.eng = Engine.product()
        self.eng.init_params(logn=logn, nlimbs=L, dnum=dnum, nspecial=self.K, slots=slots, q0_bits=q0_bits,
                             qi_bits=50, p_bits=p_bits, seed=seed)
        self.eng.lib.gpqhe_set_stream(ctypes.c_void_p(stream.cuda_stream))
        self.pk, self.sk = self.eng.pk(), self.eng.sk()
        self.eng.keypair(self.pk, self.sk)
        self.rk = self.eng.evks(slots)
        self.eng.genrk(self.rk, self.sk)
        n = 1 << logn
        self.n, self.L, self.B, self.s, self.dnum = n, L, batch, slots, self.eng.info.dnum
        rng = np.random.default_rng(seed)
        self.M = np.ascontiguousarray((rng.uniform(-1, 1, (slots, slots)) + 1j * rng.uniform(-1, 1, (slots, slots)))
                                      .ravel())
        words = 2 * L * n
        self.x = torch.empty(max(batch, 1) * words, dtype=torch.int64, device="cuda")
        self.y = torch.empty(max(batch, 1) * 2 * (L - 1) * n, dtype=torch.int64, device="cuda")
        self.r = torch.empty_like(self.x)
        torch.cuda.synchronize()
        for i in range(batch):
            self.eng.lib.poly_fill_uniform(self.x.data_ptr() + 8 * i * words, 2, L, seed + first + i)
        self.eng.sync()

    def step(self):
        self.eng.lib.he_gemv_batch(self.y.data_ptr(), self.M.ctypes.data, self.x.data_ptr(), self.B, self.L, self.rk)

    def rot_step(self):
        self.eng.lib.he_rot_batch(self.r.data_ptr(), self.x.data_ptr(), self.B, self.L, 1, self.rk)

    def alg_bytes(self):
        """Per gemv: read the ciphertext (2 L limbs), write the output (2 (L-1)
        limbs), the s - 1 rotation keys (2 dnum (L+K) limbs each) and the s
        encoded diagonals (L+K limbs each) amortised over the batch."""
        n, L, nm = self.n, self.L, self.L + self.K
        return (2 * L + 2 * (L - 1)) * n * 8 + ((self.s - 1) * 2 * self.dnum * nm + self.s * nm) * n * 8 / self.B

    def rot_alg_bytes(self):
        n, L, nm = self.n, self.L, self.L + self.K
        return 4 * L * n * 8 + 2 * self.dnum * nm * n * 8 / self.B

    def close(self):
        del self.x, self.y, self.r
        self.eng.free_evks(self.rk)
        self.eng.exit()


def design_traffic_per_op(n, L, K, dnum):
    """HBM bytes per pair that the split key switch's five kernels move by
    design: d2_rows reads a1, b1 and writes y; ks_cols4
    reads y and writes T1 (each digit's nm - alpha targets); ksq<drop> reads
    T1 of the nd = K + 1 dropped slots (less the q_top limb's own digit) and
    the 4 input limbs of q_top, writes accd; dn_cols reads accd and writes
    conv for the keep = L - 1 kept slots; ksq<keep> reads T1 (one converted
    digit per slot less), the 4 inputs and conv per kept slot, writes out."""
    alpha = -(-L // dnum)
    ndig = -(-L // alpha)
    nm, nd, keep = L + K, K + 1, L - 1
    limbs = (3 * L + (L + ndig * nm - L) + (ndig * nd - 1 + 4 + 2 * nd) + (2 * nd + 2 * keep)
             + ((ndig - 1) * keep + 4 * keep + 2 * keep + 2 * keep))
    return limbs * n * 8


def timed(fn, steps, warmup, sync, barrier):
    """W untimed steps, then K timed steps bracketed by barrier + device sync."""
    import torch
    for _ in range(warmup):
        fn()
    sync()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync()
    torch.cuda.synchronize()
    barrier()
    return time.perf_counter() - t0


def pmc_profile(workload, pairs_per_launch):
    """Newest committed PMC summary (profiles/*_pmc.json, scripts/prof_summary.py
    over separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this same
    workload) whose metadata records the same pairs per launch."""
    def order(f):  # profiles/r<round>_v<version>_pmc.json, newest first
        m = re.search(r"r(\d+)_v(\d+)_pmc", os.path.basename(f))
        return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")), key=order, reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        meta = d.get("meta", {})
        if meta.get("bench_workload") == workload and meta.get("pairs_per_launch") == pairs_per_launch:
            return d, os.path.relpath(f, ROOT)
    return None, None


def kernel_key(name):
    """Kernel identity shared by the library's own statistics and rocprofv3
    names: the base name, plus <drop>/<keep> for the two ksq_kernel stages
    (5th template argument KEEP)."""
    base = name.split("<")[0].split("(")[0].strip()
    # the column / first-pass kernels' forms by prime set (cols_f64.hip,
    # cols_mixed.hip, d2_rows_q_kernel) under the pipeline role they fill
    base = {"ks_colsf_kernel": "ks_cols4_kernel", "ks_colsm_kernel": "ks_cols4_kernel",
            "dn_colsf_kernel": "dn_cols_kernel", "dn_colsm_kernel": "dn_cols_kernel",
            "d2_rows_q_kernel": "d2_rows_kernel"}.get(base, base)
    if base == "ksq_kernel" and "<" in name:
        args = [a.strip() for a in name[name.index("<") + 1:name.index(">")].split(",")]
        if args in (["keep"], ["drop"]):
            return f"ksq_kernel<{args[0]}>"
        if len(args) >= 5:
            return "ksq_kernel<keep>" if args[4] == "true" else "ksq_kernel<drop>"
    return base


def pmc_entry(prof, kernel):
    key = kernel_key(kernel)
    for name, e in prof.get("kernels", {}).items():
        if kernel_key(name) == key and "hbm_bytes" in e:
            return e
    return None


def roofline(stats, total_s, mb, workload, pairs_per_launch):
    dom_name = max(stats, key=lambda k: stats[k][1])
    launches, tot_us, kbytes = stats[dom_name]
    avg_us = tot_us / launches
    alg = mb.alg_bytes() * pairs_per_launch
    achieved = alg / avg_us / 1e3  # GB/s
    prof, src = pmc_profile(workload, pairs_per_launch)
    e = pmc_entry(prof, dom_name) if prof else None
    dom = {"bound": "hbm", "kernel": dom_name, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": achieved / HBM_PEAK_GBS, "traffic": e["hbm_bytes"] if e else None,
           "traffic_source": src, "avg_launch_us": avg_us, "alg_bytes_per_launch": alg,
           "alg_basis": f"SURVEY 8(d): {mb.alg_bytes():.0f} B/op x {pairs_per_launch} pairs per launch",
           "kernel_streamed_bytes_per_launch": kbytes / launches,
           "kernel_streamed_GBs": kbytes / tot_us / 1e3,
           "share_of_step": tot_us / (1e6 * total_s)}
    if e:
        for k in ("valu_busy", "sq_wait_any", "mean_us", "clock_GHz"):
            if k in e:
                dom["pmc_" + k] = e[k]
        # both axes as fractions of their peaks (no single "bound" verdict: the
        # kernel sits between them): its measured HBM traffic rate against
        # 8 TB/s, and its VALU issue (SQ_INSTS_VALU x 4 cycles per wave64 FP64
        # instruction, 1024 SIMDs at the measured clock) against the time
        dom["pmc_hbm_frac"] = e["hbm_bytes"] / e["mean_us"] / 1e3 / HBM_PEAK_GBS
        if "valu_frac" in e:
            dom["valu_frac"] = e["valu_frac"]
        if "valu_mix" in e:
            mix = e["valu_mix"]
            f64 = sum(mix.get(k, 0) for k in ("fma_f64", "mul_f64", "add_f64", "trans_f64"))
            dom["valu_insts_per_pair"] = e["sq_insts_valu"] / pairs_per_launch
            dom["valu_fp64_arith_share"] = f64 / e["sq_insts_valu"]
    if prof:
        pipe = [pmc_entry(prof, k) for k in PIPELINE]
        if all(pipe):
            tot = sum(p["hbm_bytes"] for p in pipe)
            dom["pipeline_traffic_per_chunk"] = tot
            dom["pipeline_traffic_ratio"] = tot / alg
            if all("sq_insts_valu" in p and "clock_GHz" in p for p in pipe):
                # the op's VALU floor: every VALU instruction of the five kernels
                # at full issue (4 cycles per wave64 instruction on each of 1024
                # SIMDs) at the clock each kernel ran at
                dom["valu_floor_us_per_op"] = sum(
                    p["sq_insts_valu"] * 4 / 1024 / (p["clock_GHz"] * 1e3) for p in pipe) / pairs_per_launch
                # the op's VALU axis: issue time of all five kernels / their time
                issue_us = sum(p["sq_insts_valu"] * 4 / 1024 / (p["clock_GHz"] * 1e3) for p in pipe)
                dom["pipeline_valu_frac"] = issue_us / sum(p["mean_us"] for p in pipe)
                dom["pipeline_valu_insts_per_pair"] = sum(p["sq_insts_valu"] for p in pipe) / pairs_per_launch
    return dom


def ntt_roundtrip(eng, stream, logn, L, polys, reps=3):
    """Config 2: forward + inverse NTT of `polys` polynomials x L limbs at
    N=2^logn resident in HBM (poly_ntt_batch / poly_intt_batch), timed with
    HIP events on the engine stream; algorithmic bytes = read + write of every
    limb per transform (twiddles amortised), i.e. 16 n L bytes per poly per
    transform.  The roundtrip identity is checked on the whole batch."""
    import torch
    n = 1 << logn
    buf = torch.empty(polys * L * n, dtype=torch.int64, device="cuda")
    eng.lib.poly_fill_uniform(buf.data_ptr(), polys, L, 0x48454354520001)
    eng.sync()
    orig = buf.clone()  # (on torch's stream: wait for it before the engine stream runs)
    torch.cuda.synchronize()
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
    identity = bool(torch.equal(buf, orig))
    alg = 2.0 * 2 * 8 * n * L * polys  # two transforms, each reads + writes every limb once
    del buf, orig
    return {"polys": polys, "nlimbs": L, "logn": logn, "roundtrip_ms": 1e3 * dt, "polys_per_s": polys / dt,
            "alg_GBs": alg / dt / 1e9, "frac_of_8TBs": alg / dt / 8e12, "identity_ok": identity}


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
    # he_gemv calls served by the speculated gemvs (absent from older A/B baselines)
    taken = eng.lib.gpqhe_spec_gemv_taken() if hasattr(eng.lib, "gpqhe_spec_gemv_taken") else None
    reg.close()
    eng.exit()
    rel = float(max(np.max(np.abs(x - xp) / np.abs(xp)), np.max(np.abs(u - up) / np.abs(up))))
    return {"steps": steps, "horizon": pb.horizon, "slots": pb.slots, "steps_per_s": steps / dt,
            "regulator_ms_median": 1e3 * float(np.median(reg.timings)),
            "regulator_ms_first_step": 1e3 * float(reg.timings[0]), "keygen_s": reg.keygen_s,
            "max_rel_dev_vs_plaintext": rel, "spec_gemv_taken": taken, "c_caller": cstr_c_caller()}


def product_lib_dir():
    """The directory of the product library the Python legs load (GPQHE_LIB,
    as hectr_amd.gpqhe.Engine.product): the C callers link it by name."""
    lib = os.environ.get("GPQHE_LIB")
    return os.path.dirname(os.path.abspath(lib)) if lib else os.path.join(ROOT, "hectr_amd", "lib")


def cstr_c_caller(reps=3):
    """HECTR's own unchanged harness (`test-hectr cstr-hempc`: 40 steps, C
    caller, its pmu timer around the closed loop) on the product library, as a
    child process; present when the binary was built in the build container
    (oracle/_ref, `make -C harness hectr`)."""
    import tempfile
    exe = os.path.join(ROOT, "oracle", "_ref", "test-hectr")
    if not os.path.exists(exe):
        return None
    env = dict(os.environ, LD_LIBRARY_PATH=product_lib_dir(), GPQHE_SEED="5")

    def run(mode):
        ms = []
        for _ in range(reps):
            with tempfile.TemporaryDirectory() as d:
                os.makedirs(os.path.join(d, "results"))
                r = subprocess.run([exe, mode], cwd=d, env=env, capture_output=True, text=True, timeout=120)
                m = re.search(r"closed-loop simulate\s+([0-9.]+) ms", r.stdout + r.stderr)
                if r.returncode or not m:
                    return None, (r.stdout + r.stderr)[-300:]
                ms.append(float(m.group(1)))
        return ms, None

    ms, err = run("cstr-hempc")
    if err:
        return {"error": err}
    med = sorted(ms)[len(ms) // 2]
    plain, _ = run("cstr-mpc")  # the same loop with the plaintext regulator (src/ctr.c:406)
    pmed = sorted(plain)[len(plain) // 2] if plain else None
    return {"steps": 40, "closed_loop_ms_median": med, "steps_per_s": 40e3 / med, "runs_ms": ms,
            "plaintext_closed_loop_ms_median": pmed,
            "encrypted_regulator_ms_per_step": (med - pmed) / 40 if pmed is not None else None,
            "config4_c_driver": cstr_c_driver(reps)}


def cstr_c_driver(reps=3, steps=100):
    """Config 4 at its own shape: the reference's unchanged hectr_simulate
    with N = 100 (horizon 10, 32 slots) through harness/cstr_run.c on the
    product library; steps/s from the closed-loop time the reference's own
    TEST_DO/TEST_DONE prints (keygen excluded, timed separately by it)."""
    import tempfile
    exe = os.path.join(ROOT, "oracle", "_ref", "cstr-run")
    if not os.path.exists(exe):
        return None
    import numpy as np
    env = dict(os.environ, LD_LIBRARY_PATH=product_lib_dir(), GPQHE_SEED="5")
    dt = np.dtype([("k", "<u4"), ("x", "<f8", 3), ("u", "<f8", 2)])  # tests/hectr.c:812-817
    fix = np.fromfile(os.path.join(ROOT, "tests", "golden", f"cstr-mpc-{steps}.bin"), dtype=dt)
    ms, keygen, dev = [], None, None
    for _ in range(reps):
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([exe, "hempc", str(steps), os.path.join(d, "t.bin")], env=env, capture_output=True,
                               text=True, timeout=120)
            log = r.stdout + r.stderr
            m = re.search(r"closed-loop simulate\s+([0-9.]+) ms", log)
            if r.returncode or not m:
                return {"error": log[-300:]}
            ms.append(float(m.group(1)))
            k = re.search(r"he_genrk\s+([0-9.]+) ms", log)
            keygen = float(k.group(1)) if k else None
            rec = np.fromfile(os.path.join(d, "t.bin"), dtype=dt)
            if len(rec) == len(fix):
                dev = float(max(np.max(np.abs(rec["x"] - fix["x"]) / np.abs(fix["x"])),
                                np.max(np.abs(rec["u"] - fix["u"]) / np.abs(fix["u"]))))
    med = sorted(ms)[len(ms) // 2]
    return {"steps": steps, "horizon": steps // 10, "slots": 32, "closed_loop_ms_median": med,
            "steps_per_s": steps * 1e3 / med, "runs_ms": ms, "genrk_ms": keygen,
            "max_rel_dev_vs_fixture": dev,
            "note": "reference hectr_simulate unchanged. At N = 100 the reference's ctr_hempc writes 33 rows into "
                    "its 32 x 32 stack matrix BBz (src/hempc.c:233-234 -> src/matrices.c:138-140); with the "
                    "reference's -Og build that overflow corrupts a stack neighbour, so this trajectory deviates "
                    "from the plaintext fixture cstr-mpc-100.bin by max_rel_dev_vs_fixture (1.34 % at most, 0.37 % at "
                    "steady state) whatever the "
                    "engine. Parity of this binary: bit-equal to its run on the oracle "
                    "(tests/test_gpu_hectr_caller.py); with the overflow contained (ASan build) the same caller "
                    "matches the fixture to ~3e-11 (tests/test_cstr_driver.py); the Python leg `cstr` is the "
                    "clean 1e-6 pin of config 4 (max_rel_dev_vs_plaintext)"}


def usable_cpus():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1


def cgroup_cpu_quota():
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        return None


def cpu_baseline(args, logn, L, dnum):
    """The oracle (CPU restatement, -O3, OpenMP over the batch) on a bounded
    sample of the same op, at the host's CPU share (OMP_NUM_THREADS: 16 on
    the GPU box) and at 4 threads (the reference's GPQHE_NUM_THREAD,
    src/config.h:59).  `value` is the first."""
    import numpy as np

    from hectr_amd.gpqhe import Engine
    share = int(os.environ.get("OMP_NUM_THREADS", str(min(16, usable_cpus()))))
    gomp = ctypes.CDLL("libgomp.so.1")
    ora = Engine.oracle()
    K = args.nspecial or special_primes(L, dnum, q0_bits=args.q0_bits, p_bits=args.p_bits)
    ora.init_params(logn=logn, nlimbs=L, dnum=dnum, slots=64, q0_bits=args.q0_bits, qi_bits=50, p_bits=args.p_bits,
                    seed=7, nspecial=K)
    pk, sk, rlk = ora.pk(), ora.sk(), ora.evk()
    ora.keypair(pk, sk)
    ora.genrlk(rlk, sk)
    n = 1 << logn
    cnt = 4 * share  # a fixed set of pairs, multiplied repeatedly for ~cpu_seconds
    a = np.zeros(cnt * 2 * L * n, dtype=np.uint64)
    b = np.zeros_like(a)
    out = np.zeros(cnt * 2 * (L - 1) * n, dtype=np.uint64)
    ora.lib.poly_fill_uniform(a.ctypes.data, 2 * cnt, L, 11)
    ora.lib.poly_fill_uniform(b.ctypes.data, 2 * cnt, L, 12)
    legs = {}
    for threads in (share, 4):
        gomp.omp_set_num_threads(threads)
        batch = max(threads, 4)
        done, t0 = 0, time.perf_counter()
        while True:
            ora.lib.he_mul_rescale_batch(out.ctypes.data, a.ctypes.data, b.ctypes.data, batch, L, ctypes.byref(rlk))
            done += batch
            dt = time.perf_counter() - t0
            if dt >= args.cpu_seconds:
                break
        legs[threads] = (done / dt, done, dt)
    ora.exit()
    v, done, dt = legs[share]
    v4, done4, dt4 = legs[4]
    return {"value": v, "unit": "ct-mult/s", "cores": share, "kind": "port",
            "sample": f"{done} ct x ct+relin+rescale ops at N=2^{logn}, L={L}, dnum={dnum} on {share} threads "
                      f"(OpenMP over batches of {max(share, 4)} distinct pairs, {dt:.1f} s)",
            "threads_4": {"value": v4, "cores": 4, "sample": f"{done4} ops, batches of 4, {dt4:.1f} s"},
            "host_cpus_usable": usable_cpus(), "host_cpus_total": os.cpu_count(),
            "cgroup_cpu_quota": cgroup_cpu_quota(),
            "note": "threads = OMP_NUM_THREADS (this job's CPU share on the GPU box), not every visible CPU"}


def shard_check(mine, rank, world, backend, batch, make_ref, key="pairs"):
    """Every rank's output shard (global items [rank B, (rank + 1) B)) gathered
    on rank 0 and compared word for word with one context's run of the whole
    global batch of world x B items under the same key seed (make_ref(count)
    -> that run's output on the host)."""
    import torch
    import torch.distributed as dist
    parts = [mine]
    if world > 1:
        dev = "cuda" if backend == "nccl" else "cpu"
        t = mine.to(dev)
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        parts = [p.cpu() for p in parts]
    res = None
    if rank == 0:
        full = make_ref(world * batch)
        got = torch.cat(parts)
        words = full.numel() // (world * batch)
        bad = (got != full).view(world * batch, words).any(dim=1).nonzero().flatten().tolist()
        res = {key: world * batch, "ranks": world, "bit_exact": not bad, "differing_" + key: bad[:16]}
    if world > 1:
        dist.barrier()
    return res


def mul_ref(stream, logn, L, dnum, q0_bits, p_bits, nspecial, seed):
    """make_ref for shard_check: one context's he_mul_rescale_batch of the
    whole global batch."""
    def run(count):
        ref = MulBatch(stream, logn, L, dnum, q0_bits, p_bits, nspecial, count, 0, seed)
        ref.step()
        ref.eng.sync()
        out = ref.out.cpu()
        ref.close()
        return out
    return run


def gemv_pmc():
    """Newest committed gemv-leg PMC summary (profiles/r<round>_v<version>_gemv_pmc.json)."""
    def order(f):
        m = re.search(r"r(\d+)_v(\d+)_gemv_pmc", os.path.basename(f))
        return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_gemv_pmc.json")), key=order, reverse=True):
        try:
            return json.load(open(f)), os.path.relpath(f, ROOT)
        except (OSError, ValueError):
            continue
    return None


def gemv_cpu_baseline(args, slots):
    """The oracle's he_gemv_batch (CPU restatement, OpenMP over the batch: one
    ciphertext per thread) on a bounded sample of the same workload."""
    import numpy as np

    from hectr_amd.gpqhe import Engine
    share = int(os.environ.get("OMP_NUM_THREADS", str(min(16, usable_cpus()))))
    ctypes.CDLL("libgomp.so.1").omp_set_num_threads(share)
    L, logn = args.nlimbs, args.logn
    dnum = args.dnum or L
    K = args.nspecial or special_primes(L, dnum, q0_bits=args.q0_bits, p_bits=args.p_bits)
    ora = Engine.oracle()
    ora.init_params(logn=logn, nlimbs=L, dnum=dnum, slots=slots, q0_bits=args.q0_bits, qi_bits=50,
                    p_bits=args.p_bits, seed=7, nspecial=K)
    pk, sk = ora.pk(), ora.sk()
    ora.keypair(pk, sk)
    rk = ora.evks(slots)
    ora.genrk(rk, sk)
    n, cnt = 1 << logn, share
    rng = np.random.default_rng(7)
    M = np.ascontiguousarray((rng.uniform(-1, 1, (slots, slots)) + 0j).ravel())
    x = np.zeros(cnt * 2 * L * n, dtype=np.uint64)
    y = np.zeros(cnt * 2 * (L - 1) * n, dtype=np.uint64)
    ora.lib.poly_fill_uniform(x.ctypes.data, 2 * cnt, L, 11)
    done, t0 = 0, time.perf_counter()
    while True:
        ora.lib.he_gemv_batch(y.ctypes.data, M.ctypes.data, x.ctypes.data, cnt, L, rk)
        done += cnt
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds:
            break
    ora.free_evks(rk)
    ora.exit()
    return {"value": done / dt, "unit": "gemv/s", "cores": share, "kind": "port",
            "sample": f"{done} he_gemv at N=2^{logn}, L={L}, {slots} slots on {share} threads "
                      f"(batches of {cnt} distinct ciphertexts, {dt:.1f} s)"}


def gemv_leg(args, stream, rank, world, red_dev, barrier, backend):
    """HECTR's encrypted matrix-vector step, he_gemv_batch (north_star: the
    hempc ciphertext batch; Galois rotation on the hot path), at the
    headline's ring and prime sizes with HECTR's own slot count, each rank its
    shard of one global batch under one key; he_rot_batch beside it."""
    import numpy as np
    import torch
    from hectr_amd import dist as hdist
    B, s = args.gemv_batch, args.gemv_slots
    steps = max(2, args.steps // 2)
    L, dnum = args.nlimbs, args.dnum or args.nlimbs
    gb = GemvBatch(stream, args.logn, L, dnum, args.q0_bits, args.p_bits, args.nspecial, s, B, rank * B,
                   GEMV_KEY_SEED)
    t0 = time.perf_counter()
    gb.step()  # the first call folds the rotation keys with the diagonals (cached)
    gb.eng.sync()
    first_s = time.perf_counter() - t0
    t_mine = timed(gb.step, steps, 1, gb.eng.sync, barrier)
    t_all = hdist.all_values(t_mine, device=red_dev)
    t = max(t_all)
    tr = hdist.max_over_ranks(timed(gb.rot_step, steps, 1, gb.eng.sync, barrier), device=red_dev)
    gb.eng.prof_enable(True)
    ti0 = time.perf_counter()
    for _ in range(steps):
        gb.step()
    gb.eng.sync()
    step_s = (time.perf_counter() - ti0) / steps
    stats = gb.eng.prof_collect()
    gb.eng.prof_enable(False)
    leg = None
    if rank == 0:
        v, vr = world * B * steps / t, world * B * steps / tr
        dom = max(stats, key=lambda k: stats[k][1])
        launches, tot_us, kbytes = stats[dom]
        per_launch = B / (launches / steps)
        alg = gb.alg_bytes()
        avg_us = tot_us / launches
        achieved = alg * per_launch / avg_us / 1e3
        generic = None
        try:
            generic = json.load(open(os.path.join(ROOT, "profiles", "r5_gemv_baseline_generic.json")))
        except (OSError, ValueError):
            pass
        leg = {"workload": f"he_gemv_batch ({s} x {s} complex matrix, {s} non-zero diagonals, hoisted rotations), "
                           f"N=2^{args.logn}, L={L}, K={gb.K}, dnum={gb.dnum}, primes {args.q0_bits}/50/{args.p_bits} "
                           f"bits, batch={B} ciphertexts per GPU",
               "n_gpus": world, "value": v, "per_gpu_value": v / world, "unit": "gemv/s", "steps": steps,
               "ms_per_step": 1e3 * t / steps, "rank_times_s": t_all, "rank_time_min_s": min(t_all),
               "rank_time_max_s": t,
               "rotations_in_gemv_per_s": v * (s - 1), "us_per_gemv_per_gpu": 1e6 * world / v,
               "first_call_ms": 1e3 * first_s,
               "rot_batch": {"value": vr, "unit": "rotations/s", "us_per_rotation_per_gpu": 1e6 * world / vr,
                             "op_roofline_frac": gb.rot_alg_bytes() * vr / world / 1e9 / HBM_PEAK_GBS},
               "op_roofline": {"alg_bytes_per_op": alg, "achieved_GBs": alg * v / world / 1e9,
                               "frac": alg * v / world / 1e9 / HBM_PEAK_GBS,
                               "alg_basis": "read the ciphertext (2 L limbs) + write y (2 (L-1) limbs) + (s-1) "
                                            "rotation keys and s encoded diagonals / batch"},
               "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "avg_launch_us": avg_us,
                            "alg_bytes_per_launch": alg * per_launch, "cts_per_launch": per_launch,
                            "share_of_step": tot_us / (1e6 * step_s * steps)},
               "kernels": {k: {"launches": w[0], "avg_us": w[1] / w[0], "us_per_gemv": w[1] / (steps * B),
                               "streamed_GBs": w[2] / w[1] / 1e3}
                           for k, w in sorted(stats.items(), key=lambda kv: -kv[1][1])},
               "data": "synthetic random-residue ciphertexts (splitmix64), real rotation keys (he_genrk)"}
        gp = gemv_pmc()
        if gp:
            e = next((v for k, v in gp[0].get("kernels", {}).items() if k.startswith(dom)), None)
            if e and "hbm_bytes" in e:
                # the inner-product kernel's PMC passes (profiles/*_gemv_pmc.json: the
                # same batch through scripts/gemv_time.py): HBM bytes per launch and
                # its VALU issue fraction (it sits on neither roof: keys from L2)
                leg["roofline"].update({"traffic": e["hbm_bytes"], "traffic_source": gp[1],
                                        "pmc_hbm_frac": e["hbm_bytes"] / e["mean_us"] / 1e3 / HBM_PEAK_GBS,
                                        "pmc_mean_us": e["mean_us"]})
                for k in ("valu_frac", "valu_busy", "l2_hit_rate", "sq_wait_any"):
                    if k in e:
                        leg["roofline"]["pmc_" + k] = e[k]
        if generic:
            leg["generic_path_us_per_gemv"] = generic.get("gemv_batch_us_per_ct")
            leg["generic_path_source"] = "profiles/r5_gemv_baseline_generic.json (round-4 kernels, same shape)"
            leg["speedup_vs_generic"] = generic["gemv_batch_us_per_ct"] / leg["us_per_gemv_per_gpu"]
    shard_y = gb.y.cpu() if args.check_shards else None
    gb.close()
    barrier()
    if args.alt_bits and args.alt_bits != args.q0_bits:
        # the same batch at HECTR-like prime sizes (60-bit q0 / P: those slots
        # on the integer form of the inner-product kernel, the mixed-set ModUp /
        # ModDown kernels)
        ga = GemvBatch(stream, args.logn, L, dnum, args.alt_bits, args.alt_bits, 0, s, B, rank * B, GEMV_KEY_SEED)
        ga.step()
        ga.eng.sync()
        ta = hdist.max_over_ranks(timed(ga.step, steps, 1, ga.eng.sync, barrier), device=red_dev)
        tra = hdist.max_over_ranks(timed(ga.rot_step, steps, 1, ga.eng.sync, barrier), device=red_dev)
        ga.eng.prof_enable(True)
        for _ in range(steps):
            ga.step()
        ga.eng.sync()
        sta = ga.eng.prof_collect()
        ga.eng.prof_enable(False)
        if rank == 0:
            va, vra = world * B * steps / ta, world * B * steps / tra
            leg["alt_primes"] = {
                "q0_bits": args.alt_bits, "qi_bits": 50, "p_bits": args.alt_bits, "K": ga.K, "value": va,
                "unit": "gemv/s", "us_per_gemv_per_gpu": 1e6 * world / va,
                "rot_batch": {"value": vra, "unit": "rotations/s", "us_per_rotation_per_gpu": 1e6 * world / vra},
                "kernels": {k: {"launches": w[0], "avg_us": w[1] / w[0], "us_per_gemv": w[1] / (steps * B)}
                            for k, w in sorted(sta.items(), key=lambda kv: -kv[1][1])}}
            try:
                gd = json.load(open(os.path.join(ROOT, "profiles", "r5_gemv_baseline_generic_d2.json")))
                leg["alt_primes"]["generic_path_us_per_gemv"] = gd["gemv_batch_us_per_ct"]
                leg["alt_primes"]["generic_path_source"] = ("profiles/r5_gemv_baseline_generic_d2.json (round-4 "
                                                            "kernels, same shape)")
                leg["alt_primes"]["speedup_vs_generic"] = gd["gemv_batch_us_per_ct"] / (1e6 * world / va)
            except (OSError, ValueError, KeyError):
                pass
        ga.close()
        barrier()
    if args.check_shards:
        def gemv_ref(count):
            ref = GemvBatch(stream, args.logn, L, dnum, args.q0_bits, args.p_bits, args.nspecial, s, count, 0,
                            GEMV_KEY_SEED)
            ref.step()
            ref.eng.sync()
            out = ref.y.cpu()
            ref.close()
            return out
        chk = shard_check(shard_y, rank, world, backend, B, gemv_ref, key="cts")
        if rank == 0:
            leg["shard_check"] = chk
    if rank == 0 and world == 1 and not args.no_cpu:
        leg["cpu_baseline"] = gemv_cpu_baseline(args, s)
    return leg


def c5_gemv_leg(args, stream, rank, world, red_dev, barrier, backend):
    """Config 5 read as written (BASELINE configs[4]: "hempc ciphertext batch
    sharded across 8 x MI355X, N=2^17, L=12"): he_gemv_batch -- hempc's
    encrypted matrix-vector step, src/hempc.c:257,259 -- at N=2^17, L=12
    (dnum 3, K 4, the headline's prime sizes), HECTR's 16 slots, each rank its
    shard of one global batch under one key, no collective on the data path."""
    from hectr_amd import dist as hdist
    B, s = args.c5_gemv_batch, args.gemv_slots
    steps = max(2, args.steps // 4)
    gb = GemvBatch(stream, 17, 12, 3, args.q0_bits, args.p_bits, 4, s, B, rank * B, C5_GEMV_KEY_SEED)
    gb.step()  # folds the rotation keys with the diagonals (cached)
    gb.eng.sync()
    t_all = hdist.all_values(timed(gb.step, steps, 1, gb.eng.sync, barrier), device=red_dev)
    t = max(t_all)
    gb.eng.prof_enable(True)
    for _ in range(steps):
        gb.step()
    gb.eng.sync()
    st = gb.eng.prof_collect()
    gb.eng.prof_enable(False)
    leg = None
    if rank == 0:
        v = world * B * steps / t
        leg = {"workload": f"he_gemv_batch ({s} x {s} complex matrix, {s} non-zero diagonals), N=2^17, L=12, "
                           f"K=4, dnum=3, primes {args.q0_bits}/50/{args.p_bits} bits, batch={B} ciphertexts per GPU",
               "n_gpus": world, "value": v, "per_gpu_value": v / world, "unit": "gemv/s", "steps": steps,
               "ms_per_step": 1e3 * t / steps, "us_per_gemv_per_gpu": 1e6 * world / v,
               "rotations_in_gemv_per_s": v * (s - 1), "rank_times_s": t_all, "rank_time_min_s": min(t_all),
               "rank_time_max_s": t,
               "op_roofline_frac": gb.alg_bytes() * v / world / 1e9 / HBM_PEAK_GBS,
               "kernels": {k: {"launches": w[0], "avg_us": w[1] / w[0], "us_per_gemv": w[1] / (steps * B)}
                           for k, w in sorted(st.items(), key=lambda kv: -kv[1][1])}}
    shard = gb.y.cpu() if args.check_shards else None
    gb.close()
    barrier()
    if args.check_shards:
        def ref(count):
            r = GemvBatch(stream, 17, 12, 3, args.q0_bits, args.p_bits, 4, s, count, 0, C5_GEMV_KEY_SEED)
            r.step()
            r.eng.sync()
            out = r.y.cpu()
            r.close()
            return out
        chk = shard_check(shard, rank, world, backend, B, ref, key="cts")
        if rank == 0:
            leg["shard_check"] = chk
    return leg


# ---------------------------------------------------------------------------
def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    if args.launch_check:
        return launch_check(args)
    import torch
    import torch.distributed as dist

    from hectr_amd import dist as hdist

    rank, world, local = hdist.env()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    # one process per GPU; the modulus only matters for rehearsals with more
    # ranks than GPUs (HECTR_DIST_BACKEND=gloo: RCCL needs distinct devices)
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    backend = os.environ.get("HECTR_DIST_BACKEND", "nccl")
    hdist.init(backend)
    red_dev = "cuda" if backend == "nccl" else "cpu"
    barrier = hdist.barrier

    L, logn, B = args.nlimbs, args.logn, args.batch
    dnum = args.dnum or L
    stream = torch.cuda.Stream()
    mb = MulBatch(stream, logn, L, dnum, args.q0_bits, args.p_bits, args.nspecial, B, rank * B, KEY_SEED)
    eng = mb.eng
    eng.lib.gpqhe_set_streams(args.streams)
    elapsed = timed(mb.step, args.steps, args.warmup, eng.sync, barrier)
    rank_times = hdist.all_values(elapsed, device=red_dev)
    elapsed = max(rank_times)
    value = world * B * args.steps / elapsed
    ms_per_step = 1e3 * elapsed / args.steps

    # instrumented pass (same steps): per-kernel device time from HIP events on
    # the engine stream, streamed bytes per launch from the library -- with
    # the batch as one chunk on one stream, so each kernel's launch time is
    # its own (two streams overlap the kernels of the two sub-chunks)
    eng.lib.gpqhe_set_streams(1)
    eng.prof_enable(True)
    ti0 = time.perf_counter()
    for _ in range(args.steps):
        mb.step()
    eng.sync()
    ti1 = time.perf_counter()
    stats = eng.prof_collect()
    eng.prof_enable(False)
    eng.lib.gpqhe_set_streams(args.streams)
    step_s = (ti1 - ti0) / args.steps
    launches_per_step = stats[max(stats, key=lambda k: stats[k][1])][0] / args.steps
    pairs_per_launch = int(round(B / launches_per_step))
    workload = (f"ct x ct mult + relin + rescale, N=2^{logn}, L={L}, K={mb.K}, dnum={mb.dnum}, "
                f"primes {args.q0_bits}/50/{args.p_bits} bits, batch={B} pairs per GPU")

    result = None
    if rank == 0:
        kernels = {k: {"launches": v[0], "avg_us": v[1] / v[0], "share": v[1] / (1e6 * step_s * args.steps),
                       "streamed_GBs": v[2] / v[1] / 1e3} for k, v in sorted(stats.items(), key=lambda kv: -kv[1][1])}
        alg = mb.alg_bytes()
        result = {
            "metric": "ct×ct+relin/sec at N=2^16, L=8 RNS primes; encrypted CSTR-MPC steps/sec",
            "value": value,
            "unit": "ct-mult/s",
            # the headline's prime sizes beside the conventional set's rate
            # (value_60bit, below, is the same op with 60-bit q0 / P)
            "primes": f"q0 {args.q0_bits}, q1..q{L - 1} 50, P {mb.K}x{args.p_bits} bits"
                      + (" (every modulus < 2^51: FP64 butterflies)" if max(args.q0_bits, args.p_bits) <= 51 else ""),
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
                       "batch_per_gpu": B, "logn": logn, "nlimbs": L, "nspecial": mb.K,
                       "dnum": mb.dnum, "prime_bits": {"q0": args.q0_bits, "qi": 50, "p": args.p_bits},
                       "pairs_per_launch": pairs_per_launch,
                       "streams": args.streams,
                       "parallelism": f"batch-sharded x{world}"},
            "per_gpu_value": value / world,
            "rank_times_s": rank_times, "rank_time_min_s": min(rank_times), "rank_time_max_s": elapsed,
            "op_roofline": {"alg_bytes_per_op": alg, "achieved_GBs": alg * value / world / 1e9,
                            "frac": alg * value / world / 1e9 / HBM_PEAK_GBS,
                            "us_per_op": 1e6 * world / value},
            "roofline": roofline(stats, step_s * args.steps, mb, workload, pairs_per_launch),
            "kernels": kernels,
            "instrumented_ms_per_step": 1e3 * step_s,
        }
        # the op's two design floors beside the measured time: the five
        # kernels' VALU instructions at full issue (PMC profile) and their design
        # HBM traffic at the 8 TB/s peak; the frac the op could reach at each
        opr, rf = result["op_roofline"], result["roofline"]
        dt_bytes = design_traffic_per_op(1 << logn, L, mb.K, mb.dnum) if dnum == 2 else None
        if dt_bytes:
            opr["design_traffic_per_op"] = dt_bytes
            opr["design_traffic_floor_us_at_peak"] = dt_bytes / HBM_PEAK_GBS / 1e3
            opr["design_traffic_ratio"] = dt_bytes / alg
        if "valu_floor_us_per_op" in rf:
            opr["valu_floor_us_per_op"] = rf["valu_floor_us_per_op"]
            opr["valu_floor_source"] = rf.get("traffic_source")
        floors = [opr.get("valu_floor_us_per_op"), opr.get("design_traffic_floor_us_at_peak")]
        if all(floors):
            opr["frac_at_max_floor"] = alg / (max(floors) * 1e3) / HBM_PEAK_GBS
        if world == 1 and not args.no_ntt:
            result["ntt_roundtrip"] = ntt_roundtrip(eng, stream, logn, L, args.ntt_polys)
    shard_out = mb.out.cpu() if args.check_shards else None  # the last step's output (every step writes the same)
    mb.close()
    barrier()
    if args.check_shards:
        chk = shard_check(shard_out, rank, world, backend, B,
                          mul_ref(stream, logn, L, dnum, args.q0_bits, args.p_bits, args.nspecial, KEY_SEED))
        if rank == 0:
            result["shard_check"] = chk

    if args.alt_bits and args.alt_bits != args.q0_bits:
        # the conventional prime sizes (60-bit q0 and special primes: the
        # integer butterflies on those limbs), same op, batch and harness
        alt = MulBatch(stream, logn, L, dnum, args.alt_bits, args.alt_bits, 0, B, rank * B, KEY_SEED)
        alt.eng.lib.gpqhe_set_streams(args.streams)
        t = hdist.max_over_ranks(timed(alt.step, args.steps, 1, alt.eng.sync, barrier), device=red_dev)
        alt.eng.lib.gpqhe_set_streams(1)  # instrumented single-stream pass, as the headline's
        alt.eng.prof_enable(True)
        for _ in range(args.steps):
            alt.step()
        alt.eng.sync()
        sta = alt.eng.prof_collect()
        alt.eng.prof_enable(False)
        if rank == 0:
            v = world * B * args.steps / t
            result["value_60bit"] = v
            result["alt_primes"] = {"q0_bits": args.alt_bits, "qi_bits": 50, "p_bits": args.alt_bits,
                                    "nspecial": alt.K, "value": v, "unit": "ct-mult/s", "steps": args.steps,
                                    "op_roofline_frac": alt.alg_bytes() * v / world / 1e9 / HBM_PEAK_GBS,
                                    "kernels": {k: {"launches": w[0], "avg_us": w[1] / w[0],
                                                    "us_per_pair": w[1] / (args.steps * B)}
                                                for k, w in sorted(sta.items(), key=lambda kv: -kv[1][1])}}
        alt.close()
        barrier()

    if not args.no_c5:
        # config 5: n = 2^17, L = 12 (dnum 3, K 4), each rank its own shard of
        # the global batch; the headline's prime sizes (q0 and P of
        # --q0-bits / --p-bits: every modulus below 2^51) and the conventional
        # 60-bit q0 / P beside them, same harness
        steps5 = max(2, args.steps // 2)

        def c5_leg(q0_bits, p_bits):
            c5 = MulBatch(stream, 17, 12, 3, q0_bits, p_bits, 4, args.c5_batch, rank * args.c5_batch, C5_KEY_SEED)
            c5.eng.lib.gpqhe_set_streams(args.streams)
            t_all = hdist.all_values(timed(c5.step, steps5, 1, c5.eng.sync, barrier), device=red_dev)
            t = max(t_all)
            # instrumented single-stream pass, as the headline's: per-kernel time
            c5.eng.lib.gpqhe_set_streams(1)
            c5.eng.prof_enable(True)
            for _ in range(steps5):
                c5.step()
            c5.eng.sync()
            st5 = c5.eng.prof_collect()
            c5.eng.prof_enable(False)
            c5.eng.lib.gpqhe_set_streams(args.streams)
            leg = None
            if rank == 0:
                v = world * args.c5_batch * steps5 / t
                leg = {"workload": f"ct x ct mult + relin + rescale, N=2^17, L=12, K=4, dnum=3, "
                                   f"primes {q0_bits}/50/{p_bits} bits, batch={args.c5_batch} pairs per GPU",
                       "n_gpus": world, "value": v, "per_gpu_value": v / world, "unit": "ct-mult/s",
                       "steps": steps5, "ms_per_step": 1e3 * t / steps5, "rank_times_s": t_all,
                       "rank_time_min_s": min(t_all), "rank_time_max_s": t,
                       "op_roofline_frac": c5.alg_bytes() * v / world / 1e9 / HBM_PEAK_GBS,
                       "kernels": {k: {"launches": w[0], "avg_us": w[1] / w[0], "us_per_pair": w[1] / (steps5 * args.c5_batch),
                                       "streamed_GBs": w[2] / w[1] / 1e3}
                                   for k, w in sorted(st5.items(), key=lambda kv: -kv[1][1])}}
            out5 = c5.out.cpu() if args.check_shards else None
            c5.close()
            barrier()
            if args.check_shards:
                chk = shard_check(out5, rank, world, backend, args.c5_batch,
                                  mul_ref(stream, 17, 12, 3, q0_bits, p_bits, 4, C5_KEY_SEED))
                if rank == 0:
                    leg["shard_check"] = chk
            return leg

        main5 = c5_leg(args.q0_bits, args.p_bits)
        alt5 = c5_leg(args.alt_bits, args.alt_bits) if args.alt_bits and args.alt_bits != args.q0_bits else None
        if rank == 0:
            result["config5"] = main5
            if alt5:
                main5["value_60bit"] = alt5["value"]
                main5["alt_primes"] = alt5

    if not args.no_gemv:
        g = gemv_leg(args, stream, rank, world, red_dev, barrier, backend)
        if rank == 0:
            result["gemv"] = g
        if not args.no_c5 and args.c5_gemv_batch:
            g5 = c5_gemv_leg(args, stream, rank, world, red_dev, barrier, backend)
            if rank == 0:
                result["config5"]["hempc_gemv"] = g5

    if rank == 0 and world == 1 and not args.no_cstr:
        result["cstr"] = cstr_loop(args.cstr_steps)
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(args, logn, L, dnum)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
