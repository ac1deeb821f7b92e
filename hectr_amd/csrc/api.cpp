// api.cpp - the he_* / hectx_* C ABI of libgpqhe.so (include/gpqhe.h) on
// MI355X.  Host C++ orchestrating the gfx950 kernels of kernels.hip on one
// HIP stream; every object payload lives in HBM.  Call-site contract:
// reference src/ctr.c:445-618 and src/hempc.c:216-274 (see gpqhe.h).
#include "gpqhe_internal.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <list>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>

Context G;

// ===========================================================================
// Device memory pool: exact-size free lists, stream-ordered reuse.
// ===========================================================================
static std::map<size_t, std::vector<void *>> g_free;
static std::unordered_map<void *, size_t> g_size;

static size_t pool_round(size_t b)
{
  return (b + 4095) & ~(size_t)4095;
}

static void flush_ew();
static void fold_cache_trim();

void *pool_alloc(size_t bytes)
{
  const size_t b = pool_round(bytes ? bytes : 1);
  auto it = g_free.find(b);
  if (it != g_free.end() && !it->second.empty()) {
    void *p = it->second.back();
    it->second.pop_back();
    return p;
  }
  void *p = nullptr;
  hipError_t e = hipMalloc(&p, b);
  if (e != hipSuccess) {
    // give cached blocks back and retry once (queued elementwise ops may
    // still name a free-listed block: they run first); folded key sets no
    // running call reads go back too
    flush_ew();
    HIP_CHECK(hipStreamSynchronize(G.stream));
    fold_cache_trim();
    for (auto &kv : g_free)
      for (void *q : kv.second) {
        (void)hipFree(q);
        g_size.erase(q);
      }
    g_free.clear();
    HIP_CHECK(hipMalloc(&p, b));
  }
  g_size[p] = b;
  return p;
}

void pool_free(void *p)
{
  if (!p)
    return;
  auto it = g_size.find(p);
  if (it == g_size.end())
    return;  // payload of an object that outlived a previous context (already released)
  g_free[it->second].push_back(p);
}

void pool_release_all()
{
  // g_size holds every block ever allocated (free-listed or still owned by a
  // caller object that outlives the context); free each exactly once
  for (auto &kv : g_size)
    HIP_CHECK(hipFree(kv.first));
  g_size.clear();
  g_free.clear();
}

// RAII workspace
struct Ws {
  uint64_t *p;
  explicit Ws(size_t words) : p(words ? (uint64_t *)pool_alloc(words * 8) : nullptr) {}
  ~Ws() { pool_free(p); }
  Ws(const Ws &) = delete;
  Ws &operator=(const Ws &) = delete;
};

// Folded gemv / rotation keys (see gemv_fold below).
static uint64_t g_key_gen = 1;
struct FoldEntry {
  std::vector<double> M;  // the matrix (he_gemv); empty for a rotation
  unsigned s, lvl, rot;
  uint64_t gen;
  const he_evk_t *rk;
  std::vector<unsigned> d;  // rotation of each folded diagonal
  double *K;
  size_t bytes;
};
// (a list: a caller's reference to its entry survives the eviction of others)
static std::list<FoldEntry> g_folds;
static const double *g_fold_inuse = nullptr;  // the set a running call reads
// While a call reads a folded set, an out-of-memory retry inside it keeps
// that set (fold_cache_trim).
struct FoldUse {
  explicit FoldUse(const FoldEntry &f) { g_fold_inuse = f.K; }
  ~FoldUse() { g_fold_inuse = nullptr; }
};

static void fold_cache_clear();
static bool gemv_fold_fits(const double *Md, unsigned lvl, const he_evk_t rk[]);
static bool gemv_win_on(unsigned lvl);
static const FoldEntry &gemv_fold(const double *Md, unsigned lvl, const he_evk_t rk[]);
static const FoldEntry &rot_fold(unsigned r, unsigned lvl, const he_evk_t rk[]);

// Pinned staging ring for small host->device uploads (encode).
struct Stage {
  void *host = nullptr;
  hipEvent_t ev = nullptr;
  size_t bytes = 0;
};
static Stage g_stage[8];
static unsigned g_stage_next = 0;

// The next slot, free again (its last reader has run), holding a copy of src.
static Stage &stage_fill(const void *src, size_t bytes)
{
  Stage &s = g_stage[g_stage_next++ % 8];
  if (s.ev)
    HIP_CHECK(hipEventSynchronize(s.ev));
  else
    HIP_CHECK(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
  if (s.bytes < bytes) {
    if (s.host)
      HIP_CHECK(hipHostFree(s.host));
    HIP_CHECK(hipHostMalloc(&s.host, bytes, hipHostMallocDefault));
    s.bytes = bytes;
  }
  memcpy(s.host, src, bytes);
  return s;
}

static void upload(void *dst, const void *src, size_t bytes)
{
  Stage &s = stage_fill(src, bytes);
  HIP_CHECK(hipMemcpyAsync(dst, s.host, bytes, hipMemcpyHostToDevice, G.stream));
  HIP_CHECK(hipEventRecord(s.ev, G.stream));
}

// Zero-copy form for a few KB that one launch reads: the kernel reads the
// pinned slot over PCIe (no copy launch); stage_done() after that launch.
static Stage &stage_map(const void *src, size_t bytes, const void **dev)
{
  Stage &s = stage_fill(src, bytes);
  void *d = nullptr;
  HIP_CHECK(hipHostGetDevicePointer(&d, s.host, 0));
  *dev = d;
  return s;
}

static void stage_done(Stage &s) { HIP_CHECK(hipEventRecord(s.ev, G.stream)); }

static void *g_zpin = nullptr;  // pinned decode output (he_dcd_ex)
static size_t g_zpin_bytes = 0;

// he_mul_rescale_batch's second sub-chunk stream and its fork / join events
// (created on first use, released by hectx_exit: no HIP object of the engine
// is left for the runtime's or a profiler's exit handlers)
struct SecondStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, d2 = nullptr, join = nullptr;
};
static SecondStream g_s2;
static hipEvent_t g_dcd_ev = nullptr;  // end of the small-N decode (spec_launch)

static void stage_release()
{
  if (g_zpin)
    (void)hipHostFree(g_zpin);
  g_zpin = nullptr;
  g_zpin_bytes = 0;
  for (Stage &s : g_stage) {
    if (s.ev) {
      (void)hipEventSynchronize(s.ev);
      (void)hipEventDestroy(s.ev);
    }
    if (s.host)
      (void)hipHostFree(s.host);
    s = Stage{};
  }
}

// ===========================================================================
// Deferred encode + public-key encryption (the small-N latency path).
//
// HECTR encodes and encrypts its five state vectors back to back every control
// step (src/ctr.c:466-475), then frees the plaintexts.  Each he_ecd (host FFT,
// upload, lift + NTT) and he_enc_pk (sample v, e0, e1, NTT, combine) is queued
// instead of launched, and the queue runs as one batch -- one upload, one
// lift + NTT, one sampling, one NTT and one combine launch for all of them --
// when anything else touches the engine (every other entry point flushes
// first).  The RNG streams are taken at call time, so the results are the
// ones of the sequential calls bit for bit.
// ===========================================================================
struct PendEcd {
  uint64_t *dst;
  unsigned lvl, slots;
  size_t coff;  // its 2 slots coefficient values at g_pcoef + coff (hm_encode_slots)
};
struct PendEnc {
  uint64_t *c0, *c1;
  const uint64_t *m, *pk0, *pk1;
  unsigned lvl;
  uint64_t stream;
  int ecd;  // m is queued encode ecd (its coefficients join e0: EncCoef), else -1
};
static std::vector<PendEcd> g_pecd;
static std::vector<int64_t> g_pcoef;  // 2 slots coefficient values per pending encode
static std::vector<PendEnc> g_penc;

// Speculative encryption noise.  HECTR encrypts its K = 5 states every control
// step on consecutive RNG streams (src/ctr.c:471-475).  When a step ends in the
// small-N he_dcd, the noise of the next K encryptions -- streams G.counter ..
// G.counter + 3K - 1, sampled and transformed exactly as flush_pending would --
// is launched behind the decode (the host waits for the decode only), so it
// runs while the caller works on the host.  A later flush whose encryptions
// take exactly those streams at that level uses it, and its combine
// evaluates the plaintexts from their coefficients (k_enc_combine_m): the step
// starts with the combine instead of sampling and transforms.
struct SpecNoise {
  uint64_t *buf = nullptr;  // [3k][lvl][n], NTT form (pool block, kept)
  size_t words = 0;
  uint64_t base = 0;  // first stream
  unsigned k = 0, lvl = 0;
  bool valid = false;
};
static SpecNoise g_spec;
static unsigned g_spec_next_k = 0, g_spec_next_lvl = 0;  // the last flush's encryptions (one run)
static uint64_t g_step_base = 0;                          // their first stream

// Speculative ModUp.  The c1 of a fresh encryption, v pk1 + e1, does not
// depend on the plaintext, and HECTR's he_gemv inputs are differences of two
// fresh encryptions (src/hempc.c:253-259).  The queued small-N calls record
// how each c1 poly was made (C1Prov: an encryption's stream, or the he_sub of
// two of them); when a step's gemv inputs were such differences, the next
// step's he_dcd also forms the same differences from the speculative noise
// and runs their ModUp, and a he_gemv whose input c1 has exactly that
// provenance (same streams, public key and level) takes the precomputed
// digits.  Any other write clears the record (check_ctx, non-queued writers),
// so a match always names the same values.
struct C1Prov {
  uint64_t sa, sb;  // streams: the encryption's (sb unused), or a - b
  const uint64_t *pk1;
  unsigned lvl;
  bool sub;
  bool c0 = false;  // the record of an encryption's c0 poly (SpecGemv), not c1
};
static std::unordered_map<const uint64_t *, C1Prov> g_prov;
struct SpecPat {
  unsigned oa, ob;  // encryption offsets within the step's run
};
static std::vector<SpecPat> g_spec_pats_next;  // the last step's gemv inputs
static const uint64_t *g_spec_pk1_next = nullptr;
struct SpecModup {
  uint64_t *D = nullptr;  // [np][ndig][nm][n]
  size_t dwords = 0;
  uint64_t *Y = nullptr;  // [np][lvl][n] the split ModUp's hand-off (ModupHalves)
  size_t ywords = 0;
  std::vector<SpecPat> pats;
  uint64_t base = 0;
  const uint64_t *pk1 = nullptr;
  unsigned lvl = 0;
  bool valid = false;
};
static SpecModup g_smu;
// spec_attach's ModUp, launched behind the decode (spec_modup_launch)
struct SpecModupNext {
  C1Diffs cd{};
  unsigned np = 0, lvl = 0;
  size_t d_stride = 0;
  const uint64_t *pk1 = nullptr;
  bool pending = false;
};
static SpecModupNext g_smu_next;

// Speculative gemv (GPQHE_SPEC_GEMV).  Once the step's encryptions have run
// (spec_flush_early), the last step's gemvs -- the same encryption slots, the
// same matrices and keys, HECTR's he_gemv of xhat - xr and uhat - ur, src/
// hempc.c:253-259 -- run at once on this step's ciphertexts: the inner
// products on the speculated ModUp digits with the differences formed in the
// kernel, and the ModDown, into SpecGemv::Y.  That device work then overlaps
// the caller's host work up to its he_gemv calls (the horizon matrices,
// src/hempc.c:225-240) instead of running between them and the decode.  A
// he_gemv whose input is the queued difference of exactly those polys, still
// holding those encryptions (C1Prov records of c0 and c1, dropped by any
// write), with the same matrix, keys and key generation, queues a copy of its
// Y instead; anything else takes the normal path.
struct SgRec {  // a step's gemv, recorded for the next step's speculation
  SpecPat pat;
  std::vector<double> M;
  GemvDiags dg;  // its one launch's diagonals (evk filled)
  const he_evk_t *rk;
  uint64_t gen;
};
static std::vector<SgRec> g_sg_next;  // this step's gemvs (in g_spec_pats_next order)
struct SpecGemv {
  // pattern i's result, in a block shaped as a ciphertext object's (2 polys
  // of G.L limbs): a taking he_gemv swaps it with its output object's block
  uint64_t *Y[GemvJobs::MAX] = {};
  unsigned np = 0, lvl = 0;
  const uint64_t *x[GemvJobs::MAX][4];  // a0, b0, a1, b1 per pattern
  uint64_t sa[GemvJobs::MAX], sb[GemvJobs::MAX];
  SgRec rec[GemvJobs::MAX];
  bool used[GemvJobs::MAX];
  bool valid = false;
};
static SpecGemv g_sg;
static unsigned g_sg_taken = 0;  // gpqhe_spec_gemv_taken

extern "C" unsigned gpqhe_spec_gemv_taken(void)
{
  return g_sg_taken;
}

// Speculative decode of the small-N step (SpecDcd; GPQHE_SPEC_DCD=0 turns it
// off).  A step's tail -- the queued elementwise program (HECTR's he_add,
// he_neg, he_copy_ct, he_add, he_dec: src/hempc.c:261-266, src/ctr.c:486) and
// the decode -- waits on the caller: it is issued at he_dcd, after the
// caller's own host work.  Its operands are this step's speculated gemv
// results, its encryptions, its own temporaries and the secret key, so the
// last step's program, recorded by the roles of its operands (SdPat), is
// replayed on this step's objects right after the speculated gemvs (temporaries
// in scratch, the decode into pinned memory), where it runs in the caller's
// shadow.  he_dcd takes the replay's values when this step's program has the
// same pattern, reading the same blocks (the gemv results still in the blocks
// the speculation wrote, the encryptions still holding their streams:
// C1Prov), and the real program then runs without being waited for.  When the
// replay is still running at he_dcd on two consecutive steps (the caller
// outruns the device: the replay only adds work to the step's chain) it stops.
static unsigned env_u(const char *name, unsigned dflt);
enum : uint8_t { SR_OUT = 0, SR_Y = 1, SR_ENC = 2 };
struct SdRole {
  uint8_t kind = 0, idx = 0, poly = 0;
  bool operator==(const SdRole &o) const { return kind == o.kind && idx == o.idx && poly == o.poly; }
};
struct SdPat {
  unsigned count = 0, nl = 0, slots = 0, sid = 0;  // sid: the out id holding the decoded plaintext
  double scale = 0;
  const uint64_t *sk = nullptr;
  uint32_t kind[EwProg::MAX] = {}, lvl[EwProg::MAX] = {};
  SdRole out[EwProg::MAX], a[EwProg::MAX], b[EwProg::MAX];
  bool same(const SdPat &o) const
  {
    if (count != o.count || nl != o.nl || slots != o.slots || sid != o.sid || scale != o.scale || sk != o.sk)
      return false;
    for (unsigned j = 0; j < count; j++)
      if (kind[j] != o.kind[j] || lvl[j] != o.lvl[j] || !(out[j] == o.out[j]) || !(a[j] == o.a[j]) ||
          !(b[j] == o.b[j]))
        return false;
    return true;
  }
};
struct SdCtx {  // a step's role blocks (spec_gemv_launch)
  const uint64_t *y[GemvJobs::MAX] = {};
  unsigned ny = 0, ylvl = 0;
  const uint64_t *e[GPQHE_MAXGRP][2] = {};
  uint64_t es[GPQHE_MAXGRP] = {};
  unsigned ne = 0, elvl = 0;
  bool valid = false;
};
struct SpecDcd {
  SdPat pat;  // the pattern replayed this step
  uint64_t *scratch = nullptr, *cws = nullptr;
  size_t swords = 0, cwords = 0;
  void *z = nullptr;  // pinned decoded values
  size_t zbytes = 0;
  hipEvent_t ev = nullptr;
  bool valid = false;
};
static SdCtx g_sd_ctx;    // this step's roles
static SdPat g_sd_next;   // this step's pattern, replayed by the next step
static bool g_sd_next_ok = false;
static SpecDcd g_sd;
static unsigned g_sd_taken = 0, g_sd_late = 0;
static bool g_sd_off = false;

extern "C" unsigned gpqhe_spec_dcd_taken(void)
{
  return g_sd_taken;
}

// The roles of program p's operands and of the decoded plaintext ptd under the
// step roles c; false when some operand has none (or could alias one).
static bool sd_pattern(const EwProg &p, const uint64_t *ptd, unsigned nl, unsigned slots, double scale,
                       const SdCtx &c, SdPat &r)
{
  if (!c.valid || !p.count || nl < 1 || nl > 2)
    return false;
  const size_t n = G.n, ypw = (size_t)G.L << G.logn;
  r = SdPat{};
  r.count = p.count;
  r.nl = nl;
  r.slots = slots;
  r.scale = scale;
  auto ov = [&](const uint64_t *x, unsigned lx, const uint64_t *y, unsigned ly) {
    return x < y + (size_t)ly * n && y < x + (size_t)lx * n;
  };
  unsigned oid[EwProg::MAX];
  // operand x read over lv limbs before op j: the latest earlier writer of
  // exactly x (with at least those limbs), else a role block
  auto read = [&](unsigned j, const uint64_t *x, unsigned lv, SdRole &role) {
    for (int k = (int)j - 1; k >= 0; k--) {
      const EwOp &w = p.op[k];
      if (w.out == x) {
        if (w.lvl < lv)
          return false;
        role = SdRole{SR_OUT, (uint8_t)oid[k], 0};
        return true;
      }
      if (ov(w.out, w.lvl, x, lv))
        return false;
    }
    for (unsigned i = 0; i < c.ny; i++)
      for (unsigned q = 0; q < 2; q++)
        if (x == c.y[i] + q * ypw) {
          if (lv > c.ylvl)
            return false;
          role = SdRole{SR_Y, (uint8_t)i, (uint8_t)q};
          return true;
        }
    for (unsigned o = 0; o < c.ne; o++)
      for (unsigned q = 0; q < 2; q++)
        if (x == c.e[o][q]) {
          if (lv > c.elvl)
            return false;
          role = SdRole{SR_ENC, (uint8_t)o, (uint8_t)q};
          return true;
        }
    return false;
  };
  for (unsigned j = 0; j < p.count; j++) {
    const EwOp &o = p.op[j];
    r.kind[j] = o.kind;
    r.lvl[j] = o.lvl;
    oid[j] = j;
    for (unsigned k = 0; k < j; k++) {
      if (p.op[k].out == o.out) {
        oid[j] = oid[k];
        break;
      }
      if (ov(p.op[k].out, p.op[k].lvl, o.out, o.lvl))
        return false;
    }
    r.out[j] = SdRole{SR_OUT, (uint8_t)oid[j], 0};
    if (!read(j, o.a, o.lvl, r.a[j]))
      return false;
    if ((o.kind == EW_ADD || o.kind == EW_SUB || o.kind == EW_DEC) && !read(j, o.b, o.lvl, r.b[j]))
      return false;
    if (o.kind == EW_DEC) {  // the key: one block, never an output
      if (r.sk && r.sk != o.s)
        return false;
      r.sk = o.s;
      for (unsigned k = 0; k < p.count; k++)
        if (ov(p.op[k].out, p.op[k].lvl, o.s, o.lvl))
          return false;
    }
  }
  SdRole pr;
  if (!read(p.count, ptd, nl, pr) || pr.kind != SR_OUT)
    return false;
  r.sid = pr.idx;
  return true;
}

// Every encryption role of r still holds its stream (C1Prov: any write since
// dropped it).
static bool sd_enc_fresh(const SdPat &r, const SdCtx &c)
{
  auto ok = [&](const SdRole &q) {
    if (q.kind != SR_ENC)
      return true;
    auto it = g_prov.find(c.e[q.idx][q.poly]);
    return it != g_prov.end() && !it->second.sub && it->second.c0 == (q.poly == 0) && it->second.sa == c.es[q.idx] &&
           it->second.lvl == c.elvl;
  };
  for (unsigned j = 0; j < r.count; j++)
    if (!ok(r.a[j]) || !ok(r.b[j]))
      return false;
  return true;
}

// The last step's pattern on this step's roles (g_sd_ctx): the program with
// its temporaries in scratch, then the decode into pinned memory.
static void sd_replay(const SdPat &r)
{
  const size_t blk = (size_t)G.L << G.logn, ypw = blk;
  unsigned nid = 0;
  for (unsigned j = 0; j < r.count; j++)
    nid = std::max(nid, (unsigned)r.out[j].idx + 1);
  const SdCtx &c = g_sd_ctx;
  auto ptr = [&](const SdRole &q) -> const uint64_t * {
    if (q.kind == SR_OUT)
      return q.idx < nid ? g_sd.scratch + q.idx * blk : nullptr;
    if (q.kind == SR_Y)
      return q.idx < c.ny ? c.y[q.idx] + q.poly * ypw : nullptr;
    return q.idx < c.ne ? c.e[q.idx][q.poly] : nullptr;
  };
  if (g_sd.swords < nid * blk) {
    pool_free(g_sd.scratch);  // stream-ordered: its last reader was launched before
    g_sd.scratch = (uint64_t *)pool_alloc(nid * blk * 8);
    g_sd.swords = nid * blk;
  }
  if (g_sd.cwords < ((size_t)r.nl << G.logn)) {
    pool_free(g_sd.cws);
    g_sd.cws = (uint64_t *)pool_alloc(((size_t)r.nl << G.logn) * 8);
    g_sd.cwords = (size_t)r.nl << G.logn;
  }
  EwProg p{};
  p.count = r.count;
  for (unsigned j = 0; j < r.count; j++) {
    const bool hb = r.kind[j] == EW_ADD || r.kind[j] == EW_SUB || r.kind[j] == EW_DEC;
    const uint64_t *a = ptr(r.a[j]), *b = hb ? ptr(r.b[j]) : nullptr;
    if (!a || (hb && !b) || r.out[j].idx >= nid)
      return;
    p.op[j] = EwOp{g_sd.scratch + r.out[j].idx * blk, a, b, r.kind[j] == EW_DEC ? r.sk : nullptr, r.kind[j], r.lvl[j]};
  }
  const size_t zb = (size_t)r.slots * 16;
  if (g_sd.zbytes < zb) {
    if (g_sd.ev)
      HIP_CHECK(hipEventSynchronize(g_sd.ev));  // (an earlier replay may still write it)
    if (g_sd.z)
      HIP_CHECK(hipHostFree(g_sd.z));
    HIP_CHECK(hipHostMalloc(&g_sd.z, zb, hipHostMallocDefault));
    g_sd.zbytes = zb;
  }
  void *zd = nullptr;
  HIP_CHECK(hipHostGetDevicePointer(&zd, g_sd.z, 0));
  if (!g_sd.ev)
    HIP_CHECK(hipEventCreateWithFlags(&g_sd.ev, hipEventDisableTiming));
  k_ew_decode(p, (double *)zd, g_sd.scratch + r.sid * blk, r.nl, r.slots, r.scale, g_sd.cws);
  HIP_CHECK(hipEventRecord(g_sd.ev, G.stream));
  g_sd.pat = r;
  g_sd.valid = true;
}

static bool sd_on()
{
  static const bool on = env_u("GPQHE_SPEC_DCD", 1) != 0;
  return on && !g_sd_off;
}

static void prov_forget(const void *obj_data, size_t pstride_words)
{
  if (g_prov.empty() || !obj_data)
    return;
  g_prov.erase((const uint64_t *)obj_data);
  g_prov.erase((const uint64_t *)obj_data + pstride_words);
}

// he_gemv is queued the same way (at most two, run as one batch: the two
// independent products of every control step of the caller, reference
// src/hempc.c:255-262).  At any time only one of the two queues is non-empty:
// he_gemv runs the encode/encrypt queue before queueing, and a deferred
// encode / encryption runs the gemv queue first.
struct PendGemv {
  uint64_t *y;
  size_t ypstride;
  const uint64_t *x0, *x1;
  const void *xdata;
  unsigned lvl;
  std::vector<GemvDiags> dgs;  // launches of up to GemvDiags::MAX diagonals; empty: all-zero matrix
  const uint64_t *dspec = nullptr;  // x1's ModUp digits, precomputed (SpecModup), or null
  // x = a - b is a queued he_sub (ew_lazy_sub): its polys a0 - b0, a1 - b1,
  // formed where the inner products read them; null otherwise
  const uint64_t *la0 = nullptr, *lb0 = nullptr, *la1 = nullptr, *lb1 = nullptr;
};
static std::vector<PendGemv> g_pgemv;

// The elementwise calls of a control step (he_sub x2 before the gemvs; he_add,
// he_neg, he_copy_ct, he_add after them, src/hempc.c:253-266; he_dec,
// src/ctr.c:486) are queued too and run as one ew_prog_kernel launch per run
// (kernels.hip).  The queue keeps call order element by element, so a freed
// object's block may be handed out again while queued ops still name it:
// every writer outside this queue flushes it first.  The three queues are
// never non-empty at once.
static EwProg g_pew{};

static void flush_pending();
static void flush_gemvs();
static unsigned env_u(const char *name, unsigned dflt);
static bool g_spec_early = false;  // the next step's speculation rides on this step's gemv / ModDown (spec_attach)

static void flush_ew()
{
  if (!g_pew.count)
    return;
  const EwProg p = g_pew;
  g_pew.count = 0;
  k_ew_prog(p);
}

static void check_ctx()
{
  if (!G.init)
    gpqhe_die("context not initialised (hectx_init)");
  // a non-queued entry point: it may write any object (C1Prov)
  g_prov.clear();
  g_smu.valid = false;
  g_smu_next.pending = false;
  g_sd.valid = false;
  flush_ew();
  if (!g_pgemv.empty())
    flush_gemvs();
  if (!g_pecd.empty() || !g_penc.empty())
    flush_pending();
}

static inline he_ct_t *OB(void *o) { return (he_ct_t *)o; }
static inline const he_ct_t *OB(const void *o) { return (const he_ct_t *)o; }

static inline uint64_t *limb(const void *vo, unsigned p, unsigned l)
{
  const he_ct_t *o = OB(vo);
  return o->data + (((size_t)p * o->cap + l) << G.logn);
}

static inline size_t pstride(const void *vo)
{
  return (size_t)OB(vo)->cap << G.logn;
}

static LimbSet limbset(uint64_t *base, const unsigned *mods, unsigned per, unsigned groups, size_t stride)
{
  LimbSet s{};
  s.base = base;
  s.per = per;
  s.count = per * groups;
  s.stride = stride;
  for (unsigned i = 0; i < per; i++)
    s.mods[i] = (uint8_t)mods[i];
  return s;
}

static LimbSet qlimbs(uint64_t *base, unsigned lvl, unsigned groups, size_t stride)
{
  unsigned mods[GPQHE_MAXMOD];
  for (unsigned i = 0; i < lvl; i++)
    mods[i] = i;
  return limbset(base, mods, lvl, groups, stride);
}

static unsigned basis_qp(unsigned lvl, unsigned *mods)
{
  for (unsigned t = 0; t < lvl; t++)
    mods[t] = t;
  for (unsigned k = 0; k < G.K; k++)
    mods[lvl + k] = G.L + k;
  return lvl + G.K;
}

static void obj_alloc(void *vo, unsigned npoly, unsigned cap)
{
  // no flush of the queued work: a fresh block cannot alias a live object
  // that queued work refers to (objects are flushed before they are freed)
  if (!G.init)
    gpqhe_die("context not initialised (hectx_init)");
  he_ct_t *o = OB(vo);
  memset(o, 0, sizeof(*o));
  o->npoly = npoly;
  o->cap = cap;
  const size_t bytes = ((size_t)npoly * cap << G.logn) * 8;
  // No zero fill: a fresh object has nlimbs = 0, and every read of an object
  // is bounded by its nlimbs, so its payload is written before it is read.
  o->data = (uint64_t *)pool_alloc(bytes);
  prov_forget(o->data, (size_t)cap << G.logn);
}

// Freeing the target of a queued encode that no other queued work reads
// (HECTR frees its five plaintexts right after encrypting them, src/ctr.c:
// 476-480; the queued encryptions take the coefficients, not the payload):
// the encode is dropped instead of flushing the queue.  True if so.
static bool drop_dead_encode(const uint64_t *data)
{
  if (!data || !g_pgemv.empty() || g_pew.count)
    return false;
  bool target = false;
  for (const PendEcd &e : g_pecd)
    target |= e.dst == data;
  if (!target)
    return false;
  for (const PendEnc &e : g_penc)
    if (e.c0 == data || e.c1 == data || e.pk0 == data || e.pk1 == data || (e.m == data && e.ecd < 0))
      return false;
  for (PendEcd &e : g_pecd)
    if (e.dst == data)
      e.dst = nullptr;
  return true;
}

// Every queued encode dropped (its plaintext freed) and the queued
// encryptions are exactly the speculated ones (SpecNoise): they run now --
// only the combine, from the speculative noise and the plaintexts'
// coefficients -- so it overlaps the caller's host work up to its next call
// that needs them (HECTR's horizon matrices in ctr_hempc, src/hempc.c:225-240)
// instead of starting at that call.  GPQHE_SPEC_EARLY=0: at that call.
static void spec_gemv_launch(const std::vector<PendEnc> &enc, const std::vector<SgRec> &recs);

static void spec_flush_early()
{
  static const bool on = env_u("GPQHE_SPEC_EARLY", 1) != 0;
  if (!on || !g_spec.valid || g_penc.empty() || g_penc.size() != g_spec.k || !g_pgemv.empty() || g_pew.count ||
      g_penc[0].stream != g_spec.base || g_penc[0].lvl != g_spec.lvl)
    return;
  for (const PendEcd &e : g_pecd)
    if (e.dst)
      return;
  const std::vector<PendEnc> enc = g_penc;
  const std::vector<SgRec> recs = g_sg_next;  // the last step's gemvs (flush_pending starts a new record)
  flush_pending();
  spec_gemv_launch(enc, recs);
}

static void obj_free(void *vo)
{
  // a queued encode / encryption / gemv may still use the payload (queued
  // elementwise ops keep their order with any later user of the block)
  bool dropped = false;
  if (G.init && (!g_pgemv.empty() || !g_pecd.empty() || !g_penc.empty())) {
    dropped = drop_dead_encode(OB(vo)->data);
    if (!dropped)
      check_ctx();
  }
  he_ct_t *o = OB(vo);
  if (o->data && G.init) {
    prov_forget(o->data, (size_t)o->cap << G.logn);
    const uint64_t *lo = o->data, *hi = o->data + ((size_t)o->npoly * o->cap << G.logn);
    if (g_smu.pk1 >= lo && g_smu.pk1 < hi)
      g_smu.valid = false;  // the speculative ModUp's public key
    if (g_smu_next.pk1 >= lo && g_smu_next.pk1 < hi)
      g_smu_next.pending = false;  // (its pending launch reads it)
    if (g_spec_pk1_next >= lo && g_spec_pk1_next < hi)
      g_spec_pats_next.clear();
    if (g_pew.count) {
      // queued elementwise ops writing this block while no queued op reads it:
      // their results can never be read, so they are dropped (HECTR's xdiff
      // and udiff, src/hempc.c:269-270, once he_gemv read their operands)
      auto in = [&](const uint64_t *p) { return p && p >= lo && p < hi; };
      bool read = false;
      for (unsigned j = 0; j < g_pew.count; j++)
        read |= in(g_pew.op[j].a) || in(g_pew.op[j].b) || in(g_pew.op[j].s);
      if (!read) {
        unsigned w = 0;
        for (unsigned j = 0; j < g_pew.count; j++)
          if (!in(g_pew.op[j].out))
            g_pew.op[w++] = g_pew.op[j];
        g_pew.count = w;
      }
    }
    pool_free(o->data);
  }
  memset(o, 0, sizeof(*o));
  if (dropped)
    spec_flush_early();
}

static uint64_t next_stream()
{
  return G.counter++;
}

static void sample_small_ntt(uint64_t *dst, const unsigned *mods, unsigned nm, int cbd)
{
  LimbSet s = limbset(dst, mods, nm, 1, (size_t)nm << G.logn);
  k_sample_small(s, next_stream(), cbd);
  k_ntt(s, false);
}

static void sample_uniform(uint64_t *dst, const unsigned *mods, unsigned nm)
{
  LimbSet s = limbset(dst, mods, nm, 1, (size_t)nm << G.logn);
  k_sample_uniform(s, next_stream());
}

// ===========================================================================
// MPI
// ===========================================================================
struct gpqhe_mpi {
  unsigned nwords;
  uint64_t w[64];
};

extern "C" MPI gpqhe_mpi_set_ui(MPI w, unsigned long u)
{
  if (!w)
    w = (MPI)calloc(1, sizeof(*w));
  memset(w->w, 0, sizeof(w->w));
  w->w[0] = u;
  w->nwords = 1;
  return w;
}

extern "C" void gpqhe_mpi_lshift(MPI x, MPI a, unsigned int n)
{
  uint64_t src[64], dst[64];
  memcpy(src, a->w, sizeof(src));
  memset(dst, 0, sizeof(dst));
  const unsigned ws = n / 64, bs = n % 64;
  for (int i = 63; i >= 0; i--) {
    const int s = i - (int)ws;
    if (s < 0)
      continue;
    uint64_t v = src[s] << bs;
    if (bs && s > 0)
      v |= src[s - 1] >> (64 - bs);
    dst[i] = v;
  }
  memcpy(x->w, dst, sizeof(dst));
  x->nwords = 64;
}

extern "C" void gpqhe_mpi_release(MPI a)
{
  free(a);
}

extern "C" unsigned gpqhe_mpi_get_nbits(MPI a)
{
  for (int i = 63; i >= 0; i--)
    if (a->w[i])
      return (unsigned)(i * 64 + 64 - __builtin_clzll(a->w[i]));
  return 0;
}

// ===========================================================================
// Context
// ===========================================================================
static void set_seed_words(uint64_t seed)
{
  uint64_t z = seed;
  for (int i = 0; i < 4; i++) {
    z += 0x9E3779B97F4A7C15ull;
    const uint64_t x = splitmix64_mix(z);
    G.key.k[2 * i] = (uint32_t)x;
    G.key.k[2 * i + 1] = (uint32_t)(x >> 32);
  }
  G.counter = 0;
  g_spec.valid = false;  // noise of the old key
  g_smu.valid = false;
  g_smu_next.pending = false;
}

extern "C" void gpqhe_set_seed(uint64_t seed)
{
  if (G.init)
    check_ctx();  // queued encryptions sample with the current key
  set_seed_words(seed);
}

static uint64_t default_seed()
{
  const char *e = getenv("GPQHE_SEED");
  if (e && *e)
    return strtoull(e, nullptr, 0);
  uint64_t s = 0;
  FILE *f = fopen("/dev/urandom", "rb");
  if (!f || fread(&s, sizeof(s), 1, f) != 1)
    gpqhe_die("cannot read /dev/urandom");
  fclose(f);
  return s;
}

extern "C" void hectx_init_params(const gpqhe_params_t *p)
{
  if (G.init)
    hectx_exit();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    gpqhe_die("no HIP device visible: libgpqhe.so runs on MI355X only (no CPU fallback)");
  if (p->logn < 4 || p->logn > 17)
    gpqhe_die("logn %u out of range [4, 17]", p->logn);
  if (p->nlimbs < 1 || p->nspecial < 1 || p->nlimbs + p->nspecial > GPQHE_MAXMOD)
    gpqhe_die("bad limb counts L=%u K=%u", p->nlimbs, p->nspecial);
  if (p->q0_bits > 61 || p->qi_bits > 61 || p->p_bits > 61 || p->q0_bits < 32 || p->qi_bits < 32 ||
      p->p_bits < 32)
    gpqhe_die("prime sizes must be within [32, 61] bits");
  Context &C = G;
  C.logn = p->logn;
  C.n = 1u << p->logn;
  C.L = p->nlimbs;
  C.K = p->nspecial;
  C.nmod = C.L + C.K;
  C.dnum = p->dnum ? p->dnum : p->nlimbs;
  if (C.dnum > C.L)
    C.dnum = C.L;
  C.alpha = (C.L + C.dnum - 1) / C.dnum;
  C.dnum = (C.L + C.alpha - 1) / C.alpha;
  C.slots = p->slots ? p->slots : C.n / 2;
  if ((C.slots & (C.slots - 1)) || C.slots > C.n / 2)
    gpqhe_die("slots %u must be a power of two <= n/2", C.slots);
  C.delta = p->delta;
  const uint64_t two_n = 2ull * C.n;
  unsigned used = 0;
  C.q[used] = hm_pick_prime(p->q0_bits, two_n, C.q, used);
  used++;
  for (unsigned i = 1; i < C.L; i++, used++)
    C.q[used] = hm_pick_prime(p->qi_bits, two_n, C.q, used);
  for (unsigned i = 0; i < C.K; i++, used++)
    C.q[used] = hm_pick_prime(p->p_bits, two_n, C.q, used);
  for (unsigned m = 0; m < C.nmod; m++) {
    hm_modconst(C.mc[m], C.q[m]);
    C.psi[m] = hm_find_psi(C.q[m], C.n);
    C.mc[m].ninv = hm_inv_mod(C.n, C.q[m]);
    C.mc[m].ninvp = (uint64_t)(((unsigned __int128)C.mc[m].ninv << 64) / C.q[m]);
    uint64_t pm = 1;
    for (unsigned k = 0; k < C.K; k++)
      pm = hm_mul_mod(pm, C.q[C.L + k] % C.q[m], C.q[m]);
    C.mc[m].pmod = pm;
    C.mc[m].pmodp = (uint64_t)(((unsigned __int128)pm << 64) / C.q[m]);
  }
  HIP_CHECK(hipGetDevice(&C.device));
  (void)hipGetLastError();  // start from a clean error state
  if (!C.own_stream)
    HIP_CHECK(hipStreamCreateWithFlags(&C.own_stream, hipStreamNonBlocking));
  if (!C.stream)
    C.stream = C.own_stream;
  tables_upload();
  set_seed_words(p->seed ? p->seed : default_seed());
  C.init = true;
  tables_prewarm();
}

static unsigned env_u(const char *name, unsigned dflt)
{
  const char *e = getenv(name);
  return (e && *e) ? (unsigned)strtoul(e, nullptr, 0) : dflt;
}

// GPQHE_HOSTPROF=1: host time spent inside each entry point the small-N
// control step uses (outermost calls only) and between calls (the caller's
// own work), printed to stderr by hectx_exit.  Measurement aid only.
struct HostProfEntry {
  double us = 0;
  unsigned long calls = 0;
};
static std::map<std::string, HostProfEntry> g_hp;
static double g_hp_outside = 0, g_hp_last = -1;
// GPQHE_HOSTPROF=2 also keeps every outermost call (name, start, end) and
// prints one steady-state control step's calls relative to the end of the
// decode before it (the caller's host timeline between two decodes)
struct HpEvent {
  const char *name;
  double t0, t1;
};
static std::vector<HpEvent> g_hp_ev;
static int g_hp_depth = 0;
static double hp_now()
{
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static bool hp_on()
{
  static const bool on = env_u("GPQHE_HOSTPROF", 0) != 0;
  return on;
}
struct HpScope {
  const char *name;
  double t0 = 0;
  bool top = false;
  explicit HpScope(const char *nm) : name(nm)
  {
    if (!hp_on())
      return;
    top = g_hp_depth++ == 0;
    if (top) {
      t0 = hp_now();
      if (g_hp_last >= 0)
        g_hp_outside += t0 - g_hp_last;
    }
  }
  ~HpScope()
  {
    if (!hp_on())
      return;
    g_hp_depth--;
    if (top) {
      g_hp_last = hp_now();
      HostProfEntry &e = g_hp[name];
      e.us += g_hp_last - t0;
      e.calls++;
      static const bool ev = env_u("GPQHE_HOSTPROF", 0) >= 2;
      if (ev && g_hp_ev.size() < 100000)
        g_hp_ev.push_back(HpEvent{name, t0, g_hp_last});
    }
  }
};
#define HPROF(nm) HpScope hp_scope_(nm)

static void hp_report()
{
  if (!hp_on() || g_hp.empty())
    return;
  double in = 0;
  for (auto &kv : g_hp)
    in += kv.second.us;
  fprintf(stderr, "[gpqhe hostprof] inside the library %.1f us, outside (caller) %.1f us\n", in, g_hp_outside);
  for (auto &kv : g_hp)
    fprintf(stderr, "[gpqhe hostprof] %-12s %8lu calls %10.1f us %8.2f us/call\n", kv.first.c_str(), kv.second.calls,
            kv.second.us, kv.second.us / (double)kv.second.calls);
  // the calls after the (ndcd/2)-th decode up to and including the next one
  std::vector<size_t> dcd;
  for (size_t i = 0; i < g_hp_ev.size(); i++)
    if (!strcmp(g_hp_ev[i].name, "dcd"))
      dcd.push_back(i);
  if (dcd.size() >= 4) {
    const size_t a = dcd[dcd.size() / 2], b = dcd[dcd.size() / 2 + 1];
    const double t = g_hp_ev[a].t1;
    fprintf(stderr, "[gpqhe hostprof] one step, us after the decode before it returned: start end name\n");
    for (size_t i = a + 1; i <= b; i++)
      fprintf(stderr, "[gpqhe hostprof] %8.1f %8.1f %s\n", g_hp_ev[i].t0 - t, g_hp_ev[i].t1 - t, g_hp_ev[i].name);
  }
  g_hp_ev.clear();
  g_hp.clear();
  g_hp_outside = 0;
  g_hp_last = -1;
}

extern "C" void hectx_init(unsigned int logn, MPI q, unsigned int slots, uint64_t Delta)
{
  gpqhe_params_t p;
  memset(&p, 0, sizeof(p));
  const unsigned logq = gpqhe_mpi_get_nbits(q) - 1;
  const unsigned logd = 63 - (unsigned)__builtin_clzll(Delta);
  p.logn = env_u("GPQHE_LOGN", logn);
  p.slots = slots;
  p.delta = (double)Delta;
  p.qi_bits = logd;
  p.nspecial = 1;
  p.p_bits = 60;
  unsigned L = env_u("GPQHE_NLIMBS", 0);
  if (L) {
    p.nlimbs = L;
    p.q0_bits = 60;
  } else {
    L = 2;
    while (logq > (L - 1) * logd + 61)
      L++;
    p.nlimbs = L;
    p.q0_bits = logq - (L - 1) * logd;
  }
  p.dnum = env_u("GPQHE_DNUM", p.nlimbs);
  p.seed = 0;
  hectx_init_params(&p);
}

void gemv_cache_clear();

extern "C" void hectx_exit(void)
{
  if (!G.init)
    return;
  hp_report();
  check_ctx();
  HIP_CHECK(hipStreamSynchronize(G.stream));
  // every HIP object the engine created goes here, after its last use: the
  // second sub-chunk stream and its events, the decode event, the profiling
  // events and (below, with the pool) the context's own stream
  if (g_s2.s) {
    HIP_CHECK(hipStreamSynchronize(g_s2.s));
    HIP_CHECK(hipEventDestroy(g_s2.fork));
    HIP_CHECK(hipEventDestroy(g_s2.d2));
    HIP_CHECK(hipEventDestroy(g_s2.join));
    HIP_CHECK(hipStreamDestroy(g_s2.s));
    g_s2 = SecondStream{};
  }
  if (g_dcd_ev) {
    HIP_CHECK(hipEventDestroy(g_dcd_ev));
    g_dcd_ev = nullptr;
  }
  if (g_sd.ev)
    HIP_CHECK(hipEventDestroy(g_sd.ev));
  if (g_sd.z)
    HIP_CHECK(hipHostFree(g_sd.z));
  g_sd = SpecDcd{};  // (its scratch blocks go with the pool)
  g_sd_ctx = SdCtx{};
  g_sd_next_ok = false;
  g_sd_taken = g_sd_late = 0;
  g_sd_off = false;
  k_prof_release();
  gemv_cache_clear();
  fold_cache_clear();
  g_key_gen++;
  tables_free();
  g_spec = SpecNoise{};  // its blocks go with the pool
  g_spec_next_k = 0;
  g_smu = SpecModup{};
  g_smu_next = SpecModupNext{};
  g_sa = SpecAttach{};
  g_sg = SpecGemv{};
  g_sg_next.clear();
  g_sg_taken = 0;
  g_prov.clear();
  g_spec_pats_next.clear();
  g_spec_pk1_next = nullptr;
  pool_release_all();
  stage_release();
  if (G.own_stream) {
    HIP_CHECK(hipStreamDestroy(G.own_stream));
    if (G.stream == G.own_stream)
      G.stream = nullptr;  // (a caller's stream from gpqhe_set_stream stays set)
    G.own_stream = nullptr;
  }
  G.init = false;
}

extern "C" void hectx_info(gpqhe_info_t *info)
{
  check_ctx();
  memset(info, 0, sizeof(*info));
  info->logn = G.logn;
  info->n = G.n;
  info->nlimbs = G.L;
  info->nspecial = G.K;
  info->dnum = G.dnum;
  info->alpha = G.alpha;
  info->slots = G.slots;
  info->delta = G.delta;
  for (unsigned m = 0; m < G.nmod; m++) {
    info->primes[m] = G.q[m];
    info->psi[m] = G.psi[m];
  }
}

extern "C" void gpqhe_set_stream(void *stream)
{
  if (G.init)
    check_ctx();
  if (G.stream)
    HIP_CHECK(hipStreamSynchronize(G.stream));
  G.stream = stream ? (hipStream_t)stream : G.own_stream;
}

extern "C" void gpqhe_sync(void)
{
  if (G.init)
    check_ctx();
  if (G.stream)
    HIP_CHECK(hipStreamSynchronize(G.stream));
}

// ===========================================================================
// Objects
// ===========================================================================
extern "C" void he_alloc_pk(he_pk_t *pk) { obj_alloc(pk, 2, G.L); }
extern "C" void he_free_pk(he_pk_t *pk) { obj_free(pk); }
extern "C" void he_alloc_sk(poly_mpi_t *sk) { obj_alloc(sk, 1, G.nmod); }
extern "C" void he_free_sk(poly_mpi_t *sk) { obj_free(sk); }
extern "C" void he_alloc_ct(he_ct_t *ct)
{
  HPROF("alloc_ct");
  obj_alloc(ct, 2, G.L);
}
extern "C" void he_free_ct(he_ct_t *ct)
{
  HPROF("free_ct");
  obj_free(ct);
}
extern "C" void he_alloc_pt(he_pt_t *pt)
{
  HPROF("alloc_pt");
  obj_alloc(pt, 1, G.nmod);
}
extern "C" void he_free_pt(he_pt_t *pt)
{
  HPROF("free_pt");
  obj_free(pt);
}

extern "C" void he_alloc_evk(he_evk_t *evk)
{
  check_ctx();
  memset(evk, 0, sizeof(*evk));
}

// Montgomery-form shadow of a key (x 2^64 mod q), kept in `reserved`, used by
// the fused key-switch inner product.  Exported/imported keys stay canonical.
static void evk_make_mont(he_evk_t *evk)
{
  const size_t words = ((size_t)evk->npoly * evk->cap) << G.logn;
  uint64_t *m = (uint64_t *)(uintptr_t)evk->reserved;
  if (!m)
    m = (uint64_t *)pool_alloc(words * 8);
  k_to_mont(m, evk->data, evk->npoly * evk->cap);
  evk->reserved = (uint64_t)(uintptr_t)m;
}

extern "C" void he_free_evk(he_evk_t *evk)
{
  g_key_gen++;
  if (evk->reserved && G.init)
    pool_free((void *)(uintptr_t)evk->reserved);
  obj_free(evk);
}

extern "C" size_t he_export(const void *vo, uint64_t *host)
{
  check_ctx();
  const he_ct_t *o = OB(vo);
  const size_t n = G.n;
  HIP_CHECK(hipStreamSynchronize(G.stream));
  size_t w = 0;
  for (unsigned p = 0; p < o->npoly; p++) {
    HIP_CHECK(hipMemcpy(host + w, limb(o, p, 0), (size_t)o->nlimbs * n * 8, hipMemcpyDeviceToHost));
    w += (size_t)o->nlimbs * n;
  }
  return w;
}

extern "C" void he_import(void *vo, const uint64_t *host, unsigned int nlimbs, double scale, uint32_t flags)
{
  check_ctx();
  he_ct_t *o = OB(vo);
  if (!o->data) {
    const uint32_t g = o->galois, dn = o->dnum;
    if (!dn || dn != G.dnum)
      gpqhe_die("he_import into an unallocated object (evk needs dnum=%u)", G.dnum);
    obj_alloc(o, 2 * dn, G.nmod);
    o->galois = g;
    o->dnum = dn;
  }
  if (nlimbs > o->cap)
    gpqhe_die("he_import: %u limbs > capacity %u", nlimbs, o->cap);
  HIP_CHECK(hipStreamSynchronize(G.stream));
  size_t w = 0;
  for (unsigned p = 0; p < o->npoly; p++) {
    HIP_CHECK(hipMemcpy(limb(o, p, 0), host + w, (size_t)nlimbs * G.n * 8, hipMemcpyHostToDevice));
    w += (size_t)nlimbs * G.n;
  }
  o->nlimbs = nlimbs;
  o->scale = scale;
  o->flags = flags;
  if (o->dnum && o->npoly == 2 * o->dnum && o->cap == G.nmod) {
    g_key_gen++;
    evk_make_mont((he_evk_t *)o);  // key objects keep their Montgomery shadow in sync
  }
}

extern "C" void he_evk_meta(const he_evk_t *evk, uint32_t *galois, uint32_t *dnum)
{
  *galois = evk->galois;
  *dnum = evk->dnum;
}

// ===========================================================================
// Keys
// ===========================================================================
extern "C" void he_keypair(he_pk_t *pk, poly_mpi_t *sk)
{
  check_ctx();
  unsigned mods[GPQHE_MAXMOD];
  for (unsigned m = 0; m < G.nmod; m++)
    mods[m] = m;
  sample_small_ntt(sk->data, mods, G.nmod, 0);  // s: ternary over all moduli
  sk->nlimbs = G.nmod;
  sample_uniform(limb(pk, 1, 0), mods, G.L);     // a
  Ws e((size_t)G.L << G.logn);
  sample_small_ntt(e.p, mods, G.L, 1);           // e
  k_enc_sk_combine(limb(pk, 0, 0), limb(pk, 1, 0), e.p, sk->data, nullptr, G.L);  // -a s + e
  pk->nlimbs = G.L;
}

static void gen_evk(he_evk_t *evk, const uint64_t *sprime, const poly_mpi_t *sk, uint32_t galois)
{
  g_key_gen++;
  if (evk->data)
    he_free_evk(evk);
  obj_alloc(evk, 2 * G.dnum, G.nmod);
  evk->nlimbs = G.nmod;
  evk->galois = galois;
  evk->dnum = G.dnum;
  unsigned mods[GPQHE_MAXMOD];
  for (unsigned m = 0; m < G.nmod; m++)
    mods[m] = m;
  Ws e((size_t)G.nmod << G.logn);
  for (unsigned j = 0; j < G.dnum; j++) {
    sample_uniform(limb(evk, 2 * j + 1, 0), mods, G.nmod);
    sample_small_ntt(e.p, mods, G.nmod, 1);
    const unsigned lo = j * G.alpha, hi = std::min(lo + G.alpha, G.L);
    k_evk_combine(limb(evk, 2 * j, 0), limb(evk, 2 * j + 1, 0), e.p, sk->data, sprime, lo, hi);
  }
  evk_make_mont(evk);
}

static uint64_t galois_of_rot(unsigned r)
{
  return hm_pow_mod(5, r, 2ull * G.n);
}

static void gen_rot_key(he_evk_t *evk, uint64_t g, const poly_mpi_t *sk)
{
  Ws sp((size_t)G.nmod << G.logn);
  k_automorph(sp.p, sk->data, G.nmod, g);
  gen_evk(evk, sp.p, sk, (uint32_t)g);
}

extern "C" void he_genrk(he_evk_t rk[], const poly_mpi_t *sk)
{
  check_ctx();
  if (rk[0].data)
    obj_free(&rk[0]);
  rk[0].galois = 1;
  for (unsigned r = 1; r < G.slots; r++)
    gen_rot_key(&rk[r], galois_of_rot(r), sk);
}

extern "C" void he_genrot(he_evk_t *evk, unsigned int rot, const poly_mpi_t *sk)
{
  check_ctx();
  gen_rot_key(evk, galois_of_rot(rot), sk);
}

extern "C" void he_genrlk(he_evk_t *rlk, const poly_mpi_t *sk)
{
  check_ctx();
  Ws s2((size_t)G.nmod << G.logn);
  k_square(s2.p, sk->data, G.nmod);
  gen_evk(rlk, s2.p, sk, 1);
}

// ===========================================================================
// Encoding / encryption
// ===========================================================================
// Encode z at `scale` into `dst` limbs for moduli mods[0..nm) (NTT domain).
// Slot counts from which the special FFT runs on the GPU (GPQHE_GPU_ECD_MIN;
// below it the host FFT plus one upload has the lower latency, e.g. HECTR's
// 16-32 slots).
static unsigned gpu_ecd_min()
{
  static const unsigned m = env_u("GPQHE_GPU_ECD_MIN", 2048);
  return m;
}

// Deferral applies to host-FFT encodes at n <= 2^12 (the whole-limb NTT
// lifts in-kernel) into q limbs 0..lvl-1.
static bool defer_ok(unsigned s)
{
  static const bool on = env_u("GPQHE_DEFER", 1) != 0;
  return on && G.logn <= 12 && G.logn >= 10 && s < gpu_ecd_min();
}

static void flush_pending()
{
  std::vector<PendEcd> ecd;
  std::vector<PendEnc> enc;
  std::vector<int64_t> vals;
  ecd.swap(g_pecd);
  enc.swap(g_penc);
  if (!ecd.empty() || !enc.empty())
    g_sd.valid = false;  // (its outputs may take blocks the replayed tail read: SpecDcd)
  vals.swap(g_pcoef);
  const size_t n = G.n;
  // an encoding of s slots is zero off the stride n / 2s: the launches take
  // one row of the coefficients on the widest stride every queued encode
  // shares (value j = coefficient j 2^clog)
  unsigned clog = G.logn;
  for (const PendEcd &e : ecd)
    clog = std::min(clog, (unsigned)__builtin_ctz(G.n / (2 * e.slots)));
  const size_t row = n >> clog;
  std::vector<int64_t> coef(ecd.size() * row);
  for (size_t i = 0; i < ecd.size(); i++) {
    const size_t step = (n / (2 * ecd[i].slots)) >> clog;
    for (size_t t = 0; t < 2 * (size_t)ecd[i].slots; t++)
      coef[i * row + t * step] = vals[ecd[i].coff + t];
  }
  // a device-readable copy of the rows, made when a launch needs more values
  // than travel in its arguments: up to 64 KB the kernels read pinned host
  // memory, more is uploaded
  const size_t cbytes = ecd.size() * row * 8;
  Ws up(0);
  Stage *st = nullptr;
  const int64_t *dcoef = nullptr;
  auto dev_coef = [&]() {
    if (!dcoef) {
      if (cbytes <= 65536) {
        const void *dmap = nullptr;
        st = &stage_map(coef.data(), cbytes, &dmap);
        dcoef = (const int64_t *)dmap;
      } else {
        up.p = (uint64_t *)pool_alloc(cbytes);
        upload(up.p, coef.data(), cbytes);
        dcoef = (const int64_t *)up.p;
      }
    }
    return dcoef;
  };
  // the encodes whose plaintext still lives (dropped ones: drop_dead_encode)
  for (size_t i0 = 0; i0 < ecd.size();) {
    if (!ecd[i0].dst) {
      i0++;
      continue;
    }
    // one launch per run of live encodes at equal levels (at most GPQHE_MAXGRP)
    size_t i1 = i0 + 1;
    while (i1 < ecd.size() && i1 - i0 < GPQHE_MAXGRP && ecd[i1].dst && ecd[i1].lvl == ecd[i0].lvl)
      i1++;
    unsigned mods[GPQHE_MAXMOD];
    for (unsigned l = 0; l < ecd[i0].lvl; l++)
      mods[l] = l;
    LimbSet ls = limbset(nullptr, mods, ecd[i0].lvl, (unsigned)(i1 - i0), 0);
    ls.ngp = (uint32_t)(i1 - i0);
    for (size_t i = i0; i < i1; i++) {
      ls.gp[i - i0] = ecd[i].dst;
      g_prov.erase(ecd[i].dst);
    }
    // up to CoefArg::MAX values (HECTR's step: 5 x 32) in the kernel arguments
    if ((i1 - i0) * row <= CoefArg::MAX)
      k_lift_ntt_arg(ls, coef.data() + i0 * row, clog);
    else
      k_lift_ntt(ls, dev_coef() + i0 * row, clog);
    i0 = i1;
  }
  for (size_t i0 = 0; i0 < enc.size();) {
    // a run of encryptions at one level with consecutive RNG streams and the
    // same public key
    size_t i1 = i0 + 1;
    while (i1 < enc.size() && i1 - i0 < GPQHE_MAXGRP && enc[i1].lvl == enc[i0].lvl &&
           enc[i1].stream == enc[i0].stream + 3 * (i1 - i0) && enc[i1].pk0 == enc[i0].pk0)
      i1++;
    const unsigned k = (unsigned)(i1 - i0), lvl = enc[i0].lvl;
    const size_t w = (size_t)lvl << G.logn;
    unsigned mods[GPQHE_MAXMOD];
    for (unsigned l = 0; l < lvl; l++)
      mods[l] = l;
    EncBatch b{};
    for (unsigned e = 0; e < k; e++) {
      b.c0[e] = enc[i0 + e].c0;
      b.c1[e] = enc[i0 + e].c1;
      b.m[e] = enc[i0 + e].ecd >= 0 ? nullptr : enc[i0 + e].m;
    }
    if (i0 == 0 && i1 == enc.size()) {
      g_spec_next_k = k;
      g_spec_next_lvl = lvl;
      g_step_base = enc[i0].stream;
    } else {
      g_spec_next_k = 0;
    }
    if (i0 == 0) {
      g_spec_pats_next.clear();  // a new step: its gemv inputs are recorded afresh
      g_sg_next.clear();
      g_sd_ctx.valid = false;
      g_sd.valid = false;
    }
    for (unsigned e = 0; e < k; e++) {
      g_prov[enc[i0 + e].c1] = C1Prov{enc[i0 + e].stream, 0, enc[i0 + e].pk1, lvl, false};
      g_prov[enc[i0 + e].c0] = C1Prov{enc[i0 + e].stream, 0, enc[i0 + e].pk1, lvl, false, true};
    }
    // the speculative noise of exactly these streams: only the combine runs,
    // with the queued plaintexts evaluated from their coefficients
    const uint64_t off = (enc[i0].stream - g_spec.base) / 3;
    unsigned mrows = 0;
    for (unsigned e = 0; e < k; e++)
      mrows += enc[i0 + e].ecd >= 0;
    if (g_spec.valid && lvl == g_spec.lvl && enc[i0].stream >= g_spec.base &&
        (enc[i0].stream - g_spec.base) % 3 == 0 && off + k <= g_spec.k && row >= 4 && row <= EncM::MAXROW &&
        (size_t)mrows * lvl * row <= EncM::MAX) {
      EncM em{};
      em.row = (uint32_t)row;
      em.clog = clog;
      unsigned r = 0;
      for (unsigned e = 0; e < k; e++) {
        em.row_of[e] = -1;
        const int ei = enc[i0 + e].ecd;
        if (ei < 0)
          continue;
        for (unsigned l = 0; l < lvl; l++) {
          const uint64_t q = G.q[l];
          for (size_t j = 0; j < row; j++) {
            const int64_t c = coef[(size_t)ei * row + j];
            const uint64_t a = c >= 0 ? (uint64_t)c % q : (q - (uint64_t)(-(c + 1)) % q - 1) % q;
            em.v[((size_t)r * lvl + l) * row + j] = a;
          }
        }
        em.row_of[e] = (int32_t)r++;
      }
      k_enc_combine_m(b, em, k, g_spec.buf + off * 3 * w, enc[i0].pk0, enc[i0].pk1, lvl);
      i0 = i1;
      continue;
    }
    // plaintexts that are queued encodes join e0 as coefficients (EncCoef):
    // the combine then reads no NTT-form plaintext
    EncCoef ec{};
    ec.clog = clog;
    ec.row = (uint32_t)row;
    unsigned nrows = 0;
    for (unsigned e = 0; e < k; e++)
      ec.row_of[e] = enc[i0 + e].ecd;
    for (unsigned e = 0; e < k; e++)
      nrows += enc[i0 + e].ecd >= 0;
    if (nrows * row <= EncCoef::MAX) {
      unsigned r = 0;
      for (unsigned e = 0; e < k; e++)
        if (enc[i0 + e].ecd >= 0) {
          memcpy(ec.v + r * row, coef.data() + (size_t)enc[i0 + e].ecd * row, row * 8);
          ec.row_of[e] = (int32_t)r++;
        }
    } else {
      ec.p = dev_coef();
    }
    Ws vee(3 * k * w);
    LimbSet s = limbset(vee.p, mods, lvl, 3 * k, w);
    k_sample_enc(s, enc[i0].stream, 3 * k, nrows ? &ec : nullptr);
    k_ntt(s, false);
    k_enc_combine_batch(b, k, vee.p, enc[i0].pk0, enc[i0].pk1, lvl);
    i0 = i1;
  }
  if (st)
    stage_done(*st);
}

static void encode_limbs(uint64_t *dst, const double *z, unsigned s, double scale, const unsigned *mods,
                         unsigned nm)
{
  Ws dcoef(G.n);
  if (s >= gpu_ecd_min()) {
    Ws work(2 * (size_t)s + 2);
    upload(work.p, z, (size_t)s * 16);
    k_encode_coeffs((int64_t *)dcoef.p, (double *)work.p, s, scale);
  } else {
    std::vector<int64_t> coef(G.n);
    hm_encode_coeffs(coef.data(), z, s, G.n, scale);
    upload(dcoef.p, coef.data(), (size_t)G.n * 8);
  }
  LimbSet ls = limbset(dst, mods, nm, 1, (size_t)nm << G.logn);
  k_lift_ntt(ls, (const int64_t *)dcoef.p);
}

extern "C" void he_ecd_ex(he_pt_t *pt, const gpqhe_complex_t z[], unsigned int slots, double scale,
                          unsigned int nlimbs)
{
  HPROF("ecd");
  if (!G.init)
    gpqhe_die("context not initialised (hectx_init)");
  if (!defer_ok(slots))
    check_ctx();
  if (nlimbs < 1 || nlimbs > G.L)
    gpqhe_die("he_ecd_ex: bad level %u", nlimbs);
  if (defer_ok(slots)) {
    // queued (flush_pending); a plaintext a queued encryption still reads, or
    // a queued encode target, is flushed first
    flush_ew();
    if (!g_pgemv.empty())
      flush_gemvs();
    bool busy = false;
    for (const PendEnc &e : g_penc)
      busy |= e.m == pt->data || e.c0 == pt->data;
    for (const PendEcd &e : g_pecd)
      busy |= e.dst == pt->data;
    if (busy)
      flush_pending();
    if (slots > G.n / 2)
      gpqhe_die("bad slot count %u", slots);
    const size_t at = g_pcoef.size();
    g_pcoef.resize(at + 2 * (size_t)slots);
    hm_encode_slots(g_pcoef.data() + at, (const double *)z, slots, scale);
    g_pecd.push_back({pt->data, nlimbs, slots, at});
  } else {
    unsigned mods[GPQHE_MAXMOD];
    for (unsigned i = 0; i < nlimbs; i++)
      mods[i] = i;
    encode_limbs(pt->data, (const double *)z, slots, scale, mods, nlimbs);
  }
  pt->nlimbs = nlimbs;
  pt->scale = scale;
  pt->flags = 0;
}

extern "C" void he_ecd(he_pt_t *pt, const gpqhe_complex_t z[])
{
  he_ecd_ex(pt, z, G.slots, G.delta, G.L);
}

static void *zpin(size_t bytes)
{
  if (g_zpin_bytes < bytes) {
    if (g_zpin)
      HIP_CHECK(hipHostFree(g_zpin));
    HIP_CHECK(hipHostMalloc(&g_zpin, bytes, hipHostMallocDefault));
    g_zpin_bytes = bytes;
  }
  void *dz = nullptr;
  HIP_CHECK(hipHostGetDevicePointer(&dz, g_zpin, 0));
  return dz;
}

// After the small-N decode (he_dcd_ex): record the decode's end, then launch
// the next step's encryption noise (SpecNoise) if the last flush had one run
// of encryptions.  True if launched (the caller then waits on g_dcd_ev).
static bool spec_launch()
{
  static const bool on = env_u("GPQHE_SPEC", 1) != 0;
  const unsigned k = g_spec_next_k, lvl = g_spec_next_lvl;
  g_smu_next.pending = false;  // superseded
  if (!on || !k || !lvl || k > GPQHE_MAXGRP || !defer_ok(0))
    return false;
  if (!g_dcd_ev)
    HIP_CHECK(hipEventCreateWithFlags(&g_dcd_ev, hipEventDisableTiming));
  HIP_CHECK(hipEventRecord(g_dcd_ev, G.stream));
  const size_t w = (size_t)lvl << G.logn, words = 3 * (size_t)k * w;
  if (g_spec.words != words) {
    pool_free(g_spec.buf);  // stream-ordered: its last reader was launched before
    g_spec.buf = (uint64_t *)pool_alloc(words * 8);
    g_spec.words = words;
  }
  unsigned mods[GPQHE_MAXMOD];
  for (unsigned l = 0; l < lvl; l++)
    mods[l] = l;
  LimbSet s = limbset(g_spec.buf, mods, lvl, 3 * k, w);
  k_sample_enc(s, G.counter, 3 * k);
  k_ntt(s, false);
  g_spec.base = G.counter;
  g_spec.k = k;
  g_spec.lvl = lvl;
  g_spec.valid = true;
  // the gemv inputs of the last step, made from the same encryption slots of
  // this noise: their c1 differences and ModUp (SpecModup)
  g_smu.valid = false;
  const std::vector<SpecPat> &pats = g_spec_pats_next;
  bool ok = !pats.empty() && g_spec_pk1_next && lvl >= 2;
  for (const SpecPat &p : pats)
    ok &= p.oa < k && p.ob < k;
  if (ok) {
    const unsigned np = (unsigned)pats.size(), nm = lvl + G.K, ndig = (lvl + G.alpha - 1) / G.alpha;
    const size_t dw = (size_t)np * ndig * nm << G.logn;
    if (g_smu.dwords != dw) {
      pool_free(g_smu.D);
      g_smu.D = (uint64_t *)pool_alloc(dw * 8);
      g_smu.dwords = dw;
    }
    C1Diffs cd{};
    for (unsigned i = 0; i < np; i++) {
      cd.va[i] = g_spec.buf + (size_t)3 * pats[i].oa * w;
      cd.vb[i] = g_spec.buf + (size_t)3 * pats[i].ob * w;
    }
    k_modup_ntt_diffs(g_smu.D, cd, np, (size_t)ndig * nm << G.logn, g_spec_pk1_next, lvl);
    g_smu.pats = pats;
    g_smu.base = g_spec.base;
    g_smu.pk1 = g_spec_pk1_next;
    g_smu.lvl = lvl;
    g_smu.valid = true;
  }
  return true;
}

// flush_gemvs of a small-N step: the next step's speculation (the same noise
// and ModUp spec_launch runs after the decode) is carried by this step's
// gemv_inner and ModDown launches as extra workgroups (SpecAttach), where it
// uses the CUs those few-workgroup kernels leave idle.  Only when the three
// launches take it: the gemvs in one inner-product launch (one), the noise
// sampling fits its z slice, and the ModDown of P q_top drops K + 1 >= 2
// limbs (the two-launch form).  The buffers are free: this step's combine and
// inner products, which read the current speculation, run before in stream
// order.  (A second stream for this work measured 3x slower)
static bool spec_attach(bool one, unsigned glvl, const std::vector<SpecPat> &pats = g_spec_pats_next,
                        const uint64_t *pk1 = g_spec_pk1_next)
{
  static const bool on = env_u("GPQHE_SPEC", 1) != 0 && env_u("GPQHE_SPEC_ATTACH", 1) != 0;
  const unsigned k = g_spec_next_k, lvl = g_spec_next_lvl;
  if (!on || !one || !k || !lvl || k > GPQHE_MAXGRP || !defer_ok(0) || G.logn < 10 || G.logn > 12 || G.K < 1)
    return false;
  if ((size_t)3 * k * (G.n / 512) > (size_t)(G.n / 64) * (glvl + G.K))
    return false;
  const size_t w = (size_t)lvl << G.logn, words = 3 * (size_t)k * w;
  if (g_spec.words != words) {
    pool_free(g_spec.buf);  // stream-ordered: its last reader was launched before
    g_spec.buf = (uint64_t *)pool_alloc(words * 8);
    g_spec.words = words;
  }
  unsigned mods[GPQHE_MAXMOD];
  for (unsigned l = 0; l < lvl; l++)
    mods[l] = l;
  g_sa = SpecAttach{};
  g_smu_next.pending = false;
  g_sa.noise = limbset(g_spec.buf, mods, lvl, 3 * k, w);
  g_sa.stream = G.counter;
  g_sa.npoly = 3 * k;
  g_sa.sample = g_sa.ntt = true;
  g_spec.base = G.counter;
  g_spec.k = k;
  g_spec.lvl = lvl;
  g_spec.valid = true;
  g_smu.valid = false;
  bool ok = !pats.empty() && pk1 && lvl >= 2;
  for (const SpecPat &p : pats)
    ok &= p.oa < k && p.ob < k;
  if (ok) {
    const unsigned np = (unsigned)pats.size(), nm = lvl + G.K, ndig = (lvl + G.alpha - 1) / G.alpha;
    const size_t dw = (size_t)np * ndig * nm << G.logn;
    if (g_smu.dwords != dw) {
      pool_free(g_smu.D);  // stream-ordered: its last reader was launched before
      g_smu.D = (uint64_t *)pool_alloc(dw * 8);
      g_smu.dwords = dw;
    }
    // the ModUp itself runs behind this step's decode (he_dcd_ex), in the
    // device time the caller's host work leaves idle: attached to the
    // ModDown it lengthened the chain the decode waits on (13.9 -> 21.5 us)
    for (unsigned i = 0; i < np; i++) {
      g_smu_next.cd.va[i] = g_spec.buf + (size_t)3 * pats[i].oa * w;
      g_smu_next.cd.vb[i] = g_spec.buf + (size_t)3 * pats[i].ob * w;
    }
    g_smu_next.np = np;
    g_smu_next.d_stride = (size_t)ndig * nm << G.logn;
    g_smu_next.pk1 = pk1;
    g_smu_next.lvl = lvl;
    g_smu_next.pending = true;
    // its first half (the differences' inverse transforms) rides on this
    // step's ModDown (k_moddown: the launch after the noise transforms), so
    // only the second half runs behind the decode (GPQHE_SPEC_MODUP_SPLIT=0:
    // the whole ModUp there)
    static const bool split = env_u("GPQHE_SPEC_MODUP_SPLIT", 1) != 0;
    if (split) {
      const size_t yw = (size_t)np * lvl << G.logn;
      if (g_smu.ywords != yw) {
        pool_free(g_smu.Y);  // stream-ordered: its last reader was launched before
        g_smu.Y = (uint64_t *)pool_alloc(yw * 8);
        g_smu.ywords = yw;
      }
      g_sa.mh.cd = g_smu_next.cd;
      g_sa.mh.pk1 = pk1;
      g_sa.mh.D = g_smu.D;
      g_sa.mh.Y = g_smu.Y;
      g_sa.mh.d_stride = g_smu_next.d_stride;
      g_sa.mh.np = np;
      g_sa.mh.lvl = lvl;
      g_sa.modup_inv = true;
    }
    const std::vector<SpecPat> keep = pats;  // (pats may be g_smu.pats itself)
    g_smu.pats = keep;
    g_smu.base = g_spec.base;
    g_smu.pk1 = pk1;
    g_smu.lvl = lvl;
  }
  return true;
}

// The ModUp spec_attach left pending, behind the decode: true if launched.
static bool spec_modup_launch()
{
  if (!g_smu_next.pending)
    return false;
  g_smu_next.pending = false;
  if (g_sa.modup_inv_done) {  // its first half ran in this step's ModDown
    g_sa.modup_inv_done = false;
    k_modup_fwd_diffs(g_sa.mh);
  } else {
    k_modup_ntt_diffs(g_smu.D, g_smu_next.cd, g_smu_next.np, g_smu_next.d_stride, g_smu_next.pk1, g_smu_next.lvl);
  }
  g_smu.valid = true;
  return true;
}

// The last step's gemvs on this step's encryptions (SpecGemv), right after
// their combine: one inner-product launch for both (differences formed in the
// kernel, the speculated ModUp digits), one ModDown with two outputs, and the
// next step's speculation attached to them as flush_gemvs would (spec_attach,
// the patterns predicted to repeat).  Only when every recorded gemv ran one
// launch of diagonals and the ModUp digits speculated for this step are there.
static void spec_gemv_launch(const std::vector<PendEnc> &enc, const std::vector<SgRec> &recs)
{
  static const bool on = env_u("GPQHE_SPEC_GEMV", 1) != 0;
  g_sg.valid = false;
  const unsigned np = (unsigned)recs.size(), lvl = enc.empty() ? 0 : enc[0].lvl;
  if (!on || !np || np > GemvJobs::MAX || !g_smu.valid || g_smu.lvl != lvl || g_smu.base != enc[0].stream ||
      g_smu.pats.size() != np || lvl < 2)
    return;
  for (unsigned i = 0; i < np; i++) {
    const SgRec &r = recs[i];
    if (r.pat.oa != g_smu.pats[i].oa || r.pat.ob != g_smu.pats[i].ob || r.pat.oa >= enc.size() ||
        r.pat.ob >= enc.size() || r.gen != g_key_gen || !r.dg.count)
      return;
  }
  const unsigned nm = lvl + G.K, ndig = (lvl + G.alpha - 1) / G.alpha;
  const size_t n = G.n, dstride = (size_t)ndig * nm * n, ypw = (size_t)G.L * n;
  for (unsigned i = 0; i < np; i++)
    if (!g_sg.Y[i])  // (stream-ordered: a block swapped in last step was last read before this launch)
      g_sg.Y[i] = (uint64_t *)pool_alloc(2 * ypw * 8);
  Ws acc((size_t)np * 2 * nm * n);
  GemvJobs jobs;
  for (unsigned i = 0; i < np; i++) {
    const PendEnc &a = enc[recs[i].pat.oa], &b = enc[recs[i].pat.ob];
    jobs.j[i] = GemvJob{acc.p + (size_t)i * 2 * nm * n, g_smu.D + i * dstride, a.c0, a.c1, recs[i].dg, 0};
    jobs.j[i].y0 = b.c0;
    jobs.j[i].y1 = b.c1;
    g_sg.x[i][0] = a.c0;
    g_sg.x[i][1] = b.c0;
    g_sg.x[i][2] = a.c1;
    g_sg.x[i][3] = b.c1;
    g_sg.sa[i] = a.stream;
    g_sg.sb[i] = b.stream;
    g_sg.rec[i] = recs[i];
    g_sg.used[i] = false;
  }
  // the next step's noise in these launches' idle CUs, its ModUp behind the
  // decode, for the same patterns (the digits these jobs read are overwritten
  // only by that ModUp, after the decode in stream order)
  if (!g_spec_early && spec_attach(true, lvl, std::vector<SpecPat>(g_smu.pats), g_smu.pk1))
    g_spec_early = true;
  k_gemv_inner_jobs(jobs, np, lvl);
  if (np == 1)
    k_moddown(g_sg.Y[0], ypw, acc.p, nm * n, 2, lvl, 1);
  else
    k_moddown(g_sg.Y[0], ypw, acc.p, nm * n, 4, lvl, 1, g_sg.Y[1]);
  if (g_sa.sample) {  // (as flush_gemvs: work a launch did not take runs on its own)
    g_sa.sample = false;
    k_sample_enc(g_sa.noise, g_sa.stream, g_sa.npoly);
  }
  if (g_sa.ntt) {
    g_sa.ntt = false;
    k_ntt(g_sa.noise, false);
  }
  g_sg.np = np;
  g_sg.lvl = lvl;
  g_sg.valid = true;
  // this step's role blocks, and the last step's tail replayed on them (SpecDcd)
  g_sd_ctx = SdCtx{};
  for (unsigned i = 0; i < np; i++)
    g_sd_ctx.y[i] = g_sg.Y[i];
  g_sd_ctx.ny = np;
  g_sd_ctx.ylvl = lvl - 1;
  for (unsigned o = 0; o < enc.size() && o < GPQHE_MAXGRP; o++) {
    g_sd_ctx.e[o][0] = enc[o].c0;
    g_sd_ctx.e[o][1] = enc[o].c1;
    g_sd_ctx.es[o] = enc[o].stream;
    g_sd_ctx.ne = o + 1;
  }
  g_sd_ctx.elvl = lvl;
  g_sd_ctx.valid = true;
  g_sd.valid = false;
  if (g_sd_next_ok && sd_on())
    sd_replay(g_sd_next);
}

extern "C" void he_dcd_ex(gpqhe_complex_t z[], const he_pt_t *pt, unsigned int slots)
{
  HPROF("dcd");
  const size_t zb = (size_t)slots * 16;
  if (G.init && defer_ok(0) && slots && !(slots & (slots - 1)) && slots <= GPQHE_DCD_ONEPASS &&
      slots <= G.n / 2 && !(pt->flags & GPQHE_F_COEFF) && pt->nlimbs >= 1 && pt->nlimbs <= 2) {
    // the small-N step's tail: the queued elementwise program (he_add, he_neg,
    // he_copy_ct, he_add, he_dec), then the inverse transform and the decoder
    // in one more launch (k_ew_decode)
    // this step's tail pattern (replayed next step), and the replay of the
    // last step's (SpecDcd) when this step's is the same
    SdPat cur;
    const bool quiet = g_pgemv.empty() && g_pecd.empty() && g_penc.empty();
    g_sd_next_ok = quiet && sd_pattern(g_pew, pt->data, pt->nlimbs, slots, pt->scale, g_sd_ctx, cur);
    if (g_sd_next_ok)
      g_sd_next = cur;
    if (g_sd.valid && g_sd_next_ok && g_spec_early && cur.same(g_sd.pat) && sd_enc_fresh(cur, g_sd_ctx)) {
      g_sd.valid = false;
      flush_ew();  // the real program: its objects, not waited for
      g_spec_early = false;
      if (g_smu_next.pending)
        spec_modup_launch();
      const hipError_t q = hipEventQuery(g_sd.ev);
      (void)hipGetLastError();  // (not ready is no error)
      if (q != hipSuccess) {
        // the device behind the caller: the replay only lengthens the chain
        // (GPQHE_SPEC_DCD=2 keeps it on: tests)
        if (++g_sd_late >= 2 && env_u("GPQHE_SPEC_DCD", 1) != 2)
          g_sd_off = true;
      } else {
        g_sd_late = 0;
      }
      HIP_CHECK(hipEventSynchronize(g_sd.ev));
      memcpy(z, g_sd.z, zb);
      g_sd_taken++;
      return;
    }
    g_sd.valid = false;
    if (!g_pgemv.empty())
      flush_gemvs();
    if (!g_pecd.empty() || !g_penc.empty())
      flush_pending();
    // workspace and pinned buffer first: the pool's out-of-memory path flushes
    // the elementwise queue, which must still hold the program then (its ops
    // may name freed blocks the flush would otherwise release under it)
    Ws c((size_t)pt->nlimbs << G.logn);
    double *zd = (double *)zpin(zb);
    const EwProg p = g_pew;
    g_pew.count = 0;
    k_ew_decode(p, zd, pt->data, pt->nlimbs, slots, pt->scale, c.p);
    const bool early = g_spec_early;
    g_spec_early = false;
    bool spec = false;
    if (early && g_smu_next.pending) {
      if (!g_dcd_ev)
        HIP_CHECK(hipEventCreateWithFlags(&g_dcd_ev, hipEventDisableTiming));
      HIP_CHECK(hipEventRecord(g_dcd_ev, G.stream));
      spec = spec_modup_launch();
    } else if (!early) {
      spec = spec_launch();
    }
    if (spec) {
      HIP_CHECK(hipEventSynchronize(g_dcd_ev));  // the decode, not the noise behind it
    } else {
      HIP_CHECK(hipStreamSynchronize(G.stream));
    }
    memcpy(z, g_zpin, zb);
    return;
  }
  check_ctx();
  const unsigned nl = pt->nlimbs;
  const size_t words = (size_t)nl << G.logn;
  Ws c(words);
  const uint64_t *src = pt->data;
  if (!(pt->flags & GPQHE_F_COEFF)) {
    // out-of-place inverse transform (the plaintext stays in NTT form)
    k_ntt_ex(qlimbs(pt->data, nl, 1, words), qlimbs(c.p, nl, 1, words), true, nullptr);
    src = c.p;
  }
  // CRT lift + FFT on the GPU (k_decode); only the s values cross PCIe,
  // written by the kernel straight into pinned host memory when one launch
  // does it (no copy launch)
  if (slots <= GPQHE_DCD_ONEPASS) {
    k_decode((double *)zpin(zb), src, nl, slots, pt->scale);
    HIP_CHECK(hipStreamSynchronize(G.stream));
    memcpy(z, g_zpin, zb);
    return;
  }
  Ws zd(2 * (size_t)slots);
  k_decode((double *)zd.p, src, nl, slots, pt->scale);
  HIP_CHECK(hipMemcpyAsync(z, zd.p, zb, hipMemcpyDeviceToHost, G.stream));
  HIP_CHECK(hipStreamSynchronize(G.stream));
}

extern "C" void he_dcd(gpqhe_complex_t z[], const he_pt_t *pt)
{
  he_dcd_ex(z, pt, G.slots);
}

extern "C" void he_enc_pk(he_ct_t *ct, const he_pt_t *pt, const he_pk_t *pk)
{
  HPROF("enc_pk");
  if (!G.init)
    gpqhe_die("context not initialised (hectx_init)");
  const unsigned lvl = pt->nlimbs;
  if (defer_ok(0)) {
    // queued (flush_pending): streams taken now, in call order
    flush_ew();
    if (!g_pgemv.empty())
      flush_gemvs();
    bool busy = false;
    for (const PendEnc &e : g_penc)
      busy |= e.m == ct->data || e.c0 == ct->data;
    for (const PendEcd &e : g_pecd)
      busy |= e.dst == ct->data;
    if (busy)
      flush_pending();
    const uint64_t stream = next_stream();
    next_stream();
    next_stream();
    // a plaintext that is itself a queued encode (at this level) joins e0 as
    // coefficients (EncCoef)
    int ei = -1;
    for (size_t i = 0; i < g_pecd.size(); i++)
      if (g_pecd[i].dst == pt->data && g_pecd[i].lvl == lvl)
        ei = (int)i;
    g_penc.push_back({limb(ct, 0, 0), limb(ct, 1, 0), pt->data, limb(pk, 0, 0), limb(pk, 1, 0), lvl, stream, ei});
    ct->nlimbs = lvl;
    ct->scale = pt->scale;
    ct->flags = 0;
    return;
  }
  check_ctx();
  const size_t w = (size_t)lvl << G.logn;
  unsigned mods[GPQHE_MAXMOD];
  for (unsigned i = 0; i < lvl; i++)
    mods[i] = i;
  // v (ternary), e0, e1 (CBD) on consecutive streams, sampled and NTT'd in
  // one launch each (the values of three sample_small_ntt calls in order)
  Ws vee(3 * w);
  LimbSet s = limbset(vee.p, mods, lvl, 3, w);
  const uint64_t stream = next_stream();
  next_stream();
  next_stream();
  k_sample_enc(s, stream, 3);
  k_ntt(s, false);
  k_enc_combine(limb(ct, 0, 0), limb(ct, 1, 0), vee.p, vee.p + w, vee.p + 2 * w, limb(pk, 0, 0), limb(pk, 1, 0),
                pt->data, lvl);
  ct->nlimbs = lvl;
  ct->scale = pt->scale;
  ct->flags = 0;
}

extern "C" void he_enc_sk(he_ct_t *ct, const he_pt_t *pt, const poly_mpi_t *sk)
{
  check_ctx();
  const unsigned lvl = pt->nlimbs;
  unsigned mods[GPQHE_MAXMOD];
  for (unsigned i = 0; i < lvl; i++)
    mods[i] = i;
  sample_uniform(limb(ct, 1, 0), mods, lvl);
  Ws e((size_t)lvl << G.logn);
  sample_small_ntt(e.p, mods, lvl, 1);
  k_enc_sk_combine(limb(ct, 0, 0), limb(ct, 1, 0), e.p, sk->data, pt->data, lvl);
  ct->nlimbs = lvl;
  ct->scale = pt->scale;
  ct->flags = 0;
}

// Queue elementwise ops (defer_ok(0): n <= 2^12); false: run them now.
static bool ew_defer(unsigned nops)
{
  if (!defer_ok(0))
    return false;
  if (!g_pgemv.empty())
    flush_gemvs();
  if (!g_pecd.empty() || !g_penc.empty())
    flush_pending();
  if (g_pew.count + nops > EwProg::MAX)
    flush_ew();
  return true;
}

static void ew_push(uint32_t kind, uint64_t *out, const uint64_t *a, const uint64_t *b, const uint64_t *sk,
                    unsigned lvl)
{
  g_pew.op[g_pew.count++] = EwOp{out, a, b, sk, kind, lvl};
  // out's provenance after this op (C1Prov): the difference of two fresh
  // encryptions at their full level with one public key, or none
  C1Prov d{};
  bool known = false;
  if (kind == EW_SUB && !g_prov.empty()) {
    auto ia = g_prov.find(a), ib = g_prov.find(b);
    if (ia != g_prov.end() && ib != g_prov.end() && !ia->second.sub && !ib->second.sub && !ia->second.c0 &&
        !ib->second.c0 && ia->second.pk1 == ib->second.pk1 && ia->second.lvl == lvl && ib->second.lvl == lvl) {
      d = C1Prov{ia->second.sa, ib->second.sa, ia->second.pk1, lvl, true};
      known = true;
    }
  }
  if (known)
    g_prov[out] = d;
  else if (!g_prov.empty())
    g_prov.erase(out);
}

extern "C" void he_dec(he_pt_t *pt, const he_ct_t *ct, const poly_mpi_t *sk)
{
  HPROF("dec");
  if (!G.init)
    gpqhe_die("context not initialised (hectx_init)");
  if (ew_defer(1)) {
    ew_push(EW_DEC, pt->data, limb(ct, 0, 0), limb(ct, 1, 0), sk->data, ct->nlimbs);
    pt->nlimbs = ct->nlimbs;
    pt->scale = ct->scale;
    pt->flags = 0;
    return;
  }
  check_ctx();
  k_dec(pt->data, limb(ct, 0, 0), limb(ct, 1, 0), sk->data, ct->nlimbs);
  pt->nlimbs = ct->nlimbs;
  pt->scale = ct->scale;
  pt->flags = 0;
}

// ===========================================================================
// Evaluation
// ===========================================================================
static void check_scales(double a, double b, const char *op)
{
  if (fabs(a / b - 1.0) > 1e-9)
    gpqhe_die("%s: scale mismatch (%g vs %g)", op, a, b);
}

static void addsub(he_ct_t *out, const he_ct_t *a, const he_ct_t *b, int op)
{
  if (!G.init)
    gpqhe_die("context not initialised (hectx_init)");
  check_scales(a->scale, b->scale, op ? "he_sub" : "he_add");
  const unsigned lvl = std::min(a->nlimbs, b->nlimbs);
  const double scale = a->scale;
  if (ew_defer(2)) {
    for (unsigned p = 0; p < 2; p++)
      ew_push(op ? EW_SUB : EW_ADD, limb(out, p, 0), limb(a, p, 0), limb(b, p, 0), nullptr, lvl);
  } else {
    check_ctx();
    k_binop(out->data, a->data, b->data, 2, lvl, pstride(out), pstride(a), pstride(b), op);
  }
  out->nlimbs = lvl;
  out->scale = scale;
  out->flags = 0;
}

extern "C" void he_add(he_ct_t *out, const he_ct_t *a, const he_ct_t *b)
{
  HPROF("add");
  addsub(out, a, b, 0);
}
extern "C" void he_sub(he_ct_t *out, const he_ct_t *a, const he_ct_t *b)
{
  HPROF("sub");
  addsub(out, a, b, 1);
}

extern "C" void he_neg(he_ct_t *ct)
{
  HPROF("neg");
  if (!G.init)
    gpqhe_die("context not initialised (hectx_init)");
  if (ew_defer(2)) {
    for (unsigned p = 0; p < 2; p++)
      ew_push(EW_NEG, limb(ct, p, 0), limb(ct, p, 0), nullptr, nullptr, ct->nlimbs);
    return;
  }
  check_ctx();
  k_neg(ct->data, 2, ct->nlimbs, pstride(ct));
}

extern "C" void he_copy_ct(he_ct_t *dst, const he_ct_t *src)
{
  HPROF("copy_ct");
  if (!G.init)
    gpqhe_die("context not initialised (hectx_init)");
  if (dst == src)
    return;
  if (ew_defer(2)) {
    for (unsigned p = 0; p < 2; p++)
      ew_push(EW_COPY, limb(dst, p, 0), limb(src, p, 0), nullptr, nullptr, src->nlimbs);
  } else {
    check_ctx();
    const size_t bytes = ((size_t)src->nlimbs << G.logn) * 8;
    for (unsigned p = 0; p < 2; p++)
      HIP_CHECK(hipMemcpyAsync(limb(dst, p, 0), limb(src, p, 0), bytes, hipMemcpyDeviceToDevice, G.stream));
  }
  dst->nlimbs = src->nlimbs;
  dst->scale = src->scale;
  dst->flags = src->flags;
}

extern "C" void he_moddown(he_ct_t *ct)
{
  HPROF("moddown");
  // bookkeeping only (queued work captured its levels): no flush
  if (!G.init)
    gpqhe_die("context not initialised (hectx_init)");
  if (ct->nlimbs < 2)
    gpqhe_die("he_moddown: ciphertext at the lowest level");
  ct->nlimbs--;
}

extern "C" void he_add_pt(he_ct_t *out, const he_ct_t *a, const he_pt_t *pt)
{
  check_ctx();
  check_scales(a->scale, pt->scale, "he_add_pt");
  const unsigned lvl = std::min(a->nlimbs, pt->nlimbs);
  const double scale = a->scale;
  if (out != a) {
    he_copy_ct(out, a);
    flush_ew();  // the copy may have been queued
  }
  k_add_pt(out->data, out->data, pt->data, lvl, pstride(out));
  out->nlimbs = lvl;
  out->scale = scale;
  out->flags = 0;
}

extern "C" void he_mul_pt(he_ct_t *out, const he_ct_t *a, const he_pt_t *pt)
{
  check_ctx();
  const unsigned lvl = std::min(a->nlimbs, pt->nlimbs);
  const double scale = a->scale * pt->scale;
  if (pstride(out) != pstride(a))
    gpqhe_die("he_mul_pt: layout mismatch");
  k_mul_pt(out->data, a->data, pt->data, lvl, pstride(a));
  out->nlimbs = lvl;
  out->scale = scale;
  out->flags = 0;
}

// Tensor + relinearize [+ rescale] for `count` ciphertext pairs.
//   a, b: ciphertext i at a + i*in_stride, c1 at + in_pstride;
//   out:  polynomial p (= 2 i + {0,1}) at out + p*out_pstride.
// out may overlap a or b (he_mul(c, c, b)): every input read precedes the
// final ModDown kernel, the only writer of out, on one stream.
static void mul_chunk(uint64_t *out, size_t out_pstride, const uint64_t *a, const uint64_t *b, size_t in_stride,
                      size_t in_pstride, unsigned count, unsigned lvl, const he_evk_t *rlk, bool rescale)
{
  if (!rlk->data || rlk->dnum != G.dnum)
    gpqhe_die("relinearization key missing or built for another dnum");
  const unsigned nm = lvl + G.K, ndig = (lvl + G.alpha - 1) / G.alpha;
  const size_t n = G.n;
  if (k_mul_split_ok(lvl) && rlk->reserved) {
    // split key switch: the kept slots' epilogue writes out while other pairs'
    // inputs may still be unread, so out must not overlap the inputs -- except
    // he_mul(c, c, b) on one pair, where every output word replaces the input
    // word read by the same thread
    const uint64_t *evkm = (const uint64_t *)(uintptr_t)rlk->reserved;
    const unsigned keep = rescale ? lvl - 1 : lvl;
    auto span = [](const uint64_t *p, size_t hi) { return std::make_pair((uintptr_t)p, (uintptr_t)(p + hi)); };
    const auto o = span(out, (2 * (size_t)count - 1) * out_pstride + (size_t)keep * n);
    const auto ia = span(a, (count - 1) * in_stride + in_pstride + (size_t)lvl * n);
    const auto ib = span(b, (count - 1) * in_stride + in_pstride + (size_t)lvl * n);
    auto overlap = [&](std::pair<uintptr_t, uintptr_t> x) { return o.first < x.second && x.first < o.second; };
    const bool same_layout = count == 1 && out_pstride == in_pstride && (out == a || out == b);
    if ((overlap(ia) || overlap(ib)) && !(same_layout && (!overlap(ia) || out == a) && (!overlap(ib) || out == b))) {
      const size_t words = (2 * (size_t)count - 1) * out_pstride + (size_t)keep * n;
      Ws tmp(words);
      k_mul_relin_split(tmp.p, out_pstride, a, b, in_stride, in_pstride, evkm, count, lvl, rescale);
      HIP_CHECK(hipMemcpyAsync(out, tmp.p, words * 8, hipMemcpyDeviceToDevice, G.stream));
      return;
    }
    k_mul_relin_split(out, out_pstride, a, b, in_stride, in_pstride, evkm, count, lvl, rescale);
    return;
  }
  const size_t d2_stride = lvl * n, D_stride = (size_t)ndig * nm * n, acc_stride = 2 * nm * n;
  Ws d2(count * d2_stride), D(count * D_stride), acc(count * acc_stride);
  if (k_ks_fused_ok() && rlk->reserved) {
    // fused path (2^13 <= n <= 2^17): d0/d1 are formed by the key switch from
    // a and b (no tensor buffer); the ModDown runs on the dropped limbs'
    // inverse row passes
    Ws y(count * d2_stride);
    const unsigned keep = rescale ? lvl - 1 : lvl;
    const uint64_t *evkm = (const uint64_t *)(uintptr_t)rlk->reserved;
    k_mul_keyswitch_fused(acc.p, d2.p, y.p, D.p, a, b, in_stride, in_pstride, evkm, count, lvl, keep);
    k_moddown_fused(out, out_pstride, acc.p, nm * n, 2 * count, lvl, rescale ? 1 : 0);
    return;
  }
  // generic path (n <= 2^12: HECTR's own ring): materialized tensor, ModUp,
  // NTT, inner product, ModDown as separate launches
  const size_t d01_stride = 2 * lvl * n;
  Ws d01(count * d01_stride);
  k_tensor(d01.p, d2.p, a, b, lvl, in_stride, in_pstride, count, d01_stride);
  k_ntt(qlimbs(d2.p, lvl, count, d2_stride), true);
  k_modup(D.p, d2.p, count, d2_stride, D_stride, lvl);
  unsigned mods[GPQHE_MAXMOD];
  basis_qp(lvl, mods);
  k_ntt(limbset(D.p, mods, nm, count * ndig, nm * n), false);
  k_ks_inner(acc.p, D.p, count, D_stride, acc_stride, rlk->data, lvl, 1, d01.p, d01.p + lvl * n, d01_stride,
             nullptr, false);
  k_moddown(out, out_pstride, acc.p, nm * n, 2 * count, lvl, rescale ? 1 : 0);
}

static void mul_core(he_ct_t *out, const he_ct_t *a, const he_ct_t *b, const he_evk_t *rlk, bool rescale)
{
  check_ctx();
  const unsigned lvl = std::min(a->nlimbs, b->nlimbs);
  if (rescale && lvl < 2)
    gpqhe_die("he_mul_rescale: no level left to rescale");
  if (pstride(a) != pstride(b))
    gpqhe_die("he_mul: layout mismatch");
  const double scale = a->scale * b->scale;
  mul_chunk(out->data, pstride(out), a->data, b->data, 0, pstride(a), 1, lvl, rlk, rescale);
  out->nlimbs = rescale ? lvl - 1 : lvl;
  out->scale = rescale ? scale / (double)G.q[lvl - 1] : scale;
  out->flags = 0;
}

extern "C" void he_mul(he_ct_t *out, const he_ct_t *a, const he_ct_t *b, const he_evk_t *rlk)
{
  mul_core(out, a, b, rlk, false);
}

extern "C" void he_mul_rescale(he_ct_t *out, const he_ct_t *a, const he_ct_t *b, const he_evk_t *rlk)
{
  mul_core(out, a, b, rlk, true);
}

extern "C" void he_rescale(he_ct_t *ct)
{
  check_ctx();
  const unsigned lvl = ct->nlimbs;
  if (lvl < 2)
    gpqhe_die("he_rescale: ciphertext at the lowest level");
  k_moddown(ct->data, pstride(ct), ct->data, pstride(ct), 2, lvl, 2);
  ct->scale /= (double)G.q[lvl - 1];
  ct->nlimbs = lvl - 1;
}

static const he_evk_t *find_rot_key(const he_evk_t rk[], unsigned r, uint64_t g)
{
  const he_evk_t *k = &rk[r];
  if (!k->data || k->galois != (uint32_t)g)
    gpqhe_die("rotation key for r=%u (galois %llu) missing", r, (unsigned long long)g);
  if (k->dnum != G.dnum)
    gpqhe_die("rotation key built for dnum=%u, context dnum=%u", k->dnum, G.dnum);
  return k;
}

// c1 of x -> coefficient domain -> ModUp digits (NTT domain) in D.
static void hoist_modup(uint64_t *D, const he_ct_t *x, unsigned lvl)
{
  const unsigned nm = lvl + G.K, ndig = (lvl + G.alpha - 1) / G.alpha;
  XPtrs x1{};
  x1.p[0] = limb(x, 1, 0);
  k_modup_ntt(D, x1, 1, (size_t)ndig * nm * G.n, lvl);
}

extern "C" void he_rot(he_ct_t *out, const he_ct_t *in, unsigned int rot, const he_evk_t rk[])
{
  check_ctx();
  rot %= G.slots;
  if (!rot) {
    he_copy_ct(out, in);
    return;
  }
  const unsigned lvl = in->nlimbs, nm = lvl + G.K, ndig = (lvl + G.alpha - 1) / G.alpha;
  const size_t n = G.n;
  const uint64_t g = galois_of_rot(rot);
  const he_evk_t *k = find_rot_key(rk, rot, g);
  if (gemv_win_on(lvl)) {  // (reads every input word before the ModDown writes out: in place is fine)
    const FoldEntry &f = rot_fold(rot, lvl, rk);
    FoldUse use(f);
    const double scale = in->scale;
    k_gemv_batch_ex(out->data, 0, pstride(out), in->data, 0, pstride(in), 1, lvl, f.K, f.d.data(), 1, 0);
    out->nlimbs = lvl;
    out->scale = scale;
    out->flags = 0;
    return;
  }
  Ws D((size_t)ndig * nm * n), acc(2 * nm * n);
  hoist_modup(D.p, in, lvl);
  k_ks_inner(acc.p, D.p, 1, 0, 0, k->data, lvl, g, limb(in, 0, 0), nullptr, 0, nullptr, false);
  const double scale = in->scale;
  k_moddown(out->data, pstride(out), acc.p, nm * n, 2, lvl, 0);
  out->nlimbs = lvl;
  out->scale = scale;
  out->flags = 0;
}

// ---------------------------------------------------------------------------
// he_gemv: diagonal method, hoisted ModUp, diagonals encoded at scale q_top
// over the QP basis, one ModDown-and-rescale by P q_top at the end.
// Encoded diagonals are cached by content (the caller recomputes the same
// gain matrices every control step: reference src/hempc.c:232-238).
// ---------------------------------------------------------------------------
// A he_gemv of SpecGemv pattern i: y <- Y_i as two queued copies.  Returns
// i, or -1 (the normal path).
static int spec_gemv_take(he_ct_t *y, const double *Md, const he_ct_t *x, const he_evk_t rk[])
{
  if (!g_sg.valid || x->nlimbs != g_sg.lvl || !g_pgemv.empty() || !defer_ok(0))
    return -1;
  const unsigned lvl = g_sg.lvl, s = G.slots;
  // x = a - b: the last queued op writing each of its polys is a he_sub
  const uint64_t *lz[4] = {};
  const uint64_t *xp[2] = {limb(x, 0, 0), limb(x, 1, 0)};
  for (unsigned j = 0; j < g_pew.count; j++)
    for (unsigned p = 0; p < 2; p++)
      if (g_pew.op[j].out == xp[p]) {
        const EwOp &o = g_pew.op[j];
        const bool sub = o.kind == EW_SUB && o.lvl >= lvl;
        lz[2 * p] = sub ? o.a : nullptr;
        lz[2 * p + 1] = sub ? o.b : nullptr;
      }
  if (!lz[0] || !lz[2])
    return -1;
  // y must not be an operand of the queued ops (the copies run in the queue's
  // order, and a later op reading y would read the copy)
  const uint64_t *ylo = y->data, *yhi = y->data + 2 * pstride(y);
  auto hits = [&](const uint64_t *q, unsigned l) { return q && q < yhi && q + ((size_t)l << G.logn) > ylo; };
  for (unsigned j = 0; j < g_pew.count; j++) {
    const EwOp &o = g_pew.op[j];
    if (hits(o.a, o.lvl) || hits(o.b, o.lvl) || hits(o.s, o.lvl))
      return -1;
  }
  auto fresh = [&](const uint64_t *p, uint64_t stream, bool c0) {
    auto it = g_prov.find(p);
    return it != g_prov.end() && !it->second.sub && it->second.c0 == c0 && it->second.sa == stream &&
           it->second.lvl == lvl;
  };
  for (unsigned i = 0; i < g_sg.np; i++) {
    const SgRec &r = g_sg.rec[i];
    if (g_sg.used[i] || lz[0] != g_sg.x[i][0] || lz[1] != g_sg.x[i][1] || lz[2] != g_sg.x[i][2] ||
        lz[3] != g_sg.x[i][3] || r.rk != rk || r.gen != g_key_gen || r.M.size() != 2 * (size_t)s * s ||
        memcmp(r.M.data(), Md, r.M.size() * 8) || !fresh(lz[0], g_sg.sa[i], true) ||
        !fresh(lz[1], g_sg.sb[i], true) || !fresh(lz[2], g_sg.sa[i], false) || !fresh(lz[3], g_sg.sb[i], false))
      continue;
    const size_t ypw = (size_t)G.L << G.logn;
    if (!ew_defer(2))
      return -1;
    g_sg.used[i] = true;
    g_sg_taken++;
    prov_forget(y->data, pstride(y));
    if (y->npoly == 2 && y->cap == G.L && y->data) {
      // an object of the engine's own ciphertext shape: its block and Y_i's
      // trade places (no copy; the old block is the next step's Y_i -- no
      // queued op can name it: a queued op writing y would have to come
      // after this call, and the next speculation starts with empty queues)
      std::swap(y->data, g_sg.Y[i]);
    } else {
      for (unsigned p = 0; p < 2; p++)
        ew_push(EW_COPY, limb(y, p, 0), g_sg.Y[i] + p * ypw, nullptr, nullptr, lvl - 1);
    }
    return (int)i;
  }
  return -1;
}

// The pattern of a gemv input c whose c1 is the difference of two of this
// step's encryptions (C1Prov), recorded for the next step's speculation:
// its index in g_spec_pats_next, or -1.
static int spec_record_pattern(const C1Prov &c, unsigned lvl)
{
  const uint64_t span = 3 * (uint64_t)g_spec_next_k;
  if (g_spec_next_k && lvl == g_spec_next_lvl && c.sa >= g_step_base && c.sb >= g_step_base &&
      c.sa < g_step_base + span && c.sb < g_step_base + span && (c.sa - g_step_base) % 3 == 0 &&
      (c.sb - g_step_base) % 3 == 0 && g_spec_pats_next.size() < XPtrs::MAX &&
      (g_spec_pats_next.empty() || g_spec_pk1_next == c.pk1)) {
    g_spec_pk1_next = c.pk1;
    g_spec_pats_next.push_back({(unsigned)((c.sa - g_step_base) / 3), (unsigned)((c.sb - g_step_base) / 3)});
    return (int)g_spec_pats_next.size() - 1;
  }
  return -1;
}

// ... and the gemv itself (SgRec), when it is one launch of diagonals
static void spec_record_gemv(int pat, const double *Md, const PendGemv &pg, const he_evk_t rk[])
{
  if (pat < 0 || pg.dgs.size() != 1 || (size_t)pat != g_sg_next.size())
    return;
  const size_t mwords = 2 * (size_t)G.slots * G.slots;
  g_sg_next.push_back({g_spec_pats_next[pat], std::vector<double>(Md, Md + mwords), pg.dgs[0], rk, g_key_gen});
}

static std::unordered_map<std::string, uint64_t *> g_gemv_cache;
static std::vector<void *> g_gemv_blocks;  // what the cache's entries live in (one entry or a batch)
static size_t g_gemv_cache_bytes = 0;

// Whole matrices already seen (HECTR passes the same two gain matrices every
// step): the non-zero diagonals' rotations and cached encodings, so a repeat
// he_gemv costs one compare of the matrix instead of s diagonal keys.
struct GemvMat {
  unsigned s, lvl;
  std::vector<double> M;
  std::vector<GemvDiags> dgs;  // evk filled per call from its rk
  std::vector<unsigned> rot;   // the rotation of each diagonal, in dgs order
};
static std::vector<GemvMat> g_gemv_mats;

void gemv_cache_clear()
{
  for (void *b : g_gemv_blocks)
    pool_free(b);
  g_gemv_blocks.clear();
  g_gemv_cache.clear();
  g_gemv_cache_bytes = 0;
  g_gemv_mats.clear();
}

static std::string diag_key(const double *diag, unsigned s, unsigned lvl)
{
  std::string key((const char *)diag, (size_t)s * 16);
  key.append((const char *)&lvl, sizeof(lvl));
  return key;
}

// Would encoding one more diagonal at this level overflow the cache (and so
// clear it)?  he_gemv flushes its pending launch before that happens.
static bool diag_cache_full(unsigned lvl)
{
  const size_t bytes = ((size_t)(lvl + G.K) << G.logn) * 8;
  return g_gemv_cache_bytes + bytes > ((size_t)1 << 31);
}

static const uint64_t *diag_pt(const double *diag, unsigned s, unsigned lvl)
{
  const std::string key = diag_key(diag, s, lvl);
  auto it = g_gemv_cache.find(key);
  if (it != g_gemv_cache.end())
    return it->second;
  unsigned mods[GPQHE_MAXMOD];
  const unsigned nm = basis_qp(lvl, mods);
  const size_t bytes = ((size_t)nm << G.logn) * 8;
  if (g_gemv_cache_bytes + bytes > ((size_t)1 << 31))
    gemv_cache_clear();
  uint64_t *p = (uint64_t *)pool_alloc(bytes);
  g_gemv_blocks.push_back(p);
  encode_limbs(p, diag, s, (double)G.q[lvl - 1], mods, nm);
  g_gemv_cache[key] = p;
  g_gemv_cache_bytes += bytes;
  return p;
}

// x = a - b, both polys written by queued he_sub ops that nothing else in the
// queue touches (HECTR's xhat - xr and uhat - ur, src/hempc.c:253-256: the
// queue then holds exactly those four ops)?  Then he_gemv leaves them queued
// -- they run with the step's later elementwise ops -- and the inner products
// form the difference where they read x (gemv_inner_kernel), which saves the
// step a launch.  src: a0, b0, a1, b1.
static bool ew_lazy_sub(const he_ct_t *y, const he_ct_t *x, const uint64_t *src[4])
{
  static const bool on = env_u("GPQHE_DEFER_SUB", 1);
  if (!g_pew.count || !on)
    return false;
  const uint64_t *o0 = limb(x, 0, 0), *o1 = limb(x, 1, 0);
  const EwOp *m0 = nullptr, *m1 = nullptr;
  for (unsigned j = 0; j < g_pew.count; j++) {
    const EwOp &o = g_pew.op[j];
    if (o.kind != EW_SUB || o.lvl < x->nlimbs)
      return false;
    for (unsigned i = 0; i < g_pew.count; i++)  // no op reads what a queued op writes
      if (g_pew.op[i].a == o.out || g_pew.op[i].b == o.out)
        return false;
    if (o.out == o0) {
      if (m0)
        return false;
      m0 = &o;
    } else if (o.out == o1) {
      if (m1)
        return false;
      m1 = &o;
    }
  }
  if (!m0 || !m1)
    return false;
  // the gemv then runs before these ops (flush_gemvs precedes the queued
  // program): its output must not be an operand or output of any of them
  // (in-place he_gemv, or y = an operand of a sub), nor of the pending gemvs'
  // formed differences
  const uint64_t *ylo = y->data, *yhi = y->data + 2 * pstride(y);
  auto hits = [&](const uint64_t *p, unsigned lvl) { return p && p < yhi && p + ((size_t)lvl << G.logn) > ylo; };
  for (unsigned j = 0; j < g_pew.count; j++) {
    const EwOp &o = g_pew.op[j];
    if (hits(o.out, o.lvl) || hits(o.a, o.lvl) || hits(o.b, o.lvl) || hits(o.s, o.lvl))
      return false;
  }
  src[0] = m0->a;
  src[1] = m0->b;
  src[2] = m1->a;
  src[3] = m1->b;
  return true;
}

// Runs the queued gemvs: ModUp of every input in one pass (k_modup_ntt: one
// fused launch at n <= 2^12), the inner products per gemv, and one ModDown
// for each pair of outputs.  The arithmetic per
// ciphertext is that of the unbatched sequence, so the results are too.
static void flush_gemvs()
{
  std::vector<PendGemv> q;
  q.swap(g_pgemv);
  if (q.empty())
    return;
  g_sd.valid = false;  // (its outputs may take blocks the replayed tail read: SpecDcd)
  const unsigned k = (unsigned)q.size(), lvl = q[0].lvl;
  const unsigned nm = lvl + G.K, ndig = (lvl + G.alpha - 1) / G.alpha;
  const size_t n = G.n;
  // ModUp of the inputs without precomputed digits (SpecModup), in one pass
  const size_t dstride = (size_t)ndig * nm * n;
  unsigned miss = 0;
  for (unsigned i = 0; i < k; i++)
    miss += !q[i].dspec;
  Ws D((size_t)miss * dstride), acc((size_t)k * 2 * nm * n);
  std::vector<const uint64_t *> Dp(k);
  XPtrs x1{};
  for (unsigned i = 0, m = 0; i < k; i++) {
    if (q[i].dspec) {
      Dp[i] = q[i].dspec;
    } else {
      x1.p[m] = q[i].x1;
      Dp[i] = D.p + m++ * dstride;
    }
    prov_forget(q[i].y, q[i].ypstride);
  }
  if (miss)
    k_modup_ntt(D.p, x1, miss, dstride, lvl);
  // every gemv with one launch's worth of diagonals: all in one launch
  bool one = k <= GemvJobs::MAX;
  for (unsigned i = 0; i < k; i++)
    one &= q[i].dgs.size() == 1;
  if (one) {
    if (!g_spec_early && spec_attach(true, lvl))
      g_spec_early = true;
    GemvJobs jobs;
    for (unsigned i = 0; i < k; i++) {
      jobs.j[i] = GemvJob{acc.p + (size_t)i * 2 * nm * n, Dp[i], q[i].x0, q[i].x1, q[i].dgs[0], 0};
      if (q[i].lb0) {  // the queued difference, formed in the kernel
        jobs.j[i].x0 = q[i].la0;
        jobs.j[i].x1 = q[i].la1;
        jobs.j[i].y0 = q[i].lb0;
        jobs.j[i].y1 = q[i].lb1;
      }
    }
    k_gemv_inner_jobs(jobs, k, lvl);
  } else {
    for (unsigned i = 0; i < k; i++)
      if (q[i].lb0)
        flush_ew();  // the queued differences, materialised first
    for (unsigned i = 0; i < k; i++) {
      uint64_t *a = acc.p + (size_t)i * 2 * nm * n;
      bool started = false;
      for (const GemvDiags &dg : q[i].dgs) {
        k_gemv_inner(a, Dp[i], q[i].x0, q[i].x1, lvl, dg, started);
        started = true;
      }
      if (!started)  // all-zero matrix
        HIP_CHECK(hipMemsetAsync(a, 0, 2 * nm * n * 8, G.stream));
    }
  }
  if (k == 1)
    k_moddown(q[0].y, q[0].ypstride, acc.p, nm * n, 2, lvl, 1);
  else
    k_moddown(q[0].y, q[0].ypstride, acc.p, nm * n, 4, lvl, 1, q[1].y);
  // spec_attach predicts which launches take the attached work; should a
  // launch's own eligibility test (kernels.hip: gemv_inner's z slice, the
  // ModDown's dropped limbs) ever disagree, the work runs here in its own
  // launches, same streams and buffers, so the speculation stays valid
  if (g_sa.sample) {
    g_sa.sample = false;
    k_sample_enc(g_sa.noise, g_sa.stream, g_sa.npoly);
  }
  if (g_sa.ntt) {
    g_sa.ntt = false;
    k_ntt(g_sa.noise, false);
  }
}

// Unqueued he_gemv for matrices whose diagonals may overflow the cache: a
// launch that refers to cached diagonals runs before the cache is cleared.
static void gemv_now(he_ct_t *y, const double *Md, const he_ct_t *x, const he_evk_t rk[], unsigned lvl)
{
  prov_forget(y->data, pstride(y));
  const unsigned s = G.slots, nm = lvl + G.K, ndig = (lvl + G.alpha - 1) / G.alpha;
  const size_t n = G.n;
  Ws D((size_t)ndig * nm * n), acc(2 * nm * n);
  hoist_modup(D.p, x, lvl);
  std::vector<double> diag(2 * (size_t)s);
  GemvDiags dg{};
  bool started = false;
  auto flush = [&]() {
    if (!dg.count)
      return;
    k_gemv_inner(acc.p, D.p, limb(x, 0, 0), limb(x, 1, 0), lvl, dg, started);
    started = true;
    dg.count = 0;
  };
  for (unsigned d = 0; d < s; d++) {
    bool nz = false;
    for (unsigned i = 0; i < s; i++) {
      const size_t src = (size_t)i * s + (i + d) % s;
      diag[2 * i] = Md[2 * src];
      diag[2 * i + 1] = Md[2 * src + 1];
      nz |= diag[2 * i] != 0.0 || diag[2 * i + 1] != 0.0;
    }
    if (!nz)
      continue;
    if (diag_cache_full(lvl))
      flush();  // the cache may be cleared below: launch what refers to it first
    const uint64_t *pt = diag_pt(diag.data(), s, lvl);
    const uint64_t g = d == 0 ? 1 : galois_of_rot(d);
    const he_evk_t *k = d == 0 ? nullptr : find_rot_key(rk, d, g);
    dg.evk[dg.count] = k ? k->data : nullptr;
    dg.pt[dg.count] = pt;
    dg.g[dg.count] = g;
    if (++dg.count == GemvDiags::MAX)
      flush();
  }
  flush();
  if (!started)  // all-zero matrix
    HIP_CHECK(hipMemsetAsync(acc.p, 0, 2 * nm * n * 8, G.stream));
  const double scale = x->scale;
  k_moddown(y->data, pstride(y), acc.p, nm * n, 2, lvl, 1);
  y->nlimbs = lvl - 1;
  y->scale = scale;
  y->flags = 0;
}

extern "C" void he_gemv(he_ct_t *y, const gpqhe_complex_t M[], const he_ct_t *x, const he_evk_t rk[])
{
  HPROF("gemv");
  if (!G.init)
    gpqhe_die("context not initialised (hectx_init)");
  // x may be a queued difference: left queued when the inner products can
  // form it (ew_lazy_sub, only with x's ModUp digits precomputed), else run
  // the result speculated at this step's encryptions (SpecGemv): two queued
  // copies, and the pattern recorded for the next step as below (before
  // anything flushes the queued differences it matches)
  if (g_sg.valid && g_pecd.empty() && g_penc.empty()) {
    if (const int i = spec_gemv_take(y, (const double *)M, x, rk); i >= 0) {
      const unsigned lvl = x->nlimbs;
      auto pv = g_prov.find(limb(x, 1, 0));
      const int pat =
          pv != g_prov.end() && pv->second.sub && pv->second.lvl == lvl ? spec_record_pattern(pv->second, lvl) : -1;
      if (pat >= 0 && (size_t)pat == g_sg_next.size()) {
        const SgRec &r = g_sg.rec[i];
        g_sg_next.push_back({g_spec_pats_next[pat], r.M, r.dg, rk, g_key_gen});
      }
      y->nlimbs = lvl - 1;
      y->scale = x->scale;
      y->flags = 0;
      return;
    }
  }
  const uint64_t *lz[4];
  const bool lazy = ew_lazy_sub(y, x, lz);
  if (!lazy)
    flush_ew();
  if (!g_pecd.empty() || !g_penc.empty())
    flush_pending();  // x may be a queued encryption
  const unsigned lvl = x->nlimbs, s = G.slots;
  if (lvl < 2)
    gpqhe_die("he_gemv: input at the lowest level");
  const double *Md = (const double *)M;
  // n >= 2^13: the windowed batch path on one ciphertext, unqueued.  It takes
  // no part in the small-N step's queues and speculation (check_ctx drops
  // any pending speculative ModUp): those serve HECTR's own ring (n <= 2^12),
  // where a step is a handful of small launches; at 2^13 and above a gemv is
  // tens of microseconds of device work on its own.  (In place, y == x, is
  // fine: every input word is read before the ModDown writes y.)
  if (gemv_win_on(lvl) && gemv_fold_fits(Md, lvl, rk)) {
    if (lazy)
      flush_ew();
    check_ctx();
    prov_forget(y->data, pstride(y));
    const FoldEntry &f = gemv_fold(Md, lvl, rk);
    FoldUse use(f);
    const double scale = x->scale;
    k_gemv_batch_ex(y->data, 0, pstride(y), x->data, 0, pstride(x), 1, lvl, f.K, f.d.data(), (unsigned)f.d.size(), 1);
    y->nlimbs = lvl - 1;
    y->scale = scale;
    y->flags = 0;
    return;
  }
  // queue behind the pending gemv only when the two are independent, at one
  // level, with one output layout, and no diagonal encode can clear the
  // cache the pending one refers to
  static const bool defer = env_u("GPQHE_DEFER", 1) && env_u("GPQHE_DEFER_GEMV", 1);
  const size_t dbytes = ((size_t)(lvl + G.K) << G.logn) * 8;
  const bool may_clear = g_gemv_cache_bytes + (size_t)s * dbytes > ((size_t)1 << 31);
  if (may_clear) {
    // the diagonal cache may be cleared inside this call: unqueued form
    flush_gemvs();
    flush_ew();
    gemv_now(y, Md, x, rk, lvl);
    return;
  }
  if (!g_pgemv.empty()) {
    const PendGemv &p = g_pgemv.back();
    if (g_pgemv.size() >= 2 || p.lvl != lvl || p.ypstride != pstride(y) || x->data == (void *)p.y ||
        (const void *)y->data == p.xdata || y->data == p.y)
      flush_gemvs();
  }
  PendGemv pg{y->data, pstride(y), limb(x, 0, 0), limb(x, 1, 0), x->data, lvl, {}};
  prov_forget(y->data, pstride(y));
  int pat = -1;  // the pattern recorded for the next step's speculation
  // x's c1: the difference of two fresh encryptions of this step?  Then its
  // ModUp may be precomputed (SpecModup), and the pattern is kept for the
  // next step's speculation.
  auto pv = g_prov.find(pg.x1);
  if (pv != g_prov.end() && pv->second.sub && pv->second.lvl == lvl) {
    const C1Prov &c = pv->second;
    if (g_smu.valid && g_smu.lvl == lvl && g_smu.pk1 == c.pk1)
      for (size_t i = 0; i < g_smu.pats.size(); i++)
        if (g_smu.base + 3 * (uint64_t)g_smu.pats[i].oa == c.sa && g_smu.base + 3 * (uint64_t)g_smu.pats[i].ob == c.sb) {
          const unsigned nmx = lvl + G.K, ndx = (lvl + G.alpha - 1) / G.alpha;
          pg.dspec = g_smu.D + i * ((size_t)ndx * nmx << G.logn);
          break;
        }
    pat = spec_record_pattern(c, lvl);
  }
  if (lazy && pg.dspec) {
    pg.la0 = lz[0];
    pg.lb0 = lz[1];
    pg.la1 = lz[2];
    pg.lb1 = lz[3];
  } else if (lazy) {
    flush_ew();  // the ModUp reads x1 itself
  }
  const size_t mwords = 2 * (size_t)s * s;
  for (const GemvMat &gm : g_gemv_mats)
    if (gm.s == s && gm.lvl == lvl && !memcmp(gm.M.data(), Md, mwords * 8)) {
      size_t r = 0;
      pg.dgs = gm.dgs;
      for (GemvDiags &dg : pg.dgs)
        for (unsigned e = 0; e < dg.count; e++, r++)
          dg.evk[e] = gm.rot[r] ? find_rot_key(rk, gm.rot[r], dg.g[e])->data : nullptr;
      spec_record_gemv(pat, Md, pg, rk);
      g_pgemv.push_back(std::move(pg));
      if (!defer)
        flush_gemvs();
      y->nlimbs = lvl - 1;
      y->scale = x->scale;
      y->flags = 0;
      return;
    }
  std::vector<unsigned> rots;
  std::vector<double> diag(2 * (size_t)s);
  // diagonals not cached yet (host-FFT sizes) are encoded together after the
  // loop: one upload and one lift + NTT launch for all of them
  const bool batch_enc = s < gpu_ecd_min();
  const size_t n = G.n, per = (size_t)(lvl + G.K) << G.logn;
  std::vector<std::string> newkeys;
  std::unordered_map<std::string, unsigned> newidx;
  std::vector<int64_t> newcoef;
  struct Fix {
    size_t launch;
    unsigned e, idx;
  };
  std::vector<Fix> fixes;
  // all non-zero diagonals in as few launches as possible (GemvDiags::MAX each)
  GemvDiags dg{};
  for (unsigned d = 0; d < s; d++) {
    bool nz = false;
    for (unsigned i = 0; i < s; i++) {
      const size_t src = (size_t)i * s + (i + d) % s;
      diag[2 * i] = Md[2 * src];
      diag[2 * i + 1] = Md[2 * src + 1];
      nz |= diag[2 * i] != 0.0 || diag[2 * i + 1] != 0.0;
    }
    if (!nz)
      continue;
    const uint64_t *pt = nullptr;
    std::string key = diag_key(diag.data(), s, lvl);
    auto it = g_gemv_cache.find(key);
    if (it != g_gemv_cache.end()) {
      pt = it->second;
    } else if (!batch_enc) {
      pt = diag_pt(diag.data(), s, lvl);
    } else {
      auto jt = newidx.find(key);
      unsigned idx;
      if (jt == newidx.end()) {
        idx = (unsigned)newkeys.size();
        newidx.emplace(key, idx);
        newkeys.push_back(std::move(key));
        newcoef.resize((size_t)(idx + 1) * n);
        hm_encode_coeffs(newcoef.data() + (size_t)idx * n, diag.data(), s, n, (double)G.q[lvl - 1]);
      } else {
        idx = jt->second;
      }
      fixes.push_back({pg.dgs.size(), dg.count, idx});
    }
    const uint64_t g = d == 0 ? 1 : galois_of_rot(d);
    const he_evk_t *k = d == 0 ? nullptr : find_rot_key(rk, d, g);
    dg.evk[dg.count] = k ? k->data : nullptr;
    dg.pt[dg.count] = pt;
    dg.g[dg.count] = g;
    rots.push_back(d);
    if (++dg.count == GemvDiags::MAX) {
      pg.dgs.push_back(dg);
      dg.count = 0;
    }
  }
  if (dg.count)
    pg.dgs.push_back(dg);
  if (!newkeys.empty()) {
    const unsigned cnt = (unsigned)newkeys.size();
    uint64_t *slab = (uint64_t *)pool_alloc((size_t)cnt * per * 8);
    g_gemv_blocks.push_back(slab);
    Ws dcoef(newcoef.size());
    upload(dcoef.p, newcoef.data(), newcoef.size() * 8);
    unsigned mods[GPQHE_MAXMOD];
    const unsigned nm = basis_qp(lvl, mods);
    k_lift_ntt(limbset(slab, mods, nm, cnt, per), (const int64_t *)dcoef.p);
    for (unsigned i = 0; i < cnt; i++)
      g_gemv_cache[newkeys[i]] = slab + (size_t)i * per;
    g_gemv_cache_bytes += (size_t)cnt * per * 8;
    for (const Fix &f : fixes)
      pg.dgs[f.launch].pt[f.e] = slab + (size_t)f.idx * per;
  }
  if (g_gemv_mats.size() >= 8)
    g_gemv_mats.erase(g_gemv_mats.begin());
  g_gemv_mats.push_back({s, lvl, std::vector<double>(Md, Md + mwords), pg.dgs, rots});
  const double scale = x->scale;
  spec_record_gemv(pat, Md, pg, rk);
  g_pgemv.push_back(std::move(pg));
  if (!defer)
    flush_gemvs();
  y->nlimbs = lvl - 1;
  y->scale = scale;
  y->flags = 0;
}

// ===========================================================================
// Batched entry points
// ===========================================================================
static unsigned g_mul_streams = 2;  // he_mul_rescale_batch: sub-chunks on their own streams (1 or 2)

extern "C" void gpqhe_set_streams(unsigned int n)
{
  if (n != 1 && n != 2)
    gpqhe_die("gpqhe_set_streams: 1 or 2, not %u", n);
  g_mul_streams = n;
}

extern "C" void he_mul_rescale_batch(uint64_t *out, const uint64_t *a, const uint64_t *b, size_t count,
                                     unsigned int nlimbs, const he_evk_t *rlk)
{
  check_ctx();
  const unsigned lvl = nlimbs;
  if (lvl < 2 || lvl > G.L)
    gpqhe_die("he_mul_rescale_batch: bad level %u", lvl);
  const unsigned nm = lvl + G.K, ndig = (lvl + G.alpha - 1) / G.alpha;
  const size_t n = G.n;
  // workspace limbs per pair: the split key switch holds y, T1, the dropped
  // slots and conv; the streaming one d2, y, T1 and both accumulators
  const size_t per_ct = (k_mul_split_ok(lvl) ? (size_t)(lvl + ndig * nm + 2 * (G.K + 1) + 2 * lvl)
                                              : (size_t)(2 * lvl + 2 * lvl + ndig * nm + 2 * nm + 2 * lvl)) * n * 8;
  // workspace per chunk (GPQHE_WS_MIB, default 8 GiB: 292 pairs at N=2^16,
  // L=8, dnum=2 on the split key switch, so the bench's 256 pairs run as one
  // chunk: 39.7k vs 38.4k ct-mult/s for two chunks of 128, same box).  Bigger
  // chunks fill the GPU better and amortize the key tiles over more pairs;
  // 288 GB of HBM leave room.
  static const size_t budget = (size_t)env_u("GPQHE_WS_MIB", 8192) << 20;
  size_t chunk = std::max<size_t>(1, budget / per_ct);
  chunk = std::min<size_t>(chunk, 65535 / (ndig * nm));
  if (const char *e = getenv("GPQHE_CHUNK"))  // test hook: force several chunks on a small batch
    chunk = std::max<size_t>(1, std::min<size_t>(chunk, strtoul(e, nullptr, 0)));
  // equal chunks: a short last chunk runs at a fraction of the GPU's width
  const size_t nchunks = (count + chunk - 1) / chunk;
  if (nchunks)
    chunk = (count + nchunks - 1) / nchunks;
  const size_t in_stride = 2 * lvl * n, out_stride = 2 * (size_t)(lvl - 1) * n;
  // Two sub-chunks on two streams, the second started once the first's
  // d2_rows has run, so one's VALU-bound column kernels overlap the other's
  // HBM-bound kernels on the same CUs (same box: 42.1k -> 42.7k ct-mult/s,
  // 60-bit 32.3k -> 32.7k, config 5 7.87k -> 7.98k; three or four streams
  // and four or more sub-chunks were slower).  Only without aliasing: a
  // sub-chunk's output must not overlap the other's inputs.
  const unsigned nsub = g_mul_streams;
  const uint64_t *oend = out + count * out_stride, *aend = a + count * in_stride, *bend = b + count * in_stride;
  const bool alias = (out < aend && a < oend) || (out < bend && b < oend);
  const bool split2 = count >= 2 && nchunks == 1 && !alias && k_mul_split_ok(lvl) && rlk->reserved &&
                      rlk->dnum == G.dnum;
  const uint64_t *evkm = (const uint64_t *)(uintptr_t)rlk->reserved;
  // (K pipelined sub-chunks with the HBM-bound stages on one stream and the
  // VALU-bound ones on the other, with or without a CU mask on the second:
  // DESIGN 5b, profiles/r5_ab_pipe.txt and r5_ab_cumask.txt, code at 7e2495a)
  if (split2 && nsub == 2 && !g_s2.s) {
    HIP_CHECK(hipStreamCreateWithFlags(&g_s2.s, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&g_s2.fork, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&g_s2.d2, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&g_s2.join, hipEventDisableTiming));
  }
  hipStream_t s2 = g_s2.s;
  hipEvent_t ev_fork = g_s2.fork, ev_d2 = g_s2.d2, ev_join = g_s2.join;
  if (nsub == 2 && split2) {
    const unsigned c1 = (unsigned)(count / 2), c2 = (unsigned)(count - c1);
    // both workspaces come from the engine stream's pool before the fork and
    // go back to it after the join
    Ws w1(k_mul_split_ws_words(c1, lvl, true)), w2(k_mul_split_ws_words(c2, lvl, true));
    HIP_CHECK(hipEventRecord(ev_fork, G.stream));
    HIP_CHECK(hipStreamWaitEvent(s2, ev_fork, 0));
    // the second sub-chunk starts once the first's d2_rows has run (where it
    // starts -- at once, after d2_rows or after ks_cols -- was within +-1 %
    // on two boxes, profiles/r4_ab_split_shift.txt)
    k_mul_relin_split(out, (lvl - 1) * n, a, b, in_stride, lvl * n, evkm, c1, lvl, true, w1.p, 0, 1);
    HIP_CHECK(hipEventRecord(ev_d2, G.stream));
    k_mul_relin_split(out, (lvl - 1) * n, a, b, in_stride, lvl * n, evkm, c1, lvl, true, w1.p, 1, 5);
    HIP_CHECK(hipStreamWaitEvent(s2, ev_d2, 0));
    const hipStream_t eng = G.stream;
    G.stream = s2;
    k_mul_relin_split(out + c1 * out_stride, (lvl - 1) * n, a + c1 * in_stride, b + c1 * in_stride, in_stride,
                      lvl * n, evkm, c2, lvl, true, w2.p);
    G.stream = eng;
    HIP_CHECK(hipEventRecord(ev_join, s2));
    HIP_CHECK(hipStreamWaitEvent(G.stream, ev_join, 0));
    return;
  }
  for (size_t c0 = 0; c0 < count; c0 += chunk) {
    const unsigned cnt = (unsigned)std::min(chunk, count - c0);
    mul_chunk(out + c0 * out_stride, (lvl - 1) * n, a + c0 * in_stride, b + c0 * in_stride, in_stride, lvl * n, cnt,
              lvl, rlk, true);
  }
}

// ---------------------------------------------------------------------------
// he_gemv / he_rot on the windowed path (gemv_win.hip) for n >= 2^13.  The
// rotation keys are folded with their diagonals once and cached: HECTR passes
// the same gain matrices every control step (src/hempc.c:232-238), the bench
// the same matrix every step.  A change of a key (generation, import, free)
// bumps g_key_gen: entries of an older generation never match again and are
// released at the next insert (or when the pool runs out of memory).
// A matrix whose folded set would exceed the cap (GPQHE_FOLD_MIB, 16 GiB:
// (2 ndig nm + lvl) n words per non-zero diagonal, ~30 GB for a dense
// 1024-slot matrix at N=2^16, L=8) takes the per-ciphertext path, whose
// diagonal cache is bounded and streams.
// ---------------------------------------------------------------------------
static size_t fold_cap()
{
  static const size_t cap = (size_t)env_u("GPQHE_FOLD_MIB", 16384) << 20;
  return cap;
}

static void fold_cache_clear()
{
  for (FoldEntry &f : g_folds)
    pool_free(f.K);
  g_folds.clear();
}

// out of memory: every set no running call reads goes back to the pool
static void fold_cache_trim()
{
  for (auto it = g_folds.begin(); it != g_folds.end();)
    if (it->K != g_fold_inuse) {
      pool_free(it->K);
      it = g_folds.erase(it);
    } else {
      ++it;
    }
}

static const FoldEntry &fold_insert(FoldEntry &&f)
{
  // a few sets (a 16-slot gemv at N=2^16, L=8 folds to 480 MB); f.bytes is
  // within the cap (gemv_fold_fits)
  size_t total = f.bytes;
  for (auto it = g_folds.begin(); it != g_folds.end();)
    if (it->gen != g_key_gen) {  // folded with keys that changed since
      pool_free(it->K);
      it = g_folds.erase(it);
    } else {
      total += it->bytes;
      ++it;
    }
  while (!g_folds.empty() && (g_folds.size() >= 8 || total > fold_cap())) {
    total -= g_folds.front().bytes;
    pool_free(g_folds.front().K);
    g_folds.pop_front();
  }
  g_folds.push_back(std::move(f));
  return g_folds.back();
}

static bool gemv_win_on(unsigned lvl)
{
  static const bool on = env_u("GPQHE_GEMV_WIN", 1) != 0;
  return on && k_gemv_win_ok(lvl);
}

// The rotations of M's non-zero diagonals, and (diags) the diagonals
// themselves, slots complex values each.
static std::vector<unsigned> gemv_diagonals(const double *Md, std::vector<double> *diags)
{
  const unsigned s = G.slots;
  std::vector<unsigned> ds;
  for (unsigned d = 0; d < s; d++) {
    bool nz = false;
    for (unsigned i = 0; i < s && !nz; i++) {
      const size_t src = (size_t)i * s + (i + d) % s;
      nz = Md[2 * src] != 0.0 || Md[2 * src + 1] != 0.0;
    }
    if (!nz)
      continue;
    ds.push_back(d);
    if (diags)
      for (unsigned i = 0; i < s; i++) {
        const size_t src = (size_t)i * s + (i + d) % s;
        diags->push_back(Md[2 * src]);
        diags->push_back(Md[2 * src + 1]);
      }
  }
  return ds;
}

static const FoldEntry *fold_find(const double *Md, unsigned lvl, const he_evk_t rk[])
{
  const unsigned s = G.slots;
  const size_t mwords = 2 * (size_t)s * s;
  for (const FoldEntry &f : g_folds)
    if (!f.M.empty() && f.s == s && f.lvl == lvl && f.gen == g_key_gen && f.rk == rk &&
        !memcmp(f.M.data(), Md, mwords * 8))
      return &f;
  return nullptr;
}

// Would M's folded set (plus the encoded diagonals it is folded from) fit the
// cap?  Cached sets always do.
static bool gemv_fold_fits(const double *Md, unsigned lvl, const he_evk_t rk[])
{
  if (fold_find(Md, lvl, rk))
    return true;
  const size_t E = gemv_diagonals(Md, nullptr).size();
  const size_t pts = E * (((size_t)lvl + G.K) << G.logn) * 8;
  return k_gemv_fold_words((unsigned)E, lvl) * 8 + pts <= fold_cap();
}

// The non-zero diagonals of M, encoded at scale q_{lvl-1} over basis_qp(lvl),
// folded with their rotation keys (the caller checked gemv_fold_fits).
static const FoldEntry &gemv_fold(const double *Md, unsigned lvl, const he_evk_t rk[])
{
  if (const FoldEntry *f = fold_find(Md, lvl, rk))
    return *f;
  const unsigned s = G.slots;
  const size_t mwords = 2 * (size_t)s * s;
  std::vector<double> diags;
  const std::vector<unsigned> ds = gemv_diagonals(Md, &diags);
  const unsigned E = (unsigned)ds.size();
  unsigned mods[GPQHE_MAXMOD];
  const unsigned nm = basis_qp(lvl, mods);
  const size_t per = (size_t)nm << G.logn;
  Ws pts((size_t)E * per);
  std::vector<GemvDiagIn> dg(E);
  for (unsigned e = 0; e < E; e++) {
    encode_limbs(pts.p + e * per, diags.data() + 2 * (size_t)s * e, s, (double)G.q[lvl - 1], mods, nm);
    dg[e].d = ds[e];
    dg[e].pt = pts.p + e * per;
    dg[e].evk = ds[e] ? find_rot_key(rk, ds[e], galois_of_rot(ds[e]))->data : nullptr;
  }
  FoldEntry f{std::vector<double>(Md, Md + mwords), s, lvl, 0, g_key_gen, rk, ds, nullptr,
              k_gemv_fold_words(E, lvl) * 8};
  f.K = E ? k_gemv_fold(dg.data(), E, lvl) : nullptr;
  return fold_insert(std::move(f));
}

static const FoldEntry &rot_fold(unsigned r, unsigned lvl, const he_evk_t rk[])
{
  const he_evk_t *k = find_rot_key(rk, r, galois_of_rot(r));
  for (const FoldEntry &f : g_folds)
    if (f.M.empty() && f.rot == r && f.lvl == lvl && f.gen == g_key_gen && f.rk == rk)
      return f;
  const GemvDiagIn dg{r, nullptr, k->data};
  FoldEntry f{{}, G.slots, lvl, r, g_key_gen, rk, {r}, nullptr, k_gemv_fold_words(1, lvl) * 8};
  f.K = k_gemv_fold(&dg, 1, lvl);
  return fold_insert(std::move(f));
}

static bool gemv_batch_fast(uint64_t *y, const double *Md, const uint64_t *x, size_t count, unsigned lvl,
                            const he_evk_t rk[])
{
  if (!gemv_win_on(lvl) || !gemv_fold_fits(Md, lvl, rk))
    return false;
  const FoldEntry &f = gemv_fold(Md, lvl, rk);
  FoldUse use(f);
  k_gemv_batch(y, x, count, lvl, f.K, f.d.data(), (unsigned)f.d.size(), 1);
  return true;
}

static bool rot_batch_fast(uint64_t *out, const uint64_t *x, size_t count, unsigned lvl, unsigned r,
                           const he_evk_t rk[])
{
  if (!gemv_win_on(lvl))
    return false;
  const FoldEntry &f = rot_fold(r, lvl, rk);
  FoldUse use(f);
  k_gemv_batch(out, x, count, lvl, f.K, f.d.data(), 1, 0);
  return true;
}

// A ciphertext of a batch as an object view (no payload of its own).
static he_ct_t ct_view(const uint64_t *base, unsigned nlimbs)
{
  he_ct_t c{};
  c.data = (uint64_t *)base;
  c.nlimbs = c.cap = nlimbs;
  c.npoly = 2;
  c.scale = 1.0;
  return c;
}

extern "C" void he_gemv_batch(uint64_t *y, const gpqhe_complex_t M[], const uint64_t *x, size_t count,
                              unsigned int nlimbs, const he_evk_t rk[])
{
  check_ctx();
  const unsigned lvl = nlimbs;
  if (lvl < 2 || lvl > G.L)
    gpqhe_die("he_gemv_batch: bad level %u", lvl);
  const size_t n = G.n, in_words = 2 * (size_t)lvl * n, out_words = 2 * (size_t)(lvl - 1) * n;
  if (count && y < x + count * in_words && x < y + count * out_words)
    gpqhe_die("he_gemv_batch: output overlaps the input");
  if (gemv_batch_fast(y, (const double *)M, x, count, lvl, rk))
    return;
  // one ciphertext at a time on the per-call path (its diagonals cached
  // after the first)
  for (size_t i = 0; i < count; i++) {
    he_ct_t cx = ct_view(x + i * in_words, lvl), cy = ct_view(y + i * out_words, lvl - 1);
    gemv_now(&cy, (const double *)M, &cx, rk, lvl);
  }
}

extern "C" void he_rot_batch(uint64_t *out, const uint64_t *x, size_t count, unsigned int nlimbs, unsigned int rot,
                             const he_evk_t rk[])
{
  check_ctx();
  const unsigned lvl = nlimbs;
  if (lvl < 1 || lvl > G.L)
    gpqhe_die("he_rot_batch: bad level %u", lvl);
  const size_t words = 2 * (size_t)lvl * G.n;
  if (count && out < x + count * words && x < out + count * words)
    gpqhe_die("he_rot_batch: output overlaps the input");
  if (rot % G.slots && rot_batch_fast(out, x, count, lvl, rot % G.slots, rk))
    return;
  for (size_t i = 0; i < count; i++) {
    he_ct_t cx = ct_view(x + i * words, lvl), co = ct_view(out + i * words, lvl);
    he_rot(&co, &cx, rot, rk);
  }
}

static void ntt_batch(uint64_t *data, size_t npolys, unsigned nlimbs, bool inverse)
{
  check_ctx();
  // groups of ~224 MiB: a group's column-pass output is still in the 256 MB
  // Infinity Cache when its row pass reads it (config 2, 1024 polys x 8 limbs
  // at N=2^16: roundtrip 8.41 -> 7.84 ms; 32-64 MiB groups lose more to
  // launch gaps than they gain).  Sweep (scripts/gpu_ntt_group.sh, same box,
  // ms): 96 7.46-7.56, 160 7.20-7.26, 192 6.84-6.92, 224 6.62-6.82, 240
  // 6.76-6.77, 256 6.72-7.04, 320 7.24, 512 7.42, whole batch 7.31-7.34.
  // (GPQHE_NTT_GROUP_MIB: the group size for sweeps)
  static const size_t group_mib = env_u("GPQHE_NTT_GROUP_MIB", 224);
  const size_t per = std::max<size_t>(1, std::min<size_t>(65535 / nlimbs, (group_mib << 20) /
                                                                              ((size_t)nlimbs * G.n * 8)));
  // the inverse walks the groups from the last one (GPQHE_NTT_REV): after a
  // forward batch, its last group's output is what the Infinity Cache holds
  static const bool rev = env_u("GPQHE_NTT_REV", 1) != 0;
  const size_t ngroups = (npolys + per - 1) / per;
  for (size_t i = 0; i < ngroups; i++) {
    const size_t g = inverse && rev ? ngroups - 1 - i : i, p0 = g * per;
    const unsigned cnt = (unsigned)std::min(per, npolys - p0);
    k_ntt(qlimbs(data + p0 * nlimbs * G.n, nlimbs, cnt, (size_t)nlimbs * G.n), inverse);
  }
}

extern "C" void poly_ntt_batch(uint64_t *data, size_t npolys, unsigned int nlimbs)
{
  ntt_batch(data, npolys, nlimbs, false);
}

extern "C" void poly_intt_batch(uint64_t *data, size_t npolys, unsigned int nlimbs)
{
  ntt_batch(data, npolys, nlimbs, true);
}

extern "C" void poly_fill_uniform(uint64_t *data, size_t npolys, unsigned int nlimbs, uint64_t seed)
{
  check_ctx();
  k_fill_uniform(data, npolys, nlimbs, seed);
}
