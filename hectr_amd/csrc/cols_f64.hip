// cols_f64.hip - the column kernels of the split key switch for prime sets
// whose every modulus is below 2^51 (the headline's): ks_colsf_kernel (ModUp:
// inverse column pass of the digit, conversion, forward column pass -> T1) and
// dn_colsf_kernel (ModDown: the same for the dropped limbs -> conv).  They
// replace the FP64 forms of kernels.hip's ks_cols4_kernel<., 8, true, true>
// and dn_cols_kernel<., 8, ., true, true> (GPQHE_COLSF, gpqhe_internal.h)
// with the same values, scheduled so that no transform waits on a global load.
#include "ntt_device.h"
#include "tables.h"

#include <type_traits>

// ks_colsf_kernel: the next digit limb's words requested one step ahead
#ifndef COLSF_PF
#define COLSF_PF 1
#endif
// (Code size: the kernels exceed the 64 KB instruction cache; one copy of
// the column INTT / target loop on the non-lazy policy instead of one per
// policy measured slower, DESIGN 5b, and was removed.)

// ---------------------------------------------------------------------------
// The INVC ks_cols4 for every modulus below 2^51 (the headline's prime sets):
// the same steps and values, scheduled so that no transform waits on a global
// load.  A block's work is a sequence of steps -- the na inverse column
// transforms of its digit limbs, then its nt targets -- each with one barrier
// between its two register rounds:
//   * data tiles alternate between two LDS buffers (step z uses lds[z & 1]),
//     so no step needs a barrier before its first round;
//   * the step's 128 column twiddles (the only entries a T-row column pass
//     reads) sit in LDS, triple-buffered: step z + 2's are loaded into
//     registers right after step z's barrier and written before step z + 1's,
//     where no wave can still read that buffer (it held step z - 1's);
//   * the conversion constants (c, c / q_t) and the moduli of all steps are
//     staged once per block;
//   * the lazy-reduction choice is a template argument (ArF64C), so the
//     butterfly code has no run-time branches.
// (ks_cols4_kernel: every twiddle and constant by global load inside its
// transform -- five L2 round trips per target.)
// NT: targets per block (8; 12 when a digit has more than 8, config 5: its
// column INTT then still runs once per digit tile).  T = 256 (n = 2^17): two
// data tiles and three twiddle buffers would exceed the 80 KB two blocks per
// CU allow, so a single tile with a barrier before every step and two twiddle
// buffers (as dn_colsf_kernel), and scheduling barriers between the forward
// stages (ArF64C SB: no spills).
template <int LOGT, int NT>
__global__ void __launch_bounds__(256, 2) ks_colsf_kernel(const uint64_t *ybuf, size_t y_stride, uint64_t *T1,
                                                           size_t t1_stride, unsigned logn, unsigned lvl,
                                                           unsigned L, unsigned nm, unsigned ndig, unsigned members,
                                                           unsigned ngroups, UpTable tab, Tw2 tw,
                                                           const ModConst *mcs)
{
  constexpr int T = 1 << LOGT, C = 4096 / T, LEA = LOGT - 4, EA = 1 << LEA, CP = C + 1, IT = C / 16;
  constexpr int TWW = 2 * T, TWP = (TWW + 255) / 256;  // twiddle words per step, per thread
  constexpr bool DB = LOGT <= 7;                        // double-buffered data tiles
  constexpr int NB = DB ? 3 : 2;                        // twiddle buffers
  __shared__ __attribute__((aligned(16))) uint64_t lds[DB ? 2 : 1][T * CP];
  __shared__ __attribute__((aligned(16))) double twl[NB][TWW];
  __shared__ __attribute__((aligned(16))) double cst[NT][4][2];
  __shared__ double qs[4 + NT];
  __shared__ unsigned ord[NT];
  const unsigned n2 = 1u << (logn - LOGT);
  const unsigned tiles = n2 / C;
  unsigned grp, mi;  // group = (p, j, tile) on one XCD; members = target batches
  if (!xcd_group(members, ngroups, grp, mi))
    return;
  const unsigned tile = grp % tiles, pj = grp / tiles, p = pj / ndig, j = pj % ndig;
  const UpDigit *dg = tab.dig + j;
  const unsigned lo = dg->lo, na = dg->na;
  if (mi * NT >= nm - na)
    return;
  const unsigned nt = min((unsigned)NT, nm - na - mi * NT), nsteps = na + nt;
  const int th = threadIdx.x;
  // step z: digit limb lo + z (inverse table), then target ui = mi NT + z - na
  // (skipping the digit's own slots; forward table)
  auto slot = [&](unsigned u) {
    const unsigned ui = mi * NT + u;
    return ui < lo ? ui : ui + na;
  };
  auto step_mod = [&](unsigned z) { return z < na ? lo + z : basis_mod(slot(ord[z - na]), lvl, L); };
  double tv[TWP];
  auto tw_load = [&](unsigned z) {
    const double *src = (z < na ? tw.invd : tw.fwdd) + ((size_t)step_mod(z) << (logn + 1));
#pragma unroll
    for (int w = 0; w < TWP; w++)
      tv[w] = th + 256 * w < TWW ? src[th + 256 * w] : 0.0;
  };
  auto tw_store = [&](unsigned z) {
#pragma unroll
    for (int w = 0; w < TWP; w++)
      if (th + 256 * w < TWW)
        twl[z % NB][th + 256 * w] = tv[w];
  };
  // targets run lazy moduli (q < 2^50) first, then the others: two loops with
  // the policy fixed at compile time (one loop choosing per target spilled
  // ~850 B/lane); position v holds target ord[v]
  unsigned nlz = 0;
  for (unsigned u = 0; u < nt; u++)
    nlz += mcs[basis_mod(slot(u), lvl, L)].q < (1ull << 50);
  if (th < (int)nt * 8) {
    const unsigned u = th / 8, i = (th / 2) % 4, c = th & 1;
    bool lz = true;
    unsigned before = 0;
    for (unsigned u2 = 0; u2 < nt; u2++) {
      const bool l2 = mcs[basis_mod(slot(u2), lvl, L)].q < (1ull << 50);
      if (u2 == u)
        lz = l2;
      else if (u2 < u)
        before += l2;
    }
    const unsigned v = lz ? before : nlz + (u - before);
    cst[v][i][c] = i < na ? tab.cd[2 * (((size_t)j * 8 + i) * nm + slot(u)) + c] : 0.0;
    if (th % 8 == 0) {
      ord[v] = u;
      qs[na + v] = (double)mcs[basis_mod(slot(u), lvl, L)].q;
    }
  }
  if (th < (int)na)
    qs[th] = (double)mcs[lo + th].q;
  tw_load(0);
  tw_store(0);
  __syncthreads();
  if (nsteps > 1)
    tw_load(1);
  const uint64_t *yb = ybuf + p * y_stride + ((size_t)lo << logn) + (size_t)tile * C;
  double y[IT][4][EA];
  // round A words of digit limb i (16 rows of one column per thread); with
  // COLSF_PF, limb i + 1's are requested while limb i is transformed (the
  // registers of the limbs not yet converted are free then)
  uint64_t pre[16];
  auto ld_limb = [&](int i) {
    const uint64_t *src = yb + ((size_t)i << logn);
    const int c = th % C, g = th / C;
    const unsigned vo = (unsigned)(16 * g) * n2 + c;
#pragma unroll
    for (int k = 0; k < 16; k++)
      pre[k] = (src + (size_t)k * n2)[vo];
  };
  ld_limb(0);
  // the digit arrives after the inverse row pass (d2_rows_kernel, which also
  // applied n^-1 [(Qj/q_i)^-1]): the inverse column pass, limb by limb
  auto invc = [&](auto I) {
    constexpr int i = decltype(I)::value;
    if (i >= (int)na) {
#pragma unroll
      for (int it = 0; it < IT; it++)
#pragma unroll
        for (int k = 0; k < EA; k++)
          y[it][i][k] = 0.0;
      return;
    }
    uint64_t *buf = lds[DB ? i & 1 : 0];
    if (!COLSF_PF && i)
      ld_limb(i);
    if (!DB && i)
      __syncthreads();  // the previous step's round B has read the tile
    with_f64c<!DB>(qs[i], twl[i % NB], [&](const auto &ar) {
      {
        const int g = th / C;
        double r[16];
#pragma unroll
        for (int k = 0; k < 16; k++)
          r[k] = f64_from_u52(pre[k]);
        if (COLSF_PF && i + 1 < (int)na)
          ld_limb(i + 1);
        ar.template inv<4>(r, T + 16 * g, 0);
        const int c = th % C;
#pragma unroll
        for (int k = 0; k < 16; k++)
          buf[(16 * g + k) * CP + c] = (uint64_t)__double_as_longlong(r[k]);
      }
      if (i + 1 < (int)nsteps)
        tw_store(i + 1);
      __syncthreads();
      if (i + 2 < (int)nsteps)
        tw_load(i + 2);
#pragma unroll
      for (int it = 0; it < IT; it++) {
        const int item = th + 256 * it, c = item % C, l = item / C;
        double r[EA];
#pragma unroll
        for (int k = 0; k < EA; k++)
          r[k] = __longlong_as_double((long long)buf[(l + 16 * k) * CP + c]);
        ar.template inv<LEA>(r, T, 4);
#pragma unroll
        for (int k = 0; k < EA; k++) {
          const double v = f64_red(r[k], ar.q, ar.qinv);
          y[it][i][k] = v < 0 ? v + ar.q : v;  // canonical (ArF64::canon_d)
        }
      }
    });
  };
  invc(std::integral_constant<int, 0>{});
  invc(std::integral_constant<int, 1>{});
  invc(std::integral_constant<int, 2>{});
  invc(std::integral_constant<int, 3>{});
  auto target = [&](unsigned v, auto LZ) {
    const unsigned z = na + v;
    uint64_t *buf = lds[DB ? z & 1 : 0];
    uint64_t *out = T1 + p * t1_stride + (((size_t)j * nm + slot(ord[v])) << logn) + (size_t)tile * C;
    double cw[4], cq[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      cw[i] = cst[v][i][0];
      cq[i] = cst[v][i][1];
    }
    const double q = qs[z];
    if (!DB)
      __syncthreads();  // the previous step's round B has read the tile
    [&](const auto &ar) {
#pragma unroll
      for (int it = 0; it < IT; it++) {
        const int item = th + 256 * it, c = item % C, l = item / C;
        double r[EA];
#pragma unroll
        for (int k = 0; k < EA; k++) {
          const double v = fbc_term(y[it][0][k], cw[0], cq[0], ar.q) + fbc_term(y[it][1][k], cw[1], cq[1], ar.q) +
                           fbc_term(y[it][2][k], cw[2], cq[2], ar.q);
          r[k] = f64_red(v, ar.q, ar.qinv) + fbc_term(y[it][3][k], cw[3], cq[3], ar.q);  // |.| < 1.5 q
        }
        ar.template fwd<LEA>(r, T, LOGT - 1);
#pragma unroll
        for (int k = 0; k < EA; k++)
          buf[(l + 16 * k) * CP + c] = (uint64_t)__double_as_longlong(r[k]);
      }
      if (z + 1 < nsteps)
        tw_store(z + 1);
      __syncthreads();
      if (z + 2 < nsteps)
        tw_load(z + 2);
      const int c = th % C, g = th / C;
      const unsigned vo = (unsigned)(16 * g) * n2 + c;
      double r[16];
#pragma unroll
      for (int k = 0; k < 16; k++)
        r[k] = __longlong_as_double((long long)buf[(16 * g + k) * CP + c]);
      ar.template fwd<4>(r, T + 16 * g, 3);
#pragma unroll
      for (int k = 0; k < 16; k++)  // T1: read lazily by the row passes (the double itself)
        ST_STREAM((uint64_t)__double_as_longlong(r[k]), &(out + (size_t)k * n2)[vo]);
    }(make_f64c<decltype(LZ)::value, !DB>(q, twl[z % NB]));
  };
  for (unsigned v = 0; v < nlz; v++)
    target(v, std::true_type{});
  for (unsigned v = nlz; v < nt; v++)
    target(v, std::false_type{});
}

// dn_cols_kernel<., ., X5, true, true> for every modulus below 2^51 (the split
// key switch's ModDown at the headline's prime sets), scheduled like
// ks_colsf_kernel: the steps' column twiddles in LDS (double-buffered: every
// step here starts with a barrier, as the single data tile and the fifth drop
// limb's LDS slots leave no room for a second tile), the conversion constants
// and moduli staged once, the lazy-reduction choice at compile time.
template <int LOGT, bool X5>
__global__ void __launch_bounds__(256, 2) dn_colsf_kernel(const uint64_t *X, size_t x_pstride, size_t x_off,
                                                           uint64_t *conv, unsigned logn, unsigned lvl, unsigned L,
                                                           unsigned members, unsigned ngroups, DownTable tab, Tw2 tw,
                                                           const ModConst *mcs)
{
  constexpr int NT = 8, T = 1 << LOGT, C = 4096 / T, LEA = LOGT - 4, EA = 1 << LEA, CP = C + 1, IT = C / 16;
  constexpr int TWW = 2 * T, TWP = (TWW + 255) / 256;
  __shared__ __attribute__((aligned(16))) uint64_t lds[T * CP];
  __shared__ double y5[X5 ? 4096 : 1];  // fifth drop limb, thread-private slots (it EA + k) 256 + th
  __shared__ __attribute__((aligned(16))) double twl[2][TWW];
  __shared__ __attribute__((aligned(16))) double cst[NT][5][2];
  __shared__ double qs[5 + NT];
  __shared__ unsigned ord[NT];
  const unsigned n2 = 1u << (logn - LOGT);
  const unsigned tiles = n2 / C;
  unsigned grp, mi;  // group = (poly, tile) on one XCD; members = target batches
  if (!xcd_group(members, ngroups, grp, mi))
    return;
  const unsigned tile = grp % tiles, p = grp / tiles;
  const unsigned keep = tab.keep, nd = tab.nd;
  if (mi * NT >= keep)
    return;
  const unsigned nt = min((unsigned)NT, keep - mi * NT), nsteps = nd + nt;
  const int th = threadIdx.x;
  // step z: drop limb z (slot keep + z, inverse table), then target mi NT + z - nd
  auto step_mod = [&](unsigned z) { return basis_mod(z < nd ? keep + z : mi * NT + ord[z - nd], lvl, L); };
  double tv[TWP];
  auto tw_load = [&](unsigned z) {
    const double *src = (z < nd ? tw.invd : tw.fwdd) + ((size_t)step_mod(z) << (logn + 1));
#pragma unroll
    for (int w = 0; w < TWP; w++)
      tv[w] = th + 256 * w < TWW ? src[th + 256 * w] : 0.0;
  };
  auto tw_store = [&](unsigned z) {
#pragma unroll
    for (int w = 0; w < TWP; w++)
      if (th + 256 * w < TWW)
        twl[z & 1][th + 256 * w] = tv[w];
  };
  // targets: lazy moduli first, as in ks_colsf_kernel
  auto tq = [&](unsigned u) { return mcs[basis_mod(mi * NT + u, lvl, L)].q; };
  unsigned nlz = 0;
  for (unsigned u = 0; u < nt; u++)
    nlz += tq(u) < (1ull << 50);
  if (th < (int)nt * 10) {
    const unsigned u = th / 10, d = (th / 2) % 5, c = th & 1;
    bool lz = true;
    unsigned before = 0;
    for (unsigned u2 = 0; u2 < nt; u2++) {
      const bool l2 = tq(u2) < (1ull << 50);
      if (u2 == u)
        lz = l2;
      else if (u2 < u)
        before += l2;
    }
    const unsigned v = lz ? before : nlz + (u - before);
    cst[v][d][c] = d < nd ? tab.cdf[2 * ((size_t)d * keep + mi * NT + u) + c] : 0.0;
    if (th % 10 == 0) {
      ord[v] = u;
      qs[nd + v] = (double)tq(u);
    }
  }
  if (th < (int)nd)
    qs[th] = (double)mcs[basis_mod(keep + th, lvl, L)].q;
  tw_load(0);
  tw_store(0);
  __syncthreads();
  if (nsteps > 1)
    tw_load(1);
  const uint64_t *yb = X + p * x_pstride + x_off + (size_t)tile * C;
  // the drop limbs arrive after the inverse row pass (ksq_kernel<drop>, its
  // INTT scale folded into the key): the inverse column pass, limb by limb;
  // limbs 0..3 stay in registers
  double y[IT][4][EA];
  uint64_t pre[16];  // round A words of drop limb d (COLSF_PF: requested one step ahead)
  auto ld_limb = [&](int d) {
    const uint64_t *src = yb + ((size_t)d << logn);
    const int c = th % C, g = th / C;
    const unsigned vo = (unsigned)(16 * g) * n2 + c;
#pragma unroll
    for (int k = 0; k < 16; k++)
      pre[k] = (src + (size_t)k * n2)[vo];
  };
  ld_limb(0);
  auto invc = [&](auto D) {
    constexpr int d = decltype(D)::value;
    if (d >= (int)nd) {
      if constexpr (d < 4)
#pragma unroll
        for (int it = 0; it < IT; it++)
#pragma unroll
          for (int k = 0; k < EA; k++)
            y[it][d][k] = 0.0;
      return;
    }
    if (d && !(COLSF_PF && d < 4))  // (the fifth limb is not prefetched: with
      ld_limb(d);                    // four limbs held it spilled 52 B/lane)
    if (d)
      __syncthreads();  // the previous step's round B has read the tile
    with_f64c<(LOGT >= 8)>(qs[d], twl[d & 1], [&](const auto &ar) {
      {
        const int c = th % C, g = th / C;
        double r[16];
#pragma unroll
        for (int k = 0; k < 16; k++)
          r[k] = f64_from_u52(pre[k]);
        if (COLSF_PF && d + 1 < (int)nd && d + 1 < 4)
          ld_limb(d + 1);  // the next drop limb's words, in flight meanwhile
        ar.template inv<4>(r, T + 16 * g, 0);
#pragma unroll
        for (int k = 0; k < 16; k++)
          lds[(16 * g + k) * CP + c] = (uint64_t)__double_as_longlong(r[k]);
      }
      if (d + 1 < (int)nsteps)
        tw_store(d + 1);
      __syncthreads();
      if (d + 2 < (int)nsteps)
        tw_load(d + 2);
#pragma unroll
      for (int it = 0; it < IT; it++) {
        const int item = th + 256 * it, c = item % C, l = item / C;
        double r[EA];
#pragma unroll
        for (int k = 0; k < EA; k++)
          r[k] = __longlong_as_double((long long)lds[(l + 16 * k) * CP + c]);
        ar.template inv<LEA>(r, T, 4);
#pragma unroll
        for (int k = 0; k < EA; k++) {
          const double v0 = f64_red(r[k], ar.q, ar.qinv);
          const double v = v0 < 0 ? v0 + ar.q : v0;  // canonical (ArF64::canon_d)
          if constexpr (d < 4)
            y[it][d][k] = v;
          else if constexpr (X5)
            y5[(it * EA + k) * 256 + th] = v;
        }
      }
    });
  };
  invc(std::integral_constant<int, 0>{});
  invc(std::integral_constant<int, 1>{});
  invc(std::integral_constant<int, 2>{});
  invc(std::integral_constant<int, 3>{});
  if constexpr (X5)
    invc(std::integral_constant<int, 4>{});
  auto target = [&](unsigned v, auto LZ) {
    const unsigned z = nd + v, t = mi * NT + ord[v];
    uint64_t *out = conv + (((size_t)p * keep + t) << logn) + (size_t)tile * C;
    double cw[5], cq[5];
#pragma unroll
    for (int d = 0; d < 5; d++) {
      cw[d] = cst[v][d][0];
      cq[d] = cst[v][d][1];
    }
    const double q = qs[z];
    __syncthreads();  // the previous step's round B has read the tile
    [&](const auto &ar) {
#pragma unroll
      for (int it = 0; it < IT; it++) {
        const int item = th + 256 * it, c = item % C, l = item / C;
        double r[EA];
#pragma unroll
        for (int k = 0; k < EA; k++) {
          double v = fbc_term(y[it][0][k], cw[0], cq[0], ar.q) + fbc_term(y[it][1][k], cw[1], cq[1], ar.q) +
                     fbc_term(y[it][2][k], cw[2], cq[2], ar.q);
          v = f64_red(v, ar.q, ar.qinv) + fbc_term(y[it][3][k], cw[3], cq[3], ar.q);
          if constexpr (X5)
            v = f64_red(v + fbc_term(y5[(it * EA + k) * 256 + th], cw[4], cq[4], ar.q), ar.q, ar.qinv);
          r[k] = v;  // |v| < 2 q
        }
        ar.template fwd<LEA>(r, T, LOGT - 1);
#pragma unroll
        for (int k = 0; k < EA; k++)
          lds[(l + 16 * k) * CP + c] = (uint64_t)__double_as_longlong(r[k]);
      }
      if (z + 1 < nsteps)
        tw_store(z + 1);
      __syncthreads();
      if (z + 2 < nsteps)
        tw_load(z + 2);
      const int c = th % C, g = th / C;
      const unsigned vo = (unsigned)(16 * g) * n2 + c;
      double r[16];
#pragma unroll
      for (int k = 0; k < 16; k++)
        r[k] = __longlong_as_double((long long)lds[(16 * g + k) * CP + c]);
      ar.template fwd<4>(r, T + 16 * g, 3);
#pragma unroll
      for (int k = 0; k < 16; k++)  // conv: read lazily by ksq_kernel<keep> (the double itself)
        ST_STREAM((uint64_t)__double_as_longlong(r[k]), &(out + (size_t)k * n2)[vo]);
    }(make_f64c<decltype(LZ)::value, (LOGT >= 8)>(q, twl[z & 1]));
  };
  for (unsigned v = 0; v < nlz; v++)
    target(v, std::true_type{});
  for (unsigned v = nlz; v < nt; v++)
    target(v, std::false_type{});
}


// The batched NTT's column pass (config 2) for limbs on FP64 moduli: as
// kernels.hip's ntt2_cols_kernel (cols_tile), with the pass's T twiddle pairs
// staged in LDS -- their loads issued beside the data loads, one barrier --
// instead of global loads at every stage, and the lazy-reduction choice at
// compile time.  Same stages, same bits.
template <int LOGT, bool INV>
__global__ void __launch_bounds__(256) ntt2_colsf_kernel(LimbSet s, LimbSet o, unsigned logn, Tw2 tw,
                                                          const ModConst *mcs, const uint64_t *post)
{
  constexpr int T = 1 << LOGT, C = 4096 / T, CP = C + 1, LEA = LOGT - 4, EA = 1 << LEA, IT = C / 16;
  constexpr int TWW = 2 * T, TWP = (TWW + 255) / 256;
  __shared__ __attribute__((aligned(16))) uint64_t lds[T * CP];
  __shared__ __attribute__((aligned(16))) double twl[TWW];
  const unsigned n2 = 1u << (logn - LOGT);
  unsigned v, tile;
  pm_decode(s, n2 / C, v, tile);
  const unsigned m = s.mod(v);
  const ModConst mc = mcs[m];
  const uint64_t *x = s.limb(v, logn) + (size_t)tile * C;
  uint64_t *y = o.limb(v, logn) + (size_t)tile * C;
  const int th = threadIdx.x;
  const double *src = (INV ? tw.invd : tw.fwdd) + ((size_t)m << (logn + 1));
  // the whole body per lazy-reduction choice (a branch between loaded data and
  // its transform spilled)
  auto body = [&](auto LZ) {
    double tv[TWP];
#pragma unroll
    for (int w = 0; w < TWP; w++)
      tv[w] = th + 256 * w < TWW ? src[th + 256 * w] : 0.0;
    const auto ar = make_f64c<decltype(LZ)::value>((double)mc.q, twl);
    if constexpr (!INV) {
      // round A: rows l + 16 k (distances T/2 .. 16), loaded beside the twiddles
      double r[IT][EA];
#pragma unroll
      for (int it = 0; it < IT; it++) {
        const int item = th + 256 * it, c = item % C, l = item / C;
        const unsigned vo = (unsigned)l * n2 + c;
#pragma unroll
        for (int k = 0; k < EA; k++)
          r[it][k] = f64_from_u52((x + (size_t)(16 * k) * n2)[vo]);
      }
#pragma unroll
      for (int w = 0; w < TWP; w++)
        if (th + 256 * w < TWW)
          twl[th + 256 * w] = tv[w];
      __syncthreads();
#pragma unroll
      for (int it = 0; it < IT; it++) {
        const int item = th + 256 * it, c = item % C, l = item / C;
        ar.template fwd<LEA>(r[it], T, LOGT - 1);
#pragma unroll
        for (int k = 0; k < EA; k++)
          lds[(l + 16 * k) * CP + c] = (uint64_t)__double_as_longlong(r[it][k]);
      }
      __syncthreads();
      // round B: rows 16 g + k (distances 8 .. 1)
      const int c = th % C, g = th / C;
      const unsigned vo = (unsigned)(16 * g) * n2 + c;
      double rb[16];
#pragma unroll
      for (int k = 0; k < 16; k++)
        rb[k] = __longlong_as_double((long long)lds[(16 * g + k) * CP + c]);
      ar.template fwd<4>(rb, T + 16 * g, 3);
#pragma unroll
      for (int k = 0; k < 16; k++)
        (y + (size_t)k * n2)[vo] = ar.store_lazy(rb[k]);  // the row pass reads it lazily
    } else {
      // final scale: n^-1, or a caller constant per limb slot
      const uint64_t sw = post ? post[2 * (v % s.per)] : mc.ninv;
      const int c = th % C, g = th / C;
      const unsigned vo = (unsigned)(16 * g) * n2 + c;
      double ra[16];
#pragma unroll
      for (int k = 0; k < 16; k++)
        ra[k] = f64_from_u52((x + (size_t)k * n2)[vo]);
#pragma unroll
      for (int w = 0; w < TWP; w++)
        if (th + 256 * w < TWW)
          twl[th + 256 * w] = tv[w];
      __syncthreads();
      ar.template inv<4>(ra, T + 16 * g, 0);
#pragma unroll
      for (int k = 0; k < 16; k++)
        lds[(16 * g + k) * CP + c] = (uint64_t)__double_as_longlong(ra[k]);
      __syncthreads();
#pragma unroll
      for (int it = 0; it < IT; it++) {
        const int item = th + 256 * it, c2 = item % C, l = item / C;
        const unsigned vo2 = (unsigned)l * n2 + c2;
        double r[EA];
#pragma unroll
        for (int k = 0; k < EA; k++)
          r[k] = __longlong_as_double((long long)lds[(l + 16 * k) * CP + c2]);
        ar.template inv<LEA>(r, T, 4);
#pragma unroll
        for (int k = 0; k < EA; k++)
          (y + (size_t)(16 * k) * n2)[vo2] = ar.mulc(r[k], sw, 0);
      }
    }
  };
  if (mc.q < (1ull << 50))
    body(std::true_type{});
  else
    body(std::false_type{});
}

void ntt2_colsf_launch(int logt, bool inv, unsigned blocks, const LimbSet &in, const LimbSet &out,
                       const uint64_t *post)
{
  const Tw2 tw{G.tw2, G.itw2, G.twd, G.itwd};
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, G.stream, in, out, G.logn, tw, G.dev.mc,
                       inv ? post : (const uint64_t *)nullptr);
  };
  switch (logt) {
  case 6: inv ? go(ntt2_colsf_kernel<6, true>) : go(ntt2_colsf_kernel<6, false>); break;
  case 7: inv ? go(ntt2_colsf_kernel<7, true>) : go(ntt2_colsf_kernel<7, false>); break;
  case 8: inv ? go(ntt2_colsf_kernel<8, true>) : go(ntt2_colsf_kernel<8, false>); break;
  default: gpqhe_die("ntt2_colsf: column length 2^%d", logt);
  }
}

template <int LOGT, int NT>
static void ks_colsf_go(dim3 grid, const uint64_t *y, size_t y_stride, uint64_t *T1, size_t t1_stride, unsigned lvl,
                        unsigned nm, unsigned ndig, unsigned members, unsigned ngroups, const UpTable &tab,
                        const Tw2 &tw)
{
  hipLaunchKernelGGL((ks_colsf_kernel<LOGT, NT>), grid, dim3(256), 0, G.stream, y, y_stride, T1, t1_stride, G.logn, lvl, G.L,
                     nm, ndig, members, ngroups, tab, tw, G.dev.mc);
}

void ks_colsf_launch(int logt, int nt, dim3 grid, const uint64_t *y, size_t y_stride, uint64_t *T1, size_t t1_stride,
                     unsigned lvl, unsigned nm, unsigned ndig, unsigned members, unsigned ngroups, const UpTable &tab,
                     const Tw2 &tw)
{
#define KSF(LT, N) ks_colsf_go<LT, N>(grid, y, y_stride, T1, t1_stride, lvl, nm, ndig, members, ngroups, tab, tw)
  if (nt == 8 && logt == 6)
    KSF(6, 8);
  else if (nt == 8 && logt == 7)
    KSF(7, 8);
  else if (nt == 8 && logt == 8)
    KSF(8, 8);
  else if (nt == 12 && logt == 7)
    KSF(7, 12);
  else if (nt == 12 && logt == 8)
    KSF(8, 12);
  else
    gpqhe_die("ks_colsf: column length 2^%d, %d targets", logt, nt);
#undef KSF
}

template <int LOGT, bool X5>
static void dn_colsf_go(dim3 grid, const uint64_t *X, size_t x_pstride, size_t x_off, uint64_t *conv, unsigned lvl,
                        unsigned members, unsigned ngroups, const DownTable &tab, const Tw2 &tw)
{
  hipLaunchKernelGGL((dn_colsf_kernel<LOGT, X5>), grid, dim3(256), 0, G.stream, X, x_pstride, x_off, conv, G.logn,
                     lvl, G.L, members, ngroups, tab, tw, G.dev.mc);
}

void dn_colsf_launch(int logt, dim3 grid, const uint64_t *X, size_t x_pstride, size_t x_off, uint64_t *conv,
                     unsigned lvl, unsigned members, unsigned ngroups, const DownTable &tab, const Tw2 &tw)
{
  const bool x5 = tab.nd > 4;
  switch (logt) {
  case 6:
    x5 ? dn_colsf_go<6, true>(grid, X, x_pstride, x_off, conv, lvl, members, ngroups, tab, tw)
       : dn_colsf_go<6, false>(grid, X, x_pstride, x_off, conv, lvl, members, ngroups, tab, tw);
    break;
  case 7:
    x5 ? dn_colsf_go<7, true>(grid, X, x_pstride, x_off, conv, lvl, members, ngroups, tab, tw)
       : dn_colsf_go<7, false>(grid, X, x_pstride, x_off, conv, lvl, members, ngroups, tab, tw);
    break;
  case 8:
    x5 ? dn_colsf_go<8, true>(grid, X, x_pstride, x_off, conv, lvl, members, ngroups, tab, tw)
       : dn_colsf_go<8, false>(grid, X, x_pstride, x_off, conv, lvl, members, ngroups, tab, tw);
    break;
  default: gpqhe_die("dn_colsf: column length 2^%d", logt);
  }
}
