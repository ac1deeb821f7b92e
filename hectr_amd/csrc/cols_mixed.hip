// cols_mixed.hip - the split key switch's column kernels for prime sets that
// mix FP64 moduli (< 2^51) and wider integer ones (the conventional 60-bit q0
// and special primes): ks_colsm_kernel (ModUp: inverse column pass of the
// digit, conversion, forward column pass -> T1) and dn_colsm_kernel (ModDown:
// the same for the dropped limbs -> conv).  They replace kernels.hip's
// ks_cols4_kernel<., 8, true, false> and dn_cols_kernel<., 8, ., false, true>
// with the same values, scheduled as cols_f64.hip's kernels: every step's
// column twiddles in LDS (staged ahead), the conversion constants staged once,
// and the arithmetic policy of every transform fixed at compile time -- the
// targets run grouped by policy (integer, FP64 lazy, FP64), one loop each.
// (The old kernels chose the policy at run time inside their target loop and
// spilled 84 B/lane.)  The conversion is the 128-bit integer sum with one
// Montgomery REDC, as in the old kernels: a 60-bit source limb rules out the
// exact FP64 products.
#include "ntt_device.h"
#include "tables.h"

#include <type_traits>

// ArInt over an LDS twiddle table: entries [0, T) of the modulus' (w, w')
// table for the step's direction.
struct ArIntC : ArInt {};

__device__ __forceinline__ ArIntC make_intc(uint64_t q, const uint64_t *twl)
{
  ArIntC a;
  a.q = q;
  a.tw = a.itw = twl;
  return a;
}

// policy class of modulus q: 0 integer (q >= 2^51), 1 FP64 lazy (q < 2^50), 2 FP64
__device__ __forceinline__ int pol_class(uint64_t q)
{
  return q >= F64_QMAX ? 0 : q < F64_LAZY ? 1 : 2;
}

// f(policy) for modulus q with twiddles at twl (raw 64-bit words)
template <bool SB = false, class F>
__device__ __forceinline__ void with_polc(uint64_t q, const uint64_t *twl, F &&f)
{
  const int c = pol_class(q);
  if (c == 0)
    f(make_intc(q, twl));
  else if (c == 1)
    f(make_f64c<true, SB>((double)q, (const double *)twl));
  else
    f(make_f64c<false, SB>((double)q, (const double *)twl));
}

template <int C, bool SB = false>
__device__ __forceinline__ auto polc_of(uint64_t q, const uint64_t *twl)
{
  if constexpr (C == 0)
    return make_intc(q, twl);
  else
    return make_f64c<C == 1, SB>((double)q, (const double *)twl);
}

// Targets of a block in policy-class order: position v holds target ord[v];
// cnt[c] targets of class c.  Every thread computes the same order.
template <int NT, class Q>
__device__ __forceinline__ void class_order(unsigned nt, Q &&tq, unsigned (&cnt)[3], unsigned u, unsigned &v)
{
  cnt[0] = cnt[1] = cnt[2] = 0;
  for (unsigned u2 = 0; u2 < nt; u2++)
    cnt[pol_class(tq(u2))]++;
  const int cu = u < nt ? pol_class(tq(u)) : 0;
  unsigned before = 0;
  for (unsigned u2 = 0; u2 < u && u2 < nt; u2++)
    before += pol_class(tq(u2)) == cu;
  v = (cu > 0 ? cnt[0] : 0) + (cu > 1 ? cnt[1] : 0) + before;
}

template <int LOGT>
__global__ void __launch_bounds__(256, 2) ks_colsm_kernel(const uint64_t *ybuf, size_t y_stride, uint64_t *T1,
                                                           size_t t1_stride, unsigned logn, unsigned lvl,
                                                           unsigned L, unsigned nm, unsigned ndig, unsigned members,
                                                           unsigned ngroups, UpTable tab, Tw2 tw,
                                                           const ModConst *mcs)
{
  constexpr int NT = 8, T = 1 << LOGT, C = 4096 / T, LEA = LOGT - 4, EA = 1 << LEA, CP = C + 1, IT = C / 16;
  constexpr int TWW = 2 * T, TWP = (TWW + 255) / 256;
  constexpr bool DB = LOGT <= 7;  // double-buffered data tiles, else a barrier before every step
  constexpr int NB = DB ? 3 : 2;
  __shared__ __attribute__((aligned(16))) uint64_t lds[DB ? 2 : 1][T * CP];
  __shared__ __attribute__((aligned(16))) uint64_t twl[NB][TWW];
  __shared__ uint64_t cst[NT][4];
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
  auto slot = [&](unsigned u) {
    const unsigned ui = mi * NT + u;
    return ui < lo ? ui : ui + na;
  };
  auto tq = [&](unsigned u) { return mcs[basis_mod(slot(u), lvl, L)].q; };
  unsigned cnt[3], v0;
  class_order<NT>(nt, tq, cnt, th < (int)nt ? th : 0, v0);
  if (th < (int)nt)
    ord[v0] = th;
  if (th < (int)nt * 4) {
    const unsigned u = th / 4, i = th % 4;
    unsigned cn[3], v;
    class_order<NT>(nt, tq, cn, u, v);
    cst[v][i] = i < na ? tab.c[((size_t)j * 8 + i) * nm + slot(u)] : 0;
  }
  __syncthreads();  // ord, before the step moduli below read it
  auto step_mod = [&](unsigned z) { return z < na ? lo + z : basis_mod(slot(ord[z - na]), lvl, L); };
  uint64_t tv[TWP];
  auto tw_load = [&](unsigned z) {
    const unsigned m = step_mod(z);
    const bool f = mcs[m].q < F64_QMAX;
    const uint64_t *src = (const uint64_t *)(z < na ? (f ? (const void *)tw.invd : (const void *)tw.inv)
                                                    : (f ? (const void *)tw.fwdd : (const void *)tw.fwd)) +
                          ((size_t)m << (logn + 1));
#pragma unroll
    for (int w = 0; w < TWP; w++)
      tv[w] = th + 256 * w < TWW ? src[th + 256 * w] : 0;
  };
  auto tw_store = [&](unsigned z) {
#pragma unroll
    for (int w = 0; w < TWP; w++)
      if (th + 256 * w < TWW)
        twl[z % NB][th + 256 * w] = tv[w];
  };
  tw_load(0);
  tw_store(0);
  __syncthreads();
  if (nsteps > 1)
    tw_load(1);
  const uint64_t *yb = ybuf + p * y_stride + ((size_t)lo << logn) + (size_t)tile * C;
  uint64_t y[IT][4][EA];  // canonical residues of the digit's limbs
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
          y[it][i][k] = 0;
      return;
    }
    uint64_t *buf = lds[DB ? i & 1 : 0];
    if (!DB && i)
      __syncthreads();  // the previous step's round B has read the tile
    with_polc<!DB>(mcs[lo + i].q, twl[i % NB], [&](const auto &ar) {
      using A = std::decay_t<decltype(ar)>;
      using V = typename A::V;
      {
        const int g = th / C, c = th % C;
        V r[16];
#pragma unroll
        for (int k = 0; k < 16; k++)
          r[k] = A::load(pre[k]);
        if (i + 1 < (int)na)
          ld_limb(i + 1);  // the next limb's words, in flight meanwhile
        ar.template inv<4>(r, T + 16 * g, 0);
#pragma unroll
        for (int k = 0; k < 16; k++)
          buf[(16 * g + k) * CP + c] = A::bits(r[k]);
      }
      if (i + 1 < (int)nsteps)
        tw_store(i + 1);
      __syncthreads();
      if (i + 2 < (int)nsteps)
        tw_load(i + 2);
#pragma unroll
      for (int it = 0; it < IT; it++) {
        const int item = th + 256 * it, c = item % C, l = item / C;
        V r[EA];
#pragma unroll
        for (int k = 0; k < EA; k++)
          r[k] = A::unbits(buf[(l + 16 * k) * CP + c]);
        ar.template inv<LEA>(r, T, 4);
#pragma unroll
        for (int k = 0; k < EA; k++)
          y[it][i][k] = ar.canon(r[k]);
      }
    });
  };
  invc(std::integral_constant<int, 0>{});
  invc(std::integral_constant<int, 1>{});
  invc(std::integral_constant<int, 2>{});
  invc(std::integral_constant<int, 3>{});
  auto target = [&](unsigned v, auto CL) {
    constexpr int CLS = decltype(CL)::value;
    const unsigned z = na + v, t = slot(ord[v]);
    uint64_t *buf = lds[DB ? z & 1 : 0];
    uint64_t *out = T1 + p * t1_stride + (((size_t)j * nm + t) << logn) + (size_t)tile * C;
    uint64_t cc[4];
#pragma unroll
    for (int i = 0; i < 4; i++)
      cc[i] = cst[v][i];
    const ModConst mc = mcs[basis_mod(t, lvl, L)];
    if (!DB)
      __syncthreads();  // the previous step's round B has read the tile
    const auto ar = polc_of<CLS, !DB>(mc.q, twl[z % NB]);
    using A = std::decay_t<decltype(ar)>;
    using V = typename A::V;
#pragma unroll
    for (int it = 0; it < IT; it++) {
      const int item = th + 256 * it, c = item % C, l = item / C;
      V r[EA];
#pragma unroll
      for (int k = 0; k < EA; k++) {
        unsigned __int128 acc = 0;
#pragma unroll
        for (int i = 0; i < 4; i++)
          acc += (unsigned __int128)y[it][i][k] * cc[i];
        r[k] = A::load(redc128((uint64_t)(acc >> 64), (uint64_t)acc, mc));
      }
      ar.template fwd<LEA>(r, T, LOGT - 1);
#pragma unroll
      for (int k = 0; k < EA; k++)
        buf[(l + 16 * k) * CP + c] = A::bits(r[k]);
    }
    if (z + 1 < nsteps)
      tw_store(z + 1);
    __syncthreads();
    if (z + 2 < nsteps)
      tw_load(z + 2);
    const int c = th % C, g = th / C;
    const unsigned vo = (unsigned)(16 * g) * n2 + c;
    V r[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
      r[k] = A::unbits(buf[(16 * g + k) * CP + c]);
    ar.template fwd<4>(r, T + 16 * g, 3);
#pragma unroll
    for (int k = 0; k < 16; k++)  // T1: read lazily by the row passes
      ST_STREAM(ar.store_lazy(r[k]), &(out + (size_t)k * n2)[vo]);
  };
  for (unsigned v = 0; v < cnt[0]; v++)
    target(v, std::integral_constant<int, 0>{});
  for (unsigned v = cnt[0]; v < cnt[0] + cnt[1]; v++)
    target(v, std::integral_constant<int, 1>{});
  for (unsigned v = cnt[0] + cnt[1]; v < nt; v++)
    target(v, std::integral_constant<int, 2>{});
}

template <int LOGT, bool X5>
__global__ void __launch_bounds__(256, 2) dn_colsm_kernel(const uint64_t *X, size_t x_pstride, size_t x_off,
                                                           uint64_t *conv, unsigned logn, unsigned lvl, unsigned L,
                                                           unsigned members, unsigned ngroups, DownTable tab, Tw2 tw,
                                                           const ModConst *mcs)
{
  constexpr int NT = 8, T = 1 << LOGT, C = 4096 / T, LEA = LOGT - 4, EA = 1 << LEA, CP = C + 1, IT = C / 16;
  constexpr int TWW = 2 * T, TWP = (TWW + 255) / 256;
  __shared__ __attribute__((aligned(16))) uint64_t lds[T * CP];
  __shared__ uint64_t y5[X5 ? 4096 : 1];  // fifth drop limb, thread-private slots (it EA + k) 256 + th
  __shared__ __attribute__((aligned(16))) uint64_t twl[2][TWW];
  __shared__ uint64_t cst[NT][5];
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
  auto tq = [&](unsigned u) { return mcs[basis_mod(mi * NT + u, lvl, L)].q; };
  unsigned cnt[3], v0;
  class_order<NT>(nt, tq, cnt, th < (int)nt ? th : 0, v0);
  if (th < (int)nt)
    ord[v0] = th;
  if (th < (int)nt * 5) {
    const unsigned u = th / 5, d = th % 5;
    unsigned cn[3], v;
    class_order<NT>(nt, tq, cn, u, v);
    cst[v][d] = d < nd ? tab.cf[(size_t)d * keep + mi * NT + u] : 0;
  }
  __syncthreads();
  auto step_mod = [&](unsigned z) { return basis_mod(z < nd ? keep + z : mi * NT + ord[z - nd], lvl, L); };
  uint64_t tv[TWP];
  auto tw_load = [&](unsigned z) {
    const unsigned m = step_mod(z);
    const bool f = mcs[m].q < F64_QMAX;
    const uint64_t *src = (const uint64_t *)(z < nd ? (f ? (const void *)tw.invd : (const void *)tw.inv)
                                                    : (f ? (const void *)tw.fwdd : (const void *)tw.fwd)) +
                          ((size_t)m << (logn + 1));
#pragma unroll
    for (int w = 0; w < TWP; w++)
      tv[w] = th + 256 * w < TWW ? src[th + 256 * w] : 0;
  };
  auto tw_store = [&](unsigned z) {
#pragma unroll
    for (int w = 0; w < TWP; w++)
      if (th + 256 * w < TWW)
        twl[z & 1][th + 256 * w] = tv[w];
  };
  tw_load(0);
  tw_store(0);
  __syncthreads();
  if (nsteps > 1)
    tw_load(1);
  const uint64_t *yb = X + p * x_pstride + x_off + (size_t)tile * C;
  uint64_t y[IT][4][EA];
  uint64_t pre[16];
  auto ld_limb = [&](int d) {
    const uint64_t *src = yb + ((size_t)d << logn);
    const int c = th % C, g = th / C;
    const unsigned vo = (unsigned)(16 * g) * n2 + c;
#pragma unroll
    for (int k = 0; k < 16; k++)
      pre[k] = (src + (size_t)k * n2)[vo];
  };
  ld_limb(0);
  // the drop limbs arrive after the inverse row pass (ksq_kernel<drop>, its
  // INTT scale folded into the key): the inverse column pass, limb by limb
  auto invc = [&](auto D) {
    constexpr int d = decltype(D)::value;
    if (d >= (int)nd) {
      if constexpr (d < 4)
#pragma unroll
        for (int it = 0; it < IT; it++)
#pragma unroll
          for (int k = 0; k < EA; k++)
            y[it][d][k] = 0;
      return;
    }
    if (d == 4)
      ld_limb(d);  // (not prefetched: four limbs are held then)
    if (d)
      __syncthreads();  // the previous step's round B has read the tile
    with_polc<(LOGT >= 8)>(mcs[basis_mod(keep + d, lvl, L)].q, twl[d & 1], [&](const auto &ar) {
      using A = std::decay_t<decltype(ar)>;
      using V = typename A::V;
      {
        const int c = th % C, g = th / C;
        V r[16];
#pragma unroll
        for (int k = 0; k < 16; k++)
          r[k] = A::load(pre[k]);
        if (d + 1 < (int)nd && d + 1 < 4)
          ld_limb(d + 1);  // the next drop limb's words, in flight meanwhile
        ar.template inv<4>(r, T + 16 * g, 0);
#pragma unroll
        for (int k = 0; k < 16; k++)
          lds[(16 * g + k) * CP + c] = A::bits(r[k]);
      }
      if (d + 1 < (int)nsteps)
        tw_store(d + 1);
      __syncthreads();
      if (d + 2 < (int)nsteps)
        tw_load(d + 2);
#pragma unroll
      for (int it = 0; it < IT; it++) {
        const int item = th + 256 * it, c = item % C, l = item / C;
        V r[EA];
#pragma unroll
        for (int k = 0; k < EA; k++)
          r[k] = A::unbits(lds[(l + 16 * k) * CP + c]);
        ar.template inv<LEA>(r, T, 4);
#pragma unroll
        for (int k = 0; k < EA; k++) {
          const uint64_t v = ar.canon(r[k]);
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
  auto target = [&](unsigned v, auto CL) {
    constexpr int CLS = decltype(CL)::value;
    const unsigned z = nd + v, t = mi * NT + ord[v];
    uint64_t *out = conv + (((size_t)p * keep + t) << logn) + (size_t)tile * C;
    uint64_t cc[5];
#pragma unroll
    for (int d = 0; d < 5; d++)
      cc[d] = cst[v][d];
    const ModConst mc = mcs[basis_mod(t, lvl, L)];
    __syncthreads();  // the previous step's round B has read the tile
    const auto ar = polc_of<CLS, (LOGT >= 8)>(mc.q, twl[z & 1]);
    using A = std::decay_t<decltype(ar)>;
    using V = typename A::V;
#pragma unroll
    for (int it = 0; it < IT; it++) {
      const int item = th + 256 * it, c = item % C, l = item / C;
      V r[EA];
#pragma unroll
      for (int k = 0; k < EA; k++) {
        unsigned __int128 acc = 0;
#pragma unroll
        for (int d = 0; d < 4; d++)
          acc += (unsigned __int128)y[it][d][k] * cc[d];
        if constexpr (X5)
          acc += (unsigned __int128)y5[(it * EA + k) * 256 + th] * cc[4];
        r[k] = A::load(redc128((uint64_t)(acc >> 64), (uint64_t)acc, mc));
      }
      ar.template fwd<LEA>(r, T, LOGT - 1);
#pragma unroll
      for (int k = 0; k < EA; k++)
        lds[(l + 16 * k) * CP + c] = A::bits(r[k]);
    }
    if (z + 1 < nsteps)
      tw_store(z + 1);
    __syncthreads();
    if (z + 2 < nsteps)
      tw_load(z + 2);
    const int c = th % C, g = th / C;
    const unsigned vo = (unsigned)(16 * g) * n2 + c;
    V r[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
      r[k] = A::unbits(lds[(16 * g + k) * CP + c]);
    ar.template fwd<4>(r, T + 16 * g, 3);
#pragma unroll
    for (int k = 0; k < 16; k++)  // conv: read lazily by ksq_kernel<keep>
      ST_STREAM(ar.store_lazy(r[k]), &(out + (size_t)k * n2)[vo]);
  };
  for (unsigned v = 0; v < cnt[0]; v++)
    target(v, std::integral_constant<int, 0>{});
  for (unsigned v = cnt[0]; v < cnt[0] + cnt[1]; v++)
    target(v, std::integral_constant<int, 1>{});
  for (unsigned v = cnt[0] + cnt[1]; v < nt; v++)
    target(v, std::integral_constant<int, 2>{});
}

void ks_colsm_launch(int logt, dim3 grid, const uint64_t *y, size_t y_stride, uint64_t *T1, size_t t1_stride,
                     unsigned lvl, unsigned nm, unsigned ndig, unsigned members, unsigned ngroups, const UpTable &tab,
                     const Tw2 &tw)
{
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, G.stream, y, y_stride, T1, t1_stride, G.logn, lvl, G.L, nm, ndig,
                       members, ngroups, tab, tw, G.dev.mc);
  };
  switch (logt) {
  case 6: go(ks_colsm_kernel<6>); break;
  case 7: go(ks_colsm_kernel<7>); break;
  case 8: go(ks_colsm_kernel<8>); break;
  default: gpqhe_die("ks_colsm: column length 2^%d", logt);
  }
}

void dn_colsm_launch(int logt, dim3 grid, const uint64_t *X, size_t x_pstride, size_t x_off, uint64_t *conv,
                     unsigned lvl, unsigned members, unsigned ngroups, const DownTable &tab, const Tw2 &tw)
{
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, G.stream, X, x_pstride, x_off, conv, G.logn, lvl, G.L, members,
                       ngroups, tab, tw, G.dev.mc);
  };
  const bool x5 = tab.nd > 4;
  switch (logt) {
  case 6: x5 ? go(dn_colsm_kernel<6, true>) : go(dn_colsm_kernel<6, false>); break;
  case 7: x5 ? go(dn_colsm_kernel<7, true>) : go(dn_colsm_kernel<7, false>); break;
  case 8: x5 ? go(dn_colsm_kernel<8, true>) : go(dn_colsm_kernel<8, false>); break;
  default: gpqhe_die("dn_colsm: column length 2^%d", logt);
  }
}
