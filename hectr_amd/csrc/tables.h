// tables.h - basis-conversion tables of the key switch (kernels.hip builds
// them per level; the column kernels of kernels.hip and cols_f64.hip read
// them).
#pragma once

#include <stdint.h>

// ModUp table for level lvl, digit j with limbs [lo, hi) (na = hi - lo):
//   y[i] = [(Qj/q_i)^-1]_{q_i} (+ Shoup)     i in digit
//   c[i][t] = [Qj/q_i]_{mod_t}               t in basis_qp(lvl)
struct UpDigit {
  uint32_t lo, na, pad0, pad1;
  uint64_t y[8], yp[8];
};

struct UpTable {
  UpDigit *dig;   // [ndig]
  uint64_t *c;    // [ndig][8][nm]  [Qj/q_i]_t 2^64 mod q_t (Montgomery form)
  uint64_t *ysc;  // [lvl][2]       n^-1 [(Qj/q_i)^-1]_{q_i} + Shoup (folded into the INTT)
  double *cd;     // [ndig][8][nm][2] ([Qj/q_i]_t, that / q_t) as doubles (FP64 conversion)
  unsigned ndig, nm;
  int f64;        // every modulus of the basis < 2^51 (and FP64 enabled): FP64 conversion
};

// ModDown table: drop the nd basis positions [keep, nm) (kernels.hip:
// down_table), keep basis positions [0, keep).
struct DownTable {
  uint64_t *ysc;     // [nd][2]     n^-1 [(Dprod/d)^-1]_d + Shoup (folded into the INTT)
  uint64_t *y, *yp;  // [nd]        [(Dprod/d)^-1]_d
  uint64_t *c;       // [nd][keep]  [Dprod/d]_t
  uint64_t *dinv, *dinvp;  // [keep]  [Dprod^-1]_t
  double *cd;        // [nd][keep][2] ([Dprod/d]_t, that / q_t) as doubles (FP64 conversion)
  // Split key switch (mul_split_launch): the ModDown's constant factors folded
  // into the relinearization key (ksq kernels, per basis slot) and into the
  // conversion constants, so no kernel multiplies by them:
  //   kept slot t:    key x [Dprod^-1]_t; conversion [Dprod/d]_t [Dprod^-1]_t = [d^-1]_t
  //   dropped slot t: key x n^-1 [(Dprod/d)^-1]_d (the INTT's scale, ysc)
  uint64_t *ksc;     // [nm]        key scale s_t
  uint64_t *kps;     // [nm][2]     [P s_t]_t + Shoup (the P (d0, d1) term of q slots)
  uint64_t *cf;      // [nd][keep]  [d^-1]_t (Montgomery form)
  double *cdf;       // [nd][keep][2] ([d^-1]_t, that / q_t)
  unsigned keep, nd;
  int f64;           // every modulus < 2^51 (and FP64 enabled): FP64 conversion
};
