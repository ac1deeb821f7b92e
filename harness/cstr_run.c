/*
 * cstr_run.c - config 4 driver: HECTR's closed-loop CSTR
 * simulation for an arbitrary number of control steps, through the
 * reference's own unchanged libhectr.so.
 *
 *   cstr-run mpc   N out.bin    plaintext regulator: ctr_simulate
 *                               (reference src/ctr.c:363-443)
 *   cstr-run hempc N out.bin    encrypted regulator: hectr_simulate
 *                               (reference src/ctr.c:500-618) on whichever
 *                               libgpqhe.so the loader finds
 *
 * The reference's own harness hard-codes N = 40 (tests/hectr.c:795); this
 * driver is not a modified copy of it.  The plant and controller setup is the
 * problem definition the harness uses (tests/hectr.c:522-527 steady state,
 * :761-802 linearisation, output matrix, disturbance model, selector and the
 * +10 % inlet-flow step from step 9), restated here as data; every numerical
 * routine is the reference's (cstr_linearize, cstr_ode, cstr_jacobian and the
 * two simulate functions, all from libhectr.so).  horizon = N/10 and slots
 * follow from N inside the reference (src/ctr.c:376,511).
 *
 * Output: the trajectory in the harness's record format (tests/hectr.c:
 * 812-817: uint32 k, double x[3], double u[2], N + 1 records, the last u
 * repeated), and on stderr the libpmu timings the reference prints itself
 * (TEST_DO/TEST_DONE around keygen and the closed loop, src/ctr.c:528-597).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../GPQHE/src/gpqhe.h"
#include "hectr.h"

/* steady state of the CSTR (tests/hectr.c:522-527) */
static const double c_ss = 0.878, T_ss = 324.5, h_ss = 0.659; /* kmol/m^3, K, m */
static const double Tc_ss = 300, F_ss = 0.1, F0_ss = 0.1;       /* K, m^3/min, m^3/min */

enum { NX = 3, NU = 2, NP = 1, NY = NX, ND = 2 };

int main(int argc, char **argv)
{
  if (argc != 4 || (strcmp(argv[1], "mpc") && strcmp(argv[1], "hempc"))) {
    fprintf(stderr, "usage: %s mpc|hempc N out.bin\n", argv[0]);
    return 2;
  }
  const int enc = !strcmp(argv[1], "hempc");
  const unsigned int N = (unsigned int)strtoul(argv[2], NULL, 0);
  if (N < 10) {
    fprintf(stderr, "N >= 10 (the MPC horizon is N/10)\n");
    return 2;
  }
  const double xs[NX] = {c_ss, T_ss, h_ss}, us[NU] = {Tc_ss, F_ss}, ps[NP] = {F0_ss};
  const double dt = 1;
  double A[NX * NX], B[NX * NU], Bp[NX * NP], C[NY * NX];
  cstr_linearize(A, B, Bp, NX, NU, NP, xs, us, ps, dt);
  memset(C, 0, sizeof(C));
  for (unsigned int i = 0; i < NX; i++)
    C[i * NX + i] = 1; /* every state measured */
  /* offset-free disturbance model: concentration and height offsets */
  double Bd[NX * ND], Cd[NY * ND] = {1, 0, 0, 0, 0, 1};
  memset(Bd, 0, sizeof(Bd));
  /* selector: track concentration and height */
  const double Hr[NU * NY] = {1, 0, 0, 0, 0, 1};

  double *x = calloc((size_t)NX * (N + 1), sizeof(double));
  double *u = calloc((size_t)NU * N, sizeof(double));
  double *p = calloc((size_t)NP * N, sizeof(double));
  if (!x || !u || !p)
    return 1;
  for (unsigned int i = 9; i < NP * N; i++)
    p[i] = 0.1 * F0_ss; /* inlet-flow disturbance from step 9 */

  if (enc)
    hectr_simulate(x, u, p, NX, NU, NP, NY, ND, A, B, C, Bd, Cd, Hr, xs, us, ps, cstr_ode, cstr_jacobian, dt, N);
  else
    ctr_simulate(x, u, p, NX, NU, NP, NY, ND, A, B, C, Bd, Cd, Hr, xs, us, ps, cstr_ode, cstr_jacobian, dt, N);

  FILE *fd = fopen(argv[3], "wb");
  if (!fd) {
    perror(argv[3]);
    return 1;
  }
  for (unsigned int k = 0; k < N + 1; k++) {
    const double *uk = &u[(k < N ? k : N - 1) * NU];
    fwrite(&k, sizeof(unsigned int), 1, fd);
    fwrite(&x[k * NX], sizeof(double), NX, fd);
    fwrite(uk, sizeof(double), NU, fd);
  }
  fclose(fd);
  free(x);
  free(u);
  free(p);
  return 0;
}
