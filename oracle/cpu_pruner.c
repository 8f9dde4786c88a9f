/*
 * cpu_pruner.c -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
 *
 * Plain-C restatement of the pruning log-likelihood and its gradient, used
 *   (1) by tests/ as a second, fast oracle for larger parity cases, and
 *   (2) by bench.py's cpu_baseline leg as the timed CPU reference ("port").
 * Never linked into or called by the product path.
 *
 * It follows the loop structure of the Stan code phylostan emits -- site
 * outer, node, category inner (phylostan/generate_script.py:998-1011 and the
 * other three variants :984-997, :1013-1040) -- in fp64 without rescaling,
 * with P-matrices as in :755-892 (JC69 closed form; HKY / GTR through the
 * eigendecomposition of the symmetrised rate matrix, here by Jacobi
 * rotations) and Weibull rates supplied by the caller (:249-282).  The
 * gradient is the analytic pre-order pass of pruner/tree.cpp:228-242 /
 * eigen/eigen.j2:143-167 (without the times[i] factor of eigen.j2:165).
 *
 * Inputs / outputs use the C-ABI layouts of include/phylo_hip.h.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* Jacobi rotations in the parallel ordering -- per sweep three rounds of two
 * rotations on disjoint index pairs {(0,1),(2,3)}, {(0,2),(1,3)}, {(0,3),(1,2)}:
 * both rotations' parameters from the round's A, then A <- J^T A J (columns,
 * then rows) and V <- V J.  The device (csrc/phylo_hip.hip jacobi4) runs the
 * same operations in the same order, uncontracted: the same bits. */
static void jacobi_rot(double app, double aqq, double apq, double* cs, double* sn) {
  if (apq == 0.0) {
    *cs = 1.0;
    *sn = 0.0;
    return;
  }
  /* t = sgn(theta) / (|theta| + sqrt(theta^2 + 1)), theta = d / e, divisions
   * folded: cs = den / w, sn = sgn(theta) |e| / w, den = |d| + sqrt(d^2 + e^2),
   * w = sqrt(den^2 + e^2) (the device's jacobi_rot, operation for operation) */
  const double d = aqq - app, e = 2.0 * apq;
  const double den = fabs(d) + sqrt(d * d + e * e);
  const double inv = 1.0 / sqrt(den * den + e * e);
  const double ae = fabs(e);
  *cs = den * inv;
  *sn = ((d == 0.0 || (d > 0.0) == (e > 0.0)) ? ae : -ae) * inv;
}

static void jacobi4(double A[4][4], double V[4][4], double lam[4]) {
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) V[i][j] = (i == j) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 50; ++sweep) {
    double off = 0.0, tot = 0.0;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        tot += A[i][j] * A[i][j];
        if (i != j) off += A[i][j] * A[i][j];
      }
    if (off <= 1e-32 * tot || off == 0.0) break;
    for (int r = 0; r < 3; ++r) {
      int p1 = 0, q1 = r + 1, p2 = r == 0 ? 2 : 1, q2 = r == 2 ? 2 : 3;
      double c1, s1, c2, s2;
      jacobi_rot(A[p1][p1], A[q1][q1], A[p1][q1], &c1, &s1);
      jacobi_rot(A[p2][p2], A[q2][q2], A[p2][q2], &c2, &s2);
      for (int k = 0; k < 4; ++k) {
        double a1 = A[k][p1], b1 = A[k][q1], a2 = A[k][p2], b2 = A[k][q2];
        A[k][p1] = c1 * a1 - s1 * b1;
        A[k][q1] = s1 * a1 + c1 * b1;
        A[k][p2] = c2 * a2 - s2 * b2;
        A[k][q2] = s2 * a2 + c2 * b2;
      }
      for (int k = 0; k < 4; ++k) {
        double a1 = A[p1][k], b1 = A[q1][k], a2 = A[p2][k], b2 = A[q2][k];
        A[p1][k] = c1 * a1 - s1 * b1;
        A[q1][k] = s1 * a1 + c1 * b1;
        A[p2][k] = c2 * a2 - s2 * b2;
        A[q2][k] = s2 * a2 + c2 * b2;
      }
      A[p1][q1] = A[q1][p1] = 0.0;
      A[p2][q2] = A[q2][p2] = 0.0;
      for (int k = 0; k < 4; ++k) {
        double a1 = V[k][p1], b1 = V[k][q1], a2 = V[k][p2], b2 = V[k][q2];
        V[k][p1] = c1 * a1 - s1 * b1;
        V[k][q1] = s1 * a1 + c1 * b1;
        V[k][p2] = c2 * a2 - s2 * b2;
        V[k][q2] = s2 * a2 + c2 * b2;
      }
    }
  }
  for (int i = 0; i < 4; ++i) lam[i] = A[i][i];
}

/* P-matrices pm[C][B][16] and Q P (dP/dt) qp[C][B][16] for one draw.
 * kind 0 = JC69 (generate_script.py:755-780), 1/2 = HKY/GTR (:783-892). */
void oracle_pmats(int kind, int C, int B, const double* model, const double* blens, double* pm,
                  double* qp) {
  const double* f = model;
  const double* r = model + 4;
  const double* rs = model + 10;
  double Q[4][4], m1[4][4], m2[4][4], lam[4];
  if (kind == 0) {
    for (int j = 0; j < 4; ++j)
      for (int k = 0; k < 4; ++k) Q[j][k] = (j == k) ? -1.0 : 1.0 / 3.0;
  } else {
    double R[4][4] = {{0.0, r[0], r[1], r[2]},
                      {r[0], 0.0, r[3], r[4]},
                      {r[1], r[3], 0.0, r[5]},
                      {r[2], r[4], r[5], 0.0}};
    double s = 0.0;
    for (int j = 0; j < 4; ++j) {
      double row = 0.0;
      for (int k = 0; k < 4; ++k) {
        Q[j][k] = (j == k) ? 0.0 : R[j][k] * f[k];
        row += Q[j][k];
      }
      Q[j][j] = -row;
      s -= Q[j][j] * f[j];
    }
    double A[4][4], V[4][4], sq[4];
    for (int j = 0; j < 4; ++j) sq[j] = sqrt(f[j]);
    for (int j = 0; j < 4; ++j)
      for (int k = 0; k < 4; ++k) Q[j][k] /= s;
    for (int j = 0; j < 4; ++j)
      for (int k = 0; k < 4; ++k)
        A[j][k] = (j == k) ? Q[j][j] : 0.5 * (sq[j] * Q[j][k] / sq[k] + sq[k] * Q[k][j] / sq[j]);
    jacobi4(A, V, lam);
    for (int j = 0; j < 4; ++j)
      for (int k = 0; k < 4; ++k) {
        m1[j][k] = V[j][k] / sq[j];
        m2[j][k] = V[k][j] * sq[k];
      }
  }
  for (int c = 0; c < C; ++c)
    for (int b = 0; b < B; ++b) {
      const double t = blens[b] * rs[c];
      double P[16];
      if (kind == 0) {
        double ex = exp(-t / 0.75), off = 0.25 - 0.25 * ex, d = 0.25 + 0.75 * ex;
        for (int k = 0; k < 16; ++k) P[k] = (k % 5 == 0) ? d : off;
      } else {
        double E[4];
        for (int l = 0; l < 4; ++l) E[l] = exp(lam[l] * t);
        for (int j = 0; j < 4; ++j)
          for (int k = 0; k < 4; ++k) {
            double acc = 0.0;
            for (int l = 0; l < 4; ++l) acc += m1[j][l] * E[l] * m2[l][k];
            P[j * 4 + k] = acc;
          }
      }
      double* po = pm + ((size_t)c * B + b) * 16;
      double* qo = qp + ((size_t)c * B + b) * 16;
      for (int k = 0; k < 16; ++k) po[k] = P[k];
      for (int j = 0; j < 4; ++j)
        for (int k = 0; k < 4; ++k) {
          double acc = 0.0;
          for (int l = 0; l < 4; ++l) acc += Q[j][l] * P[l * 4 + k];
          qo[j * 4 + k] = acc;
        }
    }
}

static inline void mv(const double* M, const double* v, double* r) {
  for (int j = 0; j < 4; ++j)
    r[j] = M[j * 4 + 0] * v[0] + M[j * 4 + 1] * v[1] + M[j * 4 + 2] * v[2] + M[j * 4 + 3] * v[3];
}
static inline void mtv(const double* M, const double* v, double* r) {
  for (int k = 0; k < 4; ++k)
    r[k] = M[0 * 4 + k] * v[0] + M[1 * 4 + k] * v[1] + M[2 * 4 + k] * v[2] + M[3 * 4 + k] * v[3];
}
static inline void tipv(unsigned code, double* v) {
  for (int k = 0; k < 4; ++k) v[k] = (double)((code >> k) & 1u);
}

/* One draw: log-likelihood + gradient, output vector as phy_output_len().
 * peel: 0-based rows (child1, child2, parent); unrooted => last row's child2
 * (node 2S-3) has no branch.  nthreads > 1 uses OpenMP over patterns. */
int oracle_eval(int S, int P, int C, int rooted, int kind, const uint8_t* tipcodes,
                const double* w, const int32_t* peel, const double* model, const double* blens,
                double* out, double* site_ll, int nthreads) {
  const int B = rooted ? 2 * S - 2 : 2 * S - 3;
  const int N = 2 * S - 1;
  /* [ll, grad_blens, grad_rs, grad_ps, grad_freq_root(4), grad_rates(6),
   * grad_freqs(4), dL/dP]: the 10 model-parameter slots are left zero here
   * and filled by oracle/cpu.py with the host chain rule */
  const int og = 1 + B + 2 * C + 4 + 10;
  const double* f = model;
  const double* rs = model + 10;
  const double* ps = model + 10 + C;
  const int merged = rooted ? -1 : peel[3 * (S - 2) + 1];
  const int root = peel[3 * (S - 2) + 2];
  double* pm = (double*)malloc(sizeof(double) * C * B * 16);
  double* qp = (double*)malloc(sizeof(double) * C * B * 16);
  oracle_pmats(kind, C, B, model, blens, pm, qp);
  const int outlen = og + 16 * C * B;
  memset(out, 0, sizeof(double) * outlen);
  if (nthreads < 1) nthreads = 1;
#ifdef _OPENMP
  omp_set_num_threads(nthreads);
#endif
  double ll_tot = 0.0;
#pragma omp parallel if (nthreads > 1) reduction(+ : ll_tot)
  {
    double* part = (double*)malloc(sizeof(double) * C * N * 4);  /* partials[c][node][4] */
    double* moved = (double*)malloc(sizeof(double) * C * N * 4); /* P_node p_node */
    double* q = (double*)malloc(sizeof(double) * C * N * 4);
    double* G = (double*)calloc((size_t)C * B * 16, sizeof(double));
    double dps[16] = {0}, dfr[4] = {0};
#pragma omp for schedule(static)
    for (int i = 0; i < P; ++i) {
      /* forward: node loop outer, category inner (:999-1005) */
      for (int t = 0; t < S; ++t)
        for (int c = 0; c < C; ++c) tipv(tipcodes[(size_t)t * P + i], &part[((size_t)c * N + t) * 4]);
      for (int n = 0; n < S - 1; ++n) {
        const int x = peel[3 * n], y = peel[3 * n + 1], v = peel[3 * n + 2];
        for (int c = 0; c < C; ++c) {
          double* ax = &moved[((size_t)c * N + x) * 4];
          double* ay = &moved[((size_t)c * N + y) * 4];
          mv(&pm[((size_t)c * B + x) * 16], &part[((size_t)c * N + x) * 4], ax);
          if (y == merged)
            memcpy(ay, &part[((size_t)c * N + y) * 4], sizeof(double) * 4);
          else
            mv(&pm[((size_t)c * B + y) * 16], &part[((size_t)c * N + y) * 4], ay);
          for (int k = 0; k < 4; ++k) part[((size_t)c * N + v) * 4 + k] = ax[k] * ay[k];
        }
      }
      /* root (:1006-1010) */
      double L = 0.0, fp[16];
      for (int c = 0; c < C; ++c) {
        const double* pr = &part[((size_t)c * N + root) * 4];
        fp[c] = pr[0] * f[0] + pr[1] * f[1] + pr[2] * f[2] + pr[3] * f[3];
        L += ps[c] * fp[c];
      }
      const double lnL = log(L);
      if (site_ll) site_ll[i] = lnL;
      ll_tot += w[i] * lnL;
      const double sc = w[i] / L;
      for (int c = 0; c < C; ++c) {
        const double* pr = &part[((size_t)c * N + root) * 4];
        dps[c] += sc * fp[c];
        for (int k = 0; k < 4; ++k) dfr[k] += sc * ps[c] * pr[k];
      }
      /* reverse: pre-order upper partials */
      for (int c = 0; c < C; ++c) memcpy(&q[((size_t)c * N + root) * 4], f, sizeof(double) * 4);
      for (int n = S - 2; n >= 0; --n) {
        const int x = peel[3 * n], y = peel[3 * n + 1], v = peel[3 * n + 2];
        for (int c = 0; c < C; ++c) {
          const double s = sc * ps[c];
          const double* qv = &q[((size_t)c * N + v) * 4];
          const double* ax = &moved[((size_t)c * N + x) * 4];
          const double* ay = &moved[((size_t)c * N + y) * 4];
          double rx[4], ry[4];
          for (int k = 0; k < 4; ++k) {
            rx[k] = qv[k] * ay[k];
            ry[k] = qv[k] * ax[k];
          }
          const double* px = &part[((size_t)c * N + x) * 4];
          const double* py = &part[((size_t)c * N + y) * 4];
          double* gx = &G[((size_t)c * B + x) * 16];
          for (int j = 0; j < 4; ++j)
            for (int k = 0; k < 4; ++k) gx[j * 4 + k] += s * rx[j] * px[k];
          mtv(&pm[((size_t)c * B + x) * 16], rx, &q[((size_t)c * N + x) * 4]);
          if (y == merged) {
            memcpy(&q[((size_t)c * N + y) * 4], ry, sizeof(double) * 4);
          } else {
            double* gy = &G[((size_t)c * B + y) * 16];
            for (int j = 0; j < 4; ++j)
              for (int k = 0; k < 4; ++k) gy[j * 4 + k] += s * ry[j] * py[k];
            mtv(&pm[((size_t)c * B + y) * 16], ry, &q[((size_t)c * N + y) * 4]);
          }
        }
      }
    }
#pragma omp critical
    {
      for (size_t k = 0; k < (size_t)C * B * 16; ++k) out[og + k] += G[k];
      for (int c = 0; c < C; ++c) out[1 + B + C + c] += dps[c];
      for (int k = 0; k < 4; ++k) out[1 + B + 2 * C + k] += dfr[k];
    }
    free(part);
    free(moved);
    free(q);
    free(G);
  }
  out[0] = isfinite(ll_tot) ? ll_tot : -INFINITY;
  /* chain rule dP/dt = Q P  ->  blens and rates */
  for (int b = 0; b < B; ++b) {
    double s = 0.0;
    for (int c = 0; c < C; ++c) {
      double in = 0.0;
      for (int k = 0; k < 16; ++k) in += out[og + ((size_t)c * B + b) * 16 + k] * qp[((size_t)c * B + b) * 16 + k];
      s += rs[c] * in;
    }
    out[1 + b] = s;
  }
  for (int c = 0; c < C; ++c) {
    double s = 0.0;
    for (int b = 0; b < B; ++b) {
      double in = 0.0;
      for (int k = 0; k < 16; ++k) in += out[og + ((size_t)c * B + b) * 16 + k] * qp[((size_t)c * B + b) * 16 + k];
      s += blens[b] * in;
    }
    out[1 + B + c] = s;
  }
  free(pm);
  free(qp);
  return 0;
}
