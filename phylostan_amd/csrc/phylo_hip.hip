// phylo_hip.hip -- MI355X (gfx950) Felsenstein-pruning likelihood + gradient.
//
// Replaces the likelihood hot path of phylostan:
//   * P-matrices       generate_script.py:755-892  (JC69 closed form; HKY/GTR
//                      via the symmetric eigendecomposition, here on device)
//   * post-order sweep generate_script.py:984-1040 (all four variants)
//   * root / site log  generate_script.py:991-995, :1006-1010, :1022, :1035
//   * reverse pass     Stan reverse-mode autodiff of the above; algorithm of
//                      the reference prototypes pruner/tree.cpp:228-242 and
//                      eigen/eigen.j2:143-167 (pre-order upper partials).
//
// Design (DESIGN.md has the long form):
//   One lane = one (pattern, category) column, one wave = 64 patterns of ONE
//   category (so every P-matrix a wave touches is wave-uniform and is read
//   with scalar loads), one workgroup = the C category-waves of a 64-pattern
//   block (so the per-site mixture sum sum_c ps_c pi.p_root,c is an LDS
//   exchange, not a global one).  Workgroups are persistent over pattern
//   blocks.  Per block:
//     forward  -- walks a host-built post-order program whose child order
//                 minimises the stack (Strahler order); pending partials live
//                 on a per-lane LDS stack; every non-root internal partial is
//                 also written once to a per-workgroup scratch region
//                 (fp64, 16 B per lane per store, coalesced);
//     root     -- mixture sum through LDS, site log-likelihood, w/L scale;
//     reverse  -- walks the program backwards carrying the pre-order upper
//                 partial q on the LDS stack; reads each stored partial
//                 exactly once; accumulates dlogL/dP per (branch, category)
//                 by a 64-lane transpose-reduce into LDS or a workgroup-
//                 private global slot.
//   A finalize kernel sums the per-workgroup slots in a fixed order
//   (bitwise deterministic) and applies dP/dt = Q P for the branch-length
//   and rate gradients.
//
// fp64 throughout, no rescaling -- exactly as the reference
// (generate_script.py:995, :1010); parity target 1e-6 relative per site.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "phylo_hip.h"

namespace {

constexpr int WAVE = 64;
constexpr int STEP_INTS = 8;  // x, y, bx, by, vslot, pad...

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return fail(PHY_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));          \
  } while (0)

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
struct V4 {
  double x, y, z, w;
};

__device__ __forceinline__ V4 vmul(const V4& a, const V4& b) {
  return {a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w};
}
__device__ __forceinline__ V4 vscale(const V4& a, double s) {
  return {a.x * s, a.y * s, a.z * s, a.w * s};
}
__device__ __forceinline__ double vdot(const V4& a, const V4& b) {
  return fma(a.w, b.w, fma(a.z, b.z, fma(a.y, b.y, a.x * b.x)));
}

// 16 doubles of a wave-uniform matrix (row-major P[j][k]).  The address is
// built from SGPR values only, so these become scalar (s_load) loads.
struct M16 {
  double m[16];
};
__device__ __forceinline__ M16 load_m(const double* __restrict__ p) {
  M16 r;
#pragma unroll
  for (int k = 0; k < 16; ++k) r.m[k] = p[k];
  return r;
}
// P v, summed over k in order (Eigen's unrolled 4x4 product order)
__device__ __forceinline__ V4 matvec(const M16& M, const V4& v) {
  V4 r;
  r.x = fma(M.m[3], v.w, fma(M.m[2], v.z, fma(M.m[1], v.y, M.m[0] * v.x)));
  r.y = fma(M.m[7], v.w, fma(M.m[6], v.z, fma(M.m[5], v.y, M.m[4] * v.x)));
  r.z = fma(M.m[11], v.w, fma(M.m[10], v.z, fma(M.m[9], v.y, M.m[8] * v.x)));
  r.w = fma(M.m[15], v.w, fma(M.m[14], v.z, fma(M.m[13], v.y, M.m[12] * v.x)));
  return r;
}
// P^T v
__device__ __forceinline__ V4 matTvec(const M16& M, const V4& v) {
  V4 r;
  r.x = fma(M.m[12], v.w, fma(M.m[8], v.z, fma(M.m[4], v.y, M.m[0] * v.x)));
  r.y = fma(M.m[13], v.w, fma(M.m[9], v.z, fma(M.m[5], v.y, M.m[1] * v.x)));
  r.z = fma(M.m[14], v.w, fma(M.m[10], v.z, fma(M.m[6], v.y, M.m[2] * v.x)));
  r.w = fma(M.m[15], v.w, fma(M.m[11], v.z, fma(M.m[7], v.y, M.m[3] * v.x)));
  return r;
}

__device__ __forceinline__ V4 tipvec(unsigned code) {
  return {(double)(code & 1u), (double)((code >> 1) & 1u), (double)((code >> 2) & 1u),
          (double)((code >> 3) & 1u)};
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, WAVE);
  return v;
}

// Transpose-reduce of 16 per-lane values over the 64 lanes of a wave.  Each
// step halves the values a lane carries and exchanges the other half with
// its partner, so 16 sums cost 17 shuffles instead of 96.  On return lane l
// holds the full sum of entry e(l) = 8*b5 + 4*b4 + 2*b3 + b2 (bits of l),
// replicated over l&3.  The summation tree is fixed: deterministic.
__device__ __forceinline__ double reduce16(double (&v)[16], int lane) {
  {
    const bool hi = lane & 32;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const double send = hi ? v[k] : v[k + 8];
      const double keep = hi ? v[k + 8] : v[k];
      v[k] = keep + __shfl_xor(send, 32, WAVE);
    }
  }
  {
    const bool hi = lane & 16;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double send = hi ? v[k] : v[k + 4];
      const double keep = hi ? v[k + 4] : v[k];
      v[k] = keep + __shfl_xor(send, 16, WAVE);
    }
  }
  {
    const bool hi = lane & 8;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const double send = hi ? v[k] : v[k + 2];
      const double keep = hi ? v[k + 2] : v[k];
      v[k] = keep + __shfl_xor(send, 8, WAVE);
    }
  }
  {
    const bool hi = lane & 4;
    const double send = hi ? v[0] : v[1];
    const double keep = hi ? v[1] : v[0];
    v[0] = keep + __shfl_xor(send, 4, WAVE);
  }
  double s = v[0];
  s += __shfl_xor(s, 2, WAVE);
  s += __shfl_xor(s, 1, WAVE);
  return s;
}

__device__ __forceinline__ int reduce16_entry(int lane) {
  return ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
}

// ---------------------------------------------------------------------------
// kernel arguments
// ---------------------------------------------------------------------------
struct SweepArgs {
  const uint8_t* tips;    // [S][Ppad] state masks
  const double* weights;  // [Ppad]   (0 on padding)
  const int* prog;        // [nsteps][STEP_INTS]
  const double* pm;       // [draw][C][B][16]
  const double* model;    // [draw][10+2C]
  double2* scratch;       // [wg][nslots][2][C*64]
  double* gslot;          // [wg][C][B][16]
  double* sslot;          // [wg][C][8]
  double* site_ll;        // [draw][P] or null
  int S, P, Ppad, C, B, nsteps, nslots, nblk, depth;
};

// LDS carve (all offsets multiples of 16 B):
//   stacks  C * depth * 2 * 64 double2
//   tips    S * 64 bytes (rounded to 16)
//   rootL   C * 64 double
//   G       C * B * 16 double            (GLDS only)
__host__ __device__ inline size_t lds_bytes(int S, int C, int B, int depth, bool glds) {
  size_t b = (size_t)C * depth * 2 * WAVE * 16;
  b += ((size_t)S * WAVE + 15) / 16 * 16;
  b += (size_t)C * WAVE * 8;
  if (glds) b += (size_t)C * B * 16 * 8;
  return b;
}

template <bool GLDS, int MAXT>
__global__ void __launch_bounds__(MAXT) sweep_kernel(SweepArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  const int lane = threadIdx.x & (WAVE - 1);
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nthreads = blockDim.x;
  const int draw = blockIdx.y;
  const int wg = blockIdx.y * gridDim.x + blockIdx.x;
  const int C = a.C, B = a.B;
  const int ncolwg = C * WAVE;

  double2* stk = reinterpret_cast<double2*>(lds_raw) + (size_t)c * a.depth * 2 * WAVE;
  unsigned char* tipl = lds_raw + (size_t)C * a.depth * 2 * WAVE * 16;
  double* rootL = reinterpret_cast<double*>(tipl + ((size_t)a.S * WAVE + 15) / 16 * 16);
  double* gl = rootL + (size_t)C * WAVE;  // GLDS: [C][B][16]

  const double* mdl = a.model + (size_t)draw * (10 + 2 * C);
  const V4 pi = {mdl[0], mdl[1], mdl[2], mdl[3]};
  const double ps_c = mdl[10 + C + c];
  const double* pmc = a.pm + ((size_t)draw * C + c) * B * 16;
  double2* scr = a.scratch + (size_t)wg * a.nslots * 2 * ncolwg;
  double* gslot_c = a.gslot + ((size_t)wg * C + c) * B * 16;

  const int e = reduce16_entry(lane);
  const bool gowner = (lane & 3) == 0;
  if (GLDS) {
    for (int k = threadIdx.x; k < C * B * 16; k += nthreads) gl[k] = 0.0;
  } else if (gowner) {
    for (int b = 0; b < B; ++b) gslot_c[b * 16 + e] = 0.0;
  }

  double acc_ll = 0.0, acc_dps = 0.0;
  V4 acc_f = {0.0, 0.0, 0.0, 0.0};

  auto push = [&](int& sp, const V4& v) {
    stk[(sp * 2 + 0) * WAVE + lane] = make_double2(v.x, v.y);
    stk[(sp * 2 + 1) * WAVE + lane] = make_double2(v.z, v.w);
    ++sp;
  };
  auto pop = [&](int& sp) -> V4 {
    --sp;
    const double2 lo = stk[(sp * 2 + 0) * WAVE + lane];
    const double2 hi = stk[(sp * 2 + 1) * WAVE + lane];
    return {lo.x, lo.y, hi.x, hi.y};
  };
  auto gacc = [&](int b, const V4& r, const V4& p) {
    double v[16] = {r.x * p.x, r.x * p.y, r.x * p.z, r.x * p.w, r.y * p.x, r.y * p.y,
                    r.y * p.z, r.y * p.w, r.z * p.x, r.z * p.y, r.z * p.z, r.z * p.w,
                    r.w * p.x, r.w * p.y, r.w * p.z, r.w * p.w};
    const double s = reduce16(v, lane);
    if (gowner) {
      if (GLDS)
        gl[((size_t)c * B + b) * 16 + e] += s;
      else
        gslot_c[b * 16 + e] += s;
    }
  };

  for (int blk = blockIdx.x; blk < a.nblk; blk += gridDim.x) {
    const int i = blk * WAVE + lane;  // pattern of this lane
    // stage this block's tip codes in LDS: S rows x 64 bytes, shared by the
    // C category-waves and by both passes
    {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(a.tips);
      uint32_t* dst = reinterpret_cast<uint32_t*>(tipl);
      const int rowq = a.Ppad / 4;
      for (int k = threadIdx.x; k < a.S * (WAVE / 4); k += nthreads) {
        const int t = k >> 4, q = k & 15;
        dst[k] = src[(size_t)t * rowq + blk * (WAVE / 4) + q];
      }
    }
    __syncthreads();

    // ------------------------------ forward ------------------------------
    int sp = 0;
    V4 proot = {0, 0, 0, 0};
    for (int s = 0; s < a.nsteps; ++s) {
      const int* st = a.prog + s * STEP_INTS;
      const int x = st[0], y = st[1], bx = st[2], by = st[3], vs = st[4];
      V4 ay, ax;
      if (y >= 0) {
        ay = tipvec(tipl[y * WAVE + lane]);
      } else {
        ay = pop(sp);
      }
      if (by >= 0) ay = matvec(load_m(pmc + (size_t)by * 16), ay);
      if (x >= 0) {
        ax = tipvec(tipl[x * WAVE + lane]);
      } else {
        ax = pop(sp);
      }
      if (bx >= 0) ax = matvec(load_m(pmc + (size_t)bx * 16), ax);
      const V4 pv = vmul(ax, ay);
      if (vs >= 0) {
        double2* dst = scr + (size_t)vs * 2 * ncolwg + c * WAVE + lane;
        dst[0] = make_double2(pv.x, pv.y);
        dst[ncolwg] = make_double2(pv.z, pv.w);
        push(sp, pv);
      } else {
        proot = pv;
      }
    }

    // ------------------------- root / site log L -------------------------
    const double fp = vdot(pi, proot);  // pi . p_root,c
    rootL[c * WAVE + lane] = ps_c * fp;
    __syncthreads();
    double L = 0.0;
    for (int k = 0; k < C; ++k) L += rootL[k * WAVE + lane];
    __syncthreads();
    const double w = a.weights[i];
    const double lnL = log(L);
    if (c == 0) {
      acc_ll += w * lnL;
      if (a.site_ll != nullptr && i < a.P) a.site_ll[(size_t)draw * a.P + i] = lnL;
    }
    const double sc = w / L;
    const double s_c = sc * ps_c;
    acc_dps = fma(sc, fp, acc_dps);
    acc_f.x = fma(s_c, proot.x, acc_f.x);
    acc_f.y = fma(s_c, proot.y, acc_f.y);
    acc_f.z = fma(s_c, proot.z, acc_f.z);
    acc_f.w = fma(s_c, proot.w, acc_f.w);

    // ------------------------------ reverse ------------------------------
    sp = 0;
    for (int s = a.nsteps - 1; s >= 0; --s) {
      const int* st = a.prog + s * STEP_INTS;
      const int x = st[0], y = st[1], bx = st[2], by = st[3];
      const V4 qv = (s == a.nsteps - 1) ? pi : pop(sp);
      V4 px, py;
      if (x >= 0) {
        px = tipvec(tipl[x * WAVE + lane]);
      } else {
        const double2* src = scr + (size_t)(-x - 1) * 2 * ncolwg + c * WAVE + lane;
        const double2 lo = src[0], hi = src[ncolwg];
        px = {lo.x, lo.y, hi.x, hi.y};
      }
      if (y >= 0) {
        py = tipvec(tipl[y * WAVE + lane]);
      } else {
        const double2* src = scr + (size_t)(-y - 1) * 2 * ncolwg + c * WAVE + lane;
        const double2 lo = src[0], hi = src[ncolwg];
        py = {lo.x, lo.y, hi.x, hi.y};
      }
      // Matrices are re-read (scalar loads, K$ hits) rather than kept live
      // across the step: two live 4x4 fp64 matrices cost 64 SGPRs.
      const V4 ax = (bx >= 0) ? matvec(load_m(pmc + (size_t)bx * 16), px) : px;
      const V4 ay = (by >= 0) ? matvec(load_m(pmc + (size_t)by * 16), py) : py;
      const V4 rx = vmul(qv, ay);
      const V4 ry = vmul(qv, ax);
      if (bx >= 0) gacc(bx, vscale(rx, s_c), px);
      if (x < 0) push(sp, bx >= 0 ? matTvec(load_m(pmc + (size_t)bx * 16), rx) : rx);
      if (by >= 0) gacc(by, vscale(ry, s_c), py);
      if (y < 0) push(sp, by >= 0 ? matTvec(load_m(pmc + (size_t)by * 16), ry) : ry);
    }
    __syncthreads();  // tips / rootL are rewritten by the next block
  }

  // per-workgroup scalar partials: [ll, dps, dfreq0..3]
  acc_ll = wave_sum(acc_ll);
  acc_dps = wave_sum(acc_dps);
  acc_f.x = wave_sum(acc_f.x);
  acc_f.y = wave_sum(acc_f.y);
  acc_f.z = wave_sum(acc_f.z);
  acc_f.w = wave_sum(acc_f.w);
  if (lane == 0) {
    double* ss = a.sslot + ((size_t)wg * C + c) * 8;
    ss[0] = acc_ll;
    ss[1] = acc_dps;
    ss[2] = acc_f.x;
    ss[3] = acc_f.y;
    ss[4] = acc_f.z;
    ss[5] = acc_f.w;
  }
  if (GLDS) {
    __syncthreads();
    double* dst = a.gslot + (size_t)wg * C * B * 16;
    for (int k = threadIdx.x; k < C * B * 16; k += nthreads) dst[k] = gl[k];
  }
}

// ---------------------------------------------------------------------------
// P-matrices (generate_script.py:755-892), one workgroup per draw
// ---------------------------------------------------------------------------
struct PmatArgs {
  const double* model;  // [draw][10+2C]
  const double* blens;  // [draw][B]
  double* pm;           // [draw][C][B][16]
  double* qp;           // [draw][C][B][16]  Q P  (= dP/dt)
  int C, B, kind;
};

// Cyclic Jacobi eigendecomposition of a symmetric 4x4 (A overwritten).
__device__ void jacobi4(double A[4][4], double V[4][4], double lam[4]) {
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
    for (int p = 0; p < 3; ++p)
      for (int q = p + 1; q < 4; ++q) {
        const double apq = A[p][q];
        if (apq == 0.0) continue;
        const double theta = (A[q][q] - A[p][p]) / (2.0 * apq);
        const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double cs = 1.0 / sqrt(t * t + 1.0);
        const double sn = t * cs;
        for (int k = 0; k < 4; ++k) {  // A <- A R   (columns p, q)
          const double akp = A[k][p], akq = A[k][q];
          A[k][p] = cs * akp - sn * akq;
          A[k][q] = sn * akp + cs * akq;
        }
        for (int k = 0; k < 4; ++k) {  // A <- R^T A (rows p, q)
          const double apk = A[p][k], aqk = A[q][k];
          A[p][k] = cs * apk - sn * aqk;
          A[q][k] = sn * apk + cs * aqk;
        }
        A[p][q] = A[q][p] = 0.0;
        for (int k = 0; k < 4; ++k) {  // V <- V R
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = cs * vkp - sn * vkq;
          V[k][q] = sn * vkp + cs * vkq;
        }
      }
  }
  for (int i = 0; i < 4; ++i) lam[i] = A[i][i];
}

__global__ void __launch_bounds__(256) pmat_kernel(PmatArgs a) {
  __shared__ double m1[16], m2[16], lam[4], Q[16];
  const int draw = blockIdx.x;
  const int C = a.C, B = a.B;
  const double* mdl = a.model + (size_t)draw * (10 + 2 * C);
  const double* rs = mdl + 10;
  const double* bl = a.blens + (size_t)draw * B;
  if (threadIdx.x == 0) {
    if (a.kind == PHY_JC69) {
      for (int j = 0; j < 4; ++j)
        for (int k = 0; k < 4; ++k) Q[j * 4 + k] = (j == k) ? -1.0 : 1.0 / 3.0;
    } else {
      const double* f = mdl;
      const double* r = mdl + 4;  // AC AG AT CG CT GT  (generate_script.py:855-858)
      double R[4][4] = {{0.0, r[0], r[1], r[2]},
                        {r[0], 0.0, r[3], r[4]},
                        {r[1], r[3], 0.0, r[5]},
                        {r[2], r[4], r[5], 0.0}};
      double q[4][4];
      double s = 0.0;
      for (int j = 0; j < 4; ++j) {  // Q = R diag(pi), zero-sum rows (:862-867)
        double row = 0.0;
        for (int k = 0; k < 4; ++k) {
          q[j][k] = (j == k) ? 0.0 : R[j][k] * f[k];
          row += q[j][k];
        }
        q[j][j] = -row;
        s -= q[j][j] * f[j];
      }
      double A[4][4], V[4][4], l[4], sq[4];
      for (int j = 0; j < 4; ++j) sq[j] = sqrt(f[j]);
      for (int j = 0; j < 4; ++j)
        for (int k = 0; k < 4; ++k) {
          q[j][k] /= s;  // :868
          Q[j * 4 + k] = q[j][k];
        }
      for (int j = 0; j < 4; ++j)  // A = Pi^1/2 Q Pi^-1/2, symmetrised (:870)
        for (int k = 0; k < 4; ++k)
          A[j][k] = (j == k) ? q[j][j] : 0.5 * (sq[j] * q[j][k] / sq[k] + sq[k] * q[k][j] / sq[j]);
      jacobi4(A, V, l);
      for (int j = 0; j < 4; ++j) {
        lam[j] = l[j];
        for (int k = 0; k < 4; ++k) {
          m1[j * 4 + k] = V[j][k] / sq[j];  // Pi^-1/2 V      (:875)
          m2[j * 4 + k] = V[k][j] * sq[k];  // V^T Pi^1/2     (:876)
        }
      }
    }
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < C * B; idx += blockDim.x) {
    const int c = idx / B, b = idx - c * B;
    const double t = bl[b] * rs[c];
    double P[16];
    if (a.kind == PHY_JC69) {  // generate_script.py:765-769
      const double ex = exp(-t / 0.75);
      const double off = 0.25 - 0.25 * ex, d = 0.25 + 0.75 * ex;
      for (int k = 0; k < 16; ++k) P[k] = (k % 5 == 0) ? d : off;
    } else {  // m1 diag(exp(lam t)) m2   (:880)
      double E[4];
      for (int l = 0; l < 4; ++l) E[l] = exp(lam[l] * t);
      for (int j = 0; j < 4; ++j)
        for (int k = 0; k < 4; ++k) {
          double acc = 0.0;
          for (int l = 0; l < 4; ++l) acc = fma(m1[j * 4 + l] * E[l], m2[l * 4 + k], acc);
          P[j * 4 + k] = acc;
        }
    }
    double* po = a.pm + (((size_t)draw * C + c) * B + b) * 16;
    double* qo = a.qp + (((size_t)draw * C + c) * B + b) * 16;
    for (int k = 0; k < 16; ++k) po[k] = P[k];
    for (int j = 0; j < 4; ++j)
      for (int k = 0; k < 4; ++k) {
        double acc = 0.0;
        for (int l = 0; l < 4; ++l) acc = fma(Q[j * 4 + l], P[l * 4 + k], acc);
        qo[j * 4 + k] = acc;
      }
  }
}

// ---------------------------------------------------------------------------
// finalize: fixed-order sums of the per-workgroup slots + chain rule dP/dt
// ---------------------------------------------------------------------------
struct FinArgs {
  const double* gslot;  // [wg][C][B][16]
  const double* sslot;  // [wg][C][8]
  const double* qp;     // [draw][C][B][16]
  const double* blens;  // [draw][B]
  const double* model;  // [draw][10+2C]
  double* out;          // [draw][outlen]
  int C, B, gx, outlen;
};

__global__ void __launch_bounds__(256) finalize_kernel(FinArgs a) {
  extern __shared__ double inner[];  // [C][B]
  const int draw = blockIdx.x;
  const int C = a.C, B = a.B;
  double* out = a.out + (size_t)draw * a.outlen;
  const size_t wg0 = (size_t)draw * a.gx;
  const int og = 1 + B + 2 * C + 4;
  const int ng = C * B * 16;
  for (int idx = threadIdx.x; idx < ng; idx += blockDim.x) {
    double s = 0.0;
    for (int w = 0; w < a.gx; ++w) s += a.gslot[(wg0 + w) * ng + idx];
    out[og + idx] = s;
  }
  if (threadIdx.x == 0) {
    double ll = 0.0;
    for (int w = 0; w < a.gx; ++w) ll += a.sslot[((wg0 + w) * C + 0) * 8 + 0];
    out[0] = isfinite(ll) ? ll : -INFINITY;
  }
  if (threadIdx.x < C) {
    const int c = threadIdx.x;
    double d = 0.0;
    for (int w = 0; w < a.gx; ++w) d += a.sslot[((wg0 + w) * C + c) * 8 + 1];
    out[1 + B + C + c] = d;
  }
  if (threadIdx.x >= 64 && threadIdx.x < 68) {
    const int j = threadIdx.x - 64;
    double d = 0.0;
    for (int w = 0; w < a.gx; ++w)
      for (int c = 0; c < C; ++c) d += a.sslot[((wg0 + w) * C + c) * 8 + 2 + j];
    out[1 + B + 2 * C + j] = d;
  }
  __syncthreads();
  const double* qp = a.qp + (size_t)draw * C * B * 16;
  for (int idx = threadIdx.x; idx < C * B; idx += blockDim.x) {
    double s = 0.0;
    for (int k = 0; k < 16; ++k) s = fma(out[og + (size_t)idx * 16 + k], qp[(size_t)idx * 16 + k], s);
    inner[idx] = s;  // dlogL / dt_{b,c}
  }
  __syncthreads();
  const double* rs = a.model + (size_t)draw * (10 + 2 * C) + 10;
  const double* bl = a.blens + (size_t)draw * B;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    double s = 0.0;
    for (int c = 0; c < C; ++c) s = fma(rs[c], inner[c * B + b], s);
    out[1 + b] = s;
  }
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double s = 0.0;
    for (int b = 0; b < B; ++b) s = fma(bl[b], inner[c * B + b], s);
    out[1 + B + c] = s;
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct phy_ctx {
  int S, P, Ppad, C, B, rooted, kind, max_draws, device;
  int nsteps, nslots, depth, nblk;
  int wg_budget, g_mode, wg_cap;
  hipStream_t stream;
  uint8_t* d_tips = nullptr;
  double* d_w = nullptr;
  int* d_prog = nullptr;
  double* d_pm = nullptr;
  double* d_qp = nullptr;
  double* d_model = nullptr;
  double* d_blens = nullptr;
  double* d_out = nullptr;
  double* d_site = nullptr;
  double2* d_scratch = nullptr;
  double* d_gslot = nullptr;
  double* d_sslot = nullptr;
  bool timing = false;
  std::vector<hipEvent_t> ev;  // pairs
  int ev_used = 0;
  double timed_ms = 0.0;
  int timed_n = 0;
  int max_lds = 65536;
};

namespace {

void free_ctx(phy_ctx* c) {
  if (!c) return;
  int dev_old = 0;
  (void)hipGetDevice(&dev_old);
  (void)hipSetDevice(c->device);
  void* ptrs[] = {c->d_tips, c->d_w, c->d_prog, c->d_pm, c->d_qp, c->d_model, c->d_blens,
                  c->d_out, c->d_site, c->d_scratch, c->d_gslot, c->d_sslot};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  (void)hipSetDevice(dev_old);
  delete c;
}

// Build the traversal program (see DESIGN.md "Traversal program").
int build_program(int S, const int32_t* peel, int rooted, std::vector<int>& prog, int& nslots,
                  int& depth) {
  const int N = 2 * S - 1;
  std::vector<int> ch1(N, -1), ch2(N, -1);
  std::vector<int> seen(N, 0);
  for (int r = 0; r < S - 1; ++r) {
    const int a = peel[3 * r], b = peel[3 * r + 1], v = peel[3 * r + 2];
    if (a < 0 || a >= N || b < 0 || b >= N || v < S || v >= N || a == b)
      return fail(PHY_EINVAL, "peel row " + std::to_string(r) + " out of range");
    if (ch1[v] != -1) return fail(PHY_EINVAL, "node " + std::to_string(v) + " peeled twice");
    ch1[v] = a;
    ch2[v] = b;
    seen[a]++;
    seen[b]++;
  }
  const int root = peel[3 * (S - 2) + 2];
  for (int n = 0; n < N; ++n) {
    if (n != root && seen[n] != 1)
      return fail(PHY_EINVAL, "node " + std::to_string(n) + " is not a child exactly once");
    if (n >= S && ch1[n] < 0) return fail(PHY_EINVAL, "internal node without children");
  }
  if (seen[root] != 0) return fail(PHY_EINVAL, "root listed as a child");
  int merged = -1;
  if (!rooted) {
    merged = peel[3 * (S - 2) + 1];
    if (merged != 2 * S - 3)
      return fail(PHY_EINVAL,
                  "unrooted peel: last row child2 must be node 2S-3 (phylostan.py:264-267)");
  }
  // stack need per subtree; larger-need child first (Strahler order)
  std::vector<int> need(N, 0), first(N, -1), second(N, -1);
  {
    std::vector<int> order;  // post-order of the rooted tree
    std::vector<std::pair<int, int>> st{{root, 0}};
    while (!st.empty()) {
      auto& [n, k] = st.back();
      if (n < S || k == 2) {
        order.push_back(n);
        st.pop_back();
        continue;
      }
      const int child = (k == 0) ? ch1[n] : ch2[n];
      ++k;
      st.push_back({child, 0});
    }
    for (int n : order) {
      if (n < S) continue;
      const int a = ch1[n], b = ch2[n];
      auto hold = [&](int m) { return m >= S ? 1 : 0; };
      const int ab = std::max({need[a], hold(a) + need[b], 1});
      const int ba = std::max({need[b], hold(b) + need[a], 1});
      if (ba < ab) {
        first[n] = b;
        second[n] = a;
        need[n] = ba;
      } else {
        first[n] = a;
        second[n] = b;
        need[n] = ab;
      }
    }
  }
  // emit post-order with the chosen child order
  std::vector<int> steps;
  {
    std::vector<std::pair<int, int>> st{{root, 0}};
    while (!st.empty()) {
      auto& [n, k] = st.back();
      if (n < S) {
        st.pop_back();
        continue;
      }
      if (k == 2) {
        steps.push_back(n);
        st.pop_back();
        continue;
      }
      const int child = (k == 0) ? first[n] : second[n];
      ++k;
      st.push_back({child, 0});
    }
  }
  if ((int)steps.size() != S - 1) return fail(PHY_EINVAL, "tree is not binary / connected");
  std::vector<int> slot(N, -1);
  for (int s = 0; s < S - 1; ++s)
    if (steps[s] != root) slot[steps[s]] = s;
  nslots = S - 2;
  prog.assign((size_t)(S - 1) * STEP_INTS, 0);
  for (int s = 0; s < S - 1; ++s) {
    const int v = steps[s];
    const int x = first[v], y = second[v];
    int* p = &prog[(size_t)s * STEP_INTS];
    p[0] = x < S ? x : -(slot[x] + 1);
    p[1] = y < S ? y : -(slot[y] + 1);
    p[2] = (x == merged) ? -1 : x;
    p[3] = (y == merged) ? -1 : y;
    p[4] = (v == root) ? -1 : slot[v];
    p[5] = v;
  }
  // simulate both passes to size the LDS stack exactly
  int sp = 0, mx = 0;
  for (int s = 0; s < S - 1; ++s) {
    const int* p = &prog[(size_t)s * STEP_INTS];
    if (p[1] < 0) --sp;
    if (p[0] < 0) --sp;
    if (sp < 0) return fail(PHY_EINVAL, "internal: forward stack underflow");
    if (p[4] >= 0) mx = std::max(mx, ++sp);
  }
  if (sp != 0) return fail(PHY_EINVAL, "internal: forward stack not empty");
  for (int s = S - 2; s >= 0; --s) {
    const int* p = &prog[(size_t)s * STEP_INTS];
    if (s != S - 2) --sp;
    if (sp < 0) return fail(PHY_EINVAL, "internal: reverse stack underflow");
    if (p[0] < 0) mx = std::max(mx, ++sp);
    if (p[1] < 0) mx = std::max(mx, ++sp);
  }
  if (sp != 0) return fail(PHY_EINVAL, "internal: reverse stack not empty");
  depth = std::max(mx, 1);
  return PHY_OK;
}

template <typename T>
int dalloc(T** p, size_t n) {
  if (n == 0) n = 1;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T));
  if (e != hipSuccess)
    return fail(PHY_ENOMEM, std::string("hipMalloc ") + std::to_string(n * sizeof(T)) + " B: " +
                                hipGetErrorString(e));
  return PHY_OK;
}

bool use_glds(const phy_ctx* c) {
  if (c->g_mode == 1) return true;
  if (c->g_mode == 2) return false;
  return lds_bytes(c->S, c->C, c->B, c->depth, true) <= (size_t)c->max_lds;
}

int launch(phy_ctx* ctx, int n, const double* d_blens, const double* d_model, double* d_out,
           double* d_site, hipStream_t st) {
  const int C = ctx->C, B = ctx->B;
  {
    PmatArgs pa{d_model, d_blens, ctx->d_pm, ctx->d_qp, C, B, ctx->kind};
    hipLaunchKernelGGL(pmat_kernel, dim3(n), dim3(256), 0, st, pa);
    HIP_TRY(hipGetLastError());
  }
  const int gx = std::max(1, std::min(ctx->nblk, (ctx->wg_budget + n - 1) / n));
  if ((size_t)gx * n > (size_t)ctx->wg_cap) return fail(PHY_ERANGE, "workgroup cap exceeded");
  const bool glds = use_glds(ctx);
  const size_t lds = lds_bytes(ctx->S, C, B, ctx->depth, glds);
  SweepArgs sa{ctx->d_tips, ctx->d_w,       ctx->d_prog, ctx->d_pm,     d_model,
               ctx->d_scratch, ctx->d_gslot, ctx->d_sslot, d_site,       ctx->S,
               ctx->P,       ctx->Ppad,    C,           B,             ctx->nsteps,
               ctx->nslots,  ctx->nblk,    ctx->depth};
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (ctx->timing) {
    if (ctx->ev_used + 2 > (int)ctx->ev.size()) {
      // pool full: fold what is recorded so far
      HIP_TRY(hipStreamSynchronize(st));
      for (int k = 0; k + 1 < ctx->ev_used; k += 2) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, ctx->ev[k], ctx->ev[k + 1]));
        ctx->timed_ms += ms;
        ctx->timed_n += 1;
      }
      ctx->ev_used = 0;
    }
    e0 = ctx->ev[ctx->ev_used];
    e1 = ctx->ev[ctx->ev_used + 1];
    ctx->ev_used += 2;
    HIP_TRY(hipEventRecord(e0, st));
  }
  const int threads = C * WAVE;
  if (threads <= 256) {
    if (glds)
      hipLaunchKernelGGL((sweep_kernel<true, 256>), dim3(gx, n), dim3(threads), lds, st, sa);
    else
      hipLaunchKernelGGL((sweep_kernel<false, 256>), dim3(gx, n), dim3(threads), lds, st, sa);
  } else {
    if (glds)
      hipLaunchKernelGGL((sweep_kernel<true, 1024>), dim3(gx, n), dim3(threads), lds, st, sa);
    else
      hipLaunchKernelGGL((sweep_kernel<false, 1024>), dim3(gx, n), dim3(threads), lds, st, sa);
  }
  HIP_TRY(hipGetLastError());
  if (ctx->timing) HIP_TRY(hipEventRecord(e1, st));
  FinArgs fa{ctx->d_gslot, ctx->d_sslot, ctx->d_qp, d_blens, d_model, d_out, C, B, gx,
             phy_output_len(ctx)};
  hipLaunchKernelGGL(finalize_kernel, dim3(n), dim3(256), (size_t)C * B * sizeof(double), st, fa);
  HIP_TRY(hipGetLastError());
  return PHY_OK;
}

}  // namespace

extern "C" {

const char* phy_last_error(void) { return g_err.c_str(); }

int phy_create(int S, int P, int C, int rooted, int model, const uint8_t* tipcodes,
               const double* weights, const int32_t* peel, int max_draws, int device,
               phy_ctx** out) {
  g_err.clear();
  if (!out) return fail(PHY_EINVAL, "out is NULL");
  *out = nullptr;
  if (S < 3) return fail(PHY_EINVAL, "need S >= 3 taxa");
  if (P < 1) return fail(PHY_EINVAL, "need P >= 1 patterns");
  if (C < 1 || C > 16) return fail(PHY_EINVAL, "C must be in 1..16");
  if (model < PHY_JC69 || model > PHY_GTR) return fail(PHY_EINVAL, "unknown model");
  if (max_draws < 1) return fail(PHY_EINVAL, "max_draws must be >= 1");
  if (!tipcodes || !weights || !peel) return fail(PHY_EINVAL, "NULL input array");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(PHY_EINVAL, "bad device ordinal");
  for (size_t k = 0; k < (size_t)S * P; ++k)
    if (tipcodes[k] > 15) return fail(PHY_EINVAL, "tip code > 15");

  phy_ctx* c = new phy_ctx();
  c->S = S;
  c->P = P;
  c->C = C;
  c->rooted = rooted ? 1 : 0;
  c->kind = model;
  c->max_draws = max_draws;
  c->device = device;
  c->B = rooted ? 2 * S - 2 : 2 * S - 3;
  c->nblk = (P + WAVE - 1) / WAVE;
  c->Ppad = c->nblk * WAVE;
  c->stream = nullptr;
  std::vector<int> prog;
  int rc = build_program(S, peel, c->rooted, prog, c->nslots, c->depth);
  if (rc) {
    delete c;
    return rc;
  }
  c->nsteps = S - 1;
  c->g_mode = 0;
  {
    const char* env = getenv("PHY_WG_BUDGET");
    c->wg_budget = env ? std::max(1, atoi(env)) : 512;
    const char* gm = getenv("PHY_G_MODE");
    if (gm) c->g_mode = atoi(gm);
  }
  c->wg_cap = std::min<long>((long)c->nblk * max_draws, (long)c->wg_budget + max_draws);
  hipError_t he = hipSetDevice(device);
  if (he != hipSuccess) {
    delete c;
    return fail(PHY_EHIP, std::string("hipSetDevice: ") + hipGetErrorString(he));
  }
  int lds_max = 0;
  (void)hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, device);
  c->max_lds = 65536;
  if (lds_bytes(S, C, c->B, c->depth, false) > (size_t)std::max(lds_max, 65536)) {
    delete c;
    return fail(PHY_EINVAL, "tree too deep for the LDS stack");
  }
#define TRY_C(expr)              \
  do {                           \
    int r_ = (expr);             \
    if (r_) {                    \
      std::string m_ = g_err;    \
      free_ctx(c);               \
      return fail(r_, m_);       \
    }                            \
  } while (0)
#define HIP_C(expr)                                                                  \
  do {                                                                               \
    hipError_t e_ = (expr);                                                          \
    if (e_ != hipSuccess) {                                                          \
      std::string m_ = std::string(#expr) + ": " + hipGetErrorString(e_);            \
      free_ctx(c);                                                                   \
      return fail(PHY_EHIP, m_);                                                     \
    }                                                                                \
  } while (0)
  HIP_C(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  const size_t ncolwg = (size_t)C * WAVE;
  TRY_C(dalloc(&c->d_tips, (size_t)S * c->Ppad));
  TRY_C(dalloc(&c->d_w, (size_t)c->Ppad));
  TRY_C(dalloc(&c->d_prog, prog.size()));
  TRY_C(dalloc(&c->d_pm, (size_t)max_draws * C * c->B * 16));
  TRY_C(dalloc(&c->d_qp, (size_t)max_draws * C * c->B * 16));
  TRY_C(dalloc(&c->d_model, (size_t)max_draws * (10 + 2 * C)));
  TRY_C(dalloc(&c->d_blens, (size_t)max_draws * c->B));
  TRY_C(dalloc(&c->d_out, (size_t)max_draws * phy_output_len(c)));
  TRY_C(dalloc(&c->d_site, (size_t)max_draws * P));
  TRY_C(dalloc(&c->d_scratch, (size_t)c->wg_cap * std::max(c->nslots, 1) * 2 * ncolwg));
  TRY_C(dalloc(&c->d_gslot, (size_t)c->wg_cap * C * c->B * 16));
  TRY_C(dalloc(&c->d_sslot, (size_t)c->wg_cap * C * 8));
  {
    std::vector<uint8_t> tips((size_t)S * c->Ppad, 15);
    for (int t = 0; t < S; ++t)
      std::memcpy(&tips[(size_t)t * c->Ppad], tipcodes + (size_t)t * P, P);
    std::vector<double> w(c->Ppad, 0.0);
    std::memcpy(w.data(), weights, sizeof(double) * P);
    HIP_C(hipMemcpy(c->d_tips, tips.data(), tips.size(), hipMemcpyHostToDevice));
    HIP_C(hipMemcpy(c->d_w, w.data(), w.size() * sizeof(double), hipMemcpyHostToDevice));
    HIP_C(hipMemcpy(c->d_prog, prog.data(), prog.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  *out = c;
  return PHY_OK;
}

int phy_destroy(phy_ctx* ctx) {
  free_ctx(ctx);
  return PHY_OK;
}

int phy_num_branches(const phy_ctx* ctx) { return ctx ? ctx->B : -1; }

int phy_output_len(const phy_ctx* ctx) {
  return ctx ? 1 + ctx->B + 2 * ctx->C + 4 + 16 * ctx->C * ctx->B : -1;
}

int phy_program_info(const phy_ctx* ctx, int* nsteps, int* nslots, int* depth, int* nblocks) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (nsteps) *nsteps = ctx->nsteps;
  if (nslots) *nslots = ctx->nslots;
  if (depth) *depth = ctx->depth;
  if (nblocks) *nblocks = ctx->nblk;
  return PHY_OK;
}

int phy_eval_device(phy_ctx* ctx, int n_draws, const double* d_blens, const double* d_model,
                    double* d_out, double* d_site_ll, void* stream) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (n_draws < 1 || n_draws > ctx->max_draws) return fail(PHY_ERANGE, "n_draws out of range");
  if (!d_blens || !d_model || !d_out) return fail(PHY_EINVAL, "NULL device buffer");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t st = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
  return launch(ctx, n_draws, d_blens, d_model, d_out, d_site_ll, st);
}

int phy_eval(phy_ctx* ctx, int n_draws, const double* blens, const double* model, double* out,
             double* site_ll) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (n_draws < 1 || n_draws > ctx->max_draws) return fail(PHY_ERANGE, "n_draws out of range");
  if (!blens || !model || !out) return fail(PHY_EINVAL, "NULL host buffer");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  const int ml = 10 + 2 * ctx->C;
  HIP_TRY(hipMemcpyAsync(ctx->d_blens, blens, sizeof(double) * n_draws * ctx->B,
                         hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(ctx->d_model, model, sizeof(double) * n_draws * ml,
                         hipMemcpyHostToDevice, st));
  int rc = launch(ctx, n_draws, ctx->d_blens, ctx->d_model, ctx->d_out,
                  site_ll ? ctx->d_site : nullptr, st);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out, ctx->d_out, sizeof(double) * n_draws * phy_output_len(ctx),
                         hipMemcpyDeviceToHost, st));
  if (site_ll)
    HIP_TRY(hipMemcpyAsync(site_ll, ctx->d_site, sizeof(double) * n_draws * ctx->P,
                           hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return PHY_OK;
}

double phy_pruning_loglik(phy_ctx* ctx, const double* blens, const double* model, double* grad) {
  if (!ctx) {
    fail(PHY_EINVAL, "NULL ctx");
    return NAN;
  }
  std::vector<double> out(phy_output_len(ctx));
  if (phy_eval(ctx, 1, blens, model, out.data(), nullptr) != PHY_OK) return NAN;
  if (grad) std::memcpy(grad, out.data() + 1, sizeof(double) * ctx->B);
  return out[0];
}

int phy_sync(phy_ctx* ctx) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return PHY_OK;
}

int phy_timing_start(phy_ctx* ctx) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  HIP_TRY(hipSetDevice(ctx->device));
  if (ctx->ev.empty()) {
    ctx->ev.resize(4096);
    for (auto& e : ctx->ev) HIP_TRY(hipEventCreate(&e));
  }
  ctx->timing = true;
  ctx->ev_used = 0;
  ctx->timed_ms = 0.0;
  ctx->timed_n = 0;
  return PHY_OK;
}

int phy_timing_read(phy_ctx* ctx, double* total_ms, int* launches) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  HIP_TRY(hipSetDevice(ctx->device));
  for (int k = 0; k + 1 < ctx->ev_used; k += 2) {
    HIP_TRY(hipEventSynchronize(ctx->ev[k + 1]));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, ctx->ev[k], ctx->ev[k + 1]));
    ctx->timed_ms += ms;
    ctx->timed_n += 1;
  }
  ctx->ev_used = 0;
  ctx->timing = false;
  if (total_ms) *total_ms = ctx->timed_ms;
  if (launches) *launches = ctx->timed_n;
  return PHY_OK;
}

int phy_set_tuning(phy_ctx* ctx, int wg_budget, int g_mode) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (wg_budget > 0) {
    const long need = std::min<long>((long)ctx->nblk * ctx->max_draws, (long)wg_budget + ctx->max_draws);
    if (need > ctx->wg_cap) return fail(PHY_ERANGE, "wg_budget larger than allocated at create");
    ctx->wg_budget = wg_budget;
  }
  if (g_mode < 0 || g_mode > 2) return fail(PHY_EINVAL, "g_mode must be 0, 1 or 2");
  ctx->g_mode = g_mode;
  return PHY_OK;
}

}  // extern "C"
