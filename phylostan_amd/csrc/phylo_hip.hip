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
//   category (every P-matrix a wave touches is wave-uniform: LDS broadcast
//   reads), one workgroup = the C category-waves of a 64-pattern block (the
//   per-site mixture sum sum_c ps_c pi.p_root,c is an LDS exchange).
//   Workgroups are persistent over pattern blocks.  Per block:
//     forward  -- walks a host-built post-order program whose child order
//                 minimises the stack (Strahler order).  Step v turns its
//                 children's "moved" partials a = P p into p_v = a_x * a_y
//                 and its own a_v = P_v p_v; a_v goes on a per-lane LDS stack
//                 and, once, to a per-workgroup HBM scratch region (fp64,
//                 16 B per lane per store, coalesced);
//     root     -- mixture sum through LDS, site log-likelihood, w/L scale;
//     reverse  -- walks the program backwards carrying the upper partial r
//                 of each branch on the stack: q_v = P_v^T r_v,
//                 r_x = q_v * a_y, and dL/dP_v += r_v (x) (a_x * a_y).  Each
//                 stored a is read exactly once (buffer-descriptor prefetch,
//                 one step ahead); dL/dP is reduced over the wave with
//                 permlane/DPP ops into an LDS accumulator.
//   P-matrices and their dL/dP accumulators are staged in LDS in chunks of
//   the program ("matrices in order of use"), sized to the LDS budget.
//   Finalize kernels sum the per-workgroup slots in a fixed order (bitwise
//   deterministic) and apply dP/dt = Q P for the branch-length and rate
//   gradients.
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
#ifndef PHY_ABLATE
#define PHY_ABLATE 0  // diagnostic builds only: 1 no dL/dP accumulation, 2 no reverse pass, 4 no scratch stores
#endif
// Program step (8 ints): x, y (child codes: tip index >= 0, or -(slot+1) of
// an internal child's stored moved partial), mx, my (matrix of a tip child,
// -1 if internal), mv (matrix of the step's own branch, -1 at the root),
// vslot (scratch slot of a_v, -1 at the root), flags (bit 0: mv is a real
// branch, not the merged identity), node id.
constexpr int STEP_INTS = 8;
// Per-draw eigensystem record: P(t) = m1 diag(exp(lam t)) m2, plus Q.
constexpr int EIG_LEN = 56;  // m1[16] lam[4] m2[16] Q[16] (+pad)
constexpr int EIG_M1 = 0, EIG_LAM = 16, EIG_M2 = 20, EIG_Q = 36;

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

// Same products with the matrix read straight from LDS at the point of use
// (wave-uniform address: broadcast reads), so no 32-VGPR copy stays live.
__device__ __forceinline__ V4 matvec_p(const double* __restrict__ M, const V4& v) {
  const double2 m01 = *reinterpret_cast<const double2*>(M + 0), m23 = *reinterpret_cast<const double2*>(M + 2);
  const double2 m45 = *reinterpret_cast<const double2*>(M + 4), m67 = *reinterpret_cast<const double2*>(M + 6);
  const double2 m89 = *reinterpret_cast<const double2*>(M + 8), mab = *reinterpret_cast<const double2*>(M + 10);
  const double2 mcd = *reinterpret_cast<const double2*>(M + 12), mef = *reinterpret_cast<const double2*>(M + 14);
  V4 r;
  r.x = fma(m23.y, v.w, fma(m23.x, v.z, fma(m01.y, v.y, m01.x * v.x)));
  r.y = fma(m67.y, v.w, fma(m67.x, v.z, fma(m45.y, v.y, m45.x * v.x)));
  r.z = fma(mab.y, v.w, fma(mab.x, v.z, fma(m89.y, v.y, m89.x * v.x)));
  r.w = fma(mef.y, v.w, fma(mef.x, v.z, fma(mcd.y, v.y, mcd.x * v.x)));
  return r;
}
__device__ __forceinline__ V4 matTvec_p(const double* __restrict__ M, const V4& v) {
  const double2 m01 = *reinterpret_cast<const double2*>(M + 0), m23 = *reinterpret_cast<const double2*>(M + 2);
  const double2 m45 = *reinterpret_cast<const double2*>(M + 4), m67 = *reinterpret_cast<const double2*>(M + 6);
  const double2 m89 = *reinterpret_cast<const double2*>(M + 8), mab = *reinterpret_cast<const double2*>(M + 10);
  const double2 mcd = *reinterpret_cast<const double2*>(M + 12), mef = *reinterpret_cast<const double2*>(M + 14);
  V4 r;
  r.x = fma(mcd.x, v.w, fma(m89.x, v.z, fma(m45.x, v.y, m01.x * v.x)));
  r.y = fma(mcd.y, v.w, fma(m89.y, v.z, fma(m45.y, v.y, m01.y * v.x)));
  r.z = fma(mef.x, v.w, fma(mab.x, v.z, fma(m67.x, v.y, m23.x * v.x)));
  r.w = fma(mef.y, v.w, fma(mab.y, v.z, fma(m67.y, v.y, m23.y * v.x)));
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

// Cross-lane moves on doubles (two 32-bit halves each).
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
// v_permlane32_swap (gfx950): a <- [a_lo | b_lo], b <- [a_hi | b_hi]  (32-lane halves)
__device__ __forceinline__ void swap32(double& a, double& b) {
  auto l = __builtin_amdgcn_permlane32_swap(__double2loint(a), __double2loint(b), false, false);
  auto h = __builtin_amdgcn_permlane32_swap(__double2hiint(a), __double2hiint(b), false, false);
  a = __hiloint2double(h[0], l[0]);
  b = __hiloint2double(h[1], l[1]);
}
// v_permlane16_swap (gfx950): odd 16-lane rows of a <-> even rows of b
__device__ __forceinline__ void swap16(double& a, double& b) {
  auto l = __builtin_amdgcn_permlane16_swap(__double2loint(a), __double2loint(b), false, false);
  auto h = __builtin_amdgcn_permlane16_swap(__double2hiint(a), __double2hiint(b), false, false);
  a = __hiloint2double(h[0], l[0]);
  b = __hiloint2double(h[1], l[1]);
}
constexpr int DPP_ROW_ROR8 = 0x128;       // lane l <- l ^ 8 within a 16-lane row
constexpr int DPP_ROW_HALF_MIRROR = 0x141;  // lane i <- 7 - i within 8 lanes (bit 2 flips)
constexpr int DPP_QUAD_XOR1 = 0xB1;       // quad_perm [1,0,3,2]
constexpr int DPP_QUAD_XOR2 = 0x4E;       // quad_perm [2,3,0,1]

// Transpose-reduce of 16 per-lane values over the 64 lanes of a wave, all in
// VALU cross-lane ops (no LDS, no waitcnt).  Each halving stage pairs lanes
// that differ in one bit and leaves each lane with the half selected by that
// bit, summed with its partner's: bit 5 and bit 4 by the gfx950 permlane32/16
// swaps (no selects needed), bit 3 by DPP row_ror:8, bit 2 by DPP
// row_half_mirror; two quad DPP adds finish the sums.  On return lane l holds
// the full sum of entry e(l) = 8*b5 + 4*b4 + 2*b3 + b2 (bits of l),
// replicated over l&3.  The summation tree is fixed: deterministic.
__device__ __forceinline__ double reduce16(double (&v)[16], int lane) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {  // bit 5: lanes <32 keep entry k, >=32 entry k+8
    swap32(v[k], v[k + 8]);
    v[k] += v[k + 8];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // bit 4: even rows keep k, odd rows k+4
    swap16(v[k], v[k + 4]);
    v[k] += v[k + 4];
  }
  {
    const bool hi = lane & 8;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const double send = hi ? v[k] : v[k + 2];
      const double keep = hi ? v[k + 2] : v[k];
      v[k] = keep + dpp_d<DPP_ROW_ROR8>(send);
    }
  }
  {
    const bool hi = lane & 4;
    const double send = hi ? v[0] : v[1];
    const double keep = hi ? v[1] : v[0];
    v[0] = keep + dpp_d<DPP_ROW_HALF_MIRROR>(send);
  }
  double s = v[0];
  s += dpp_d<DPP_QUAD_XOR1>(s);
  s += dpp_d<DPP_QUAD_XOR2>(s);
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
  const double* pmat;     // [draw][C][nmat][16]  P of every branch, in program-use order
  const double* model;    // [draw][10+2C]
  double2* scratch;       // [wg][nslots][K][2][C*64]   stored moved partials
  double* gslot;          // [wg][C][nmat][16]          dL/dP partial sums, program-use order
  double* sslot;          // [wg][C][8]
  double* site_ll;        // [draw][P] or null
  unsigned long long* stamps;  // diagnostic builds (PHY_STAMP): [wg][C][8] s_memtime
  double* out;            // [draw][outlen]: dL/dP rows written in place when g_direct
  const int* mat_branch;  // [nmat] branch of matrix m (-1: identity)
  const double* eig;      // [draw][EIG_LEN] (Q for the chain rule)
  double* inner;          // [draw][C][B] <G, Q P> when g_direct
  int S, P, Ppad, C, nsteps, nslots, nblk, depth, nmat, cap_m;
  int B, outlen, g_direct;  // g_direct: one workgroup per draw
};

#ifndef PHY_STAMP
#define PHY_STAMP 0
#endif
#ifndef PHY_PF
#define PHY_PF 1  // reverse-pass prefetch distance (steps): 1 or 2
#endif
#define STAMP(k)                                                                      \
  do {                                                                                \
    if (PHY_STAMP && a.stamps && blk0 && lane == 0)                                   \
      a.stamps[((size_t)wg * C + c) * 8 + (k)] = __builtin_amdgcn_s_memtime();         \
  } while (0)

// LDS carve (all offsets multiples of 16 B), K columns per lane:
//   P chunk  C * cap_m * 16 double   (matrices [m0, m0+cap_m) of the chunk)
//   G chunk  C * cap_m * 16 double   (their dL/dP accumulators)
//   stacks   C waves x max(depth-1, 1) entries x K x 2 x 64 double2 (the
//            top entry lives in registers); wave c's slice of the root
//            exchange rootL (K x 64 double) aliases the start of its own
//            stack, which is empty at the root
//   tips     S * 64 * K bytes (rounded to 16)
__host__ __device__ inline size_t wave_stack_bytes(int depth, int K) {
  return (size_t)(depth > 2 ? depth - 1 : 1) * K * 2 * WAVE * 16;
}
__host__ __device__ inline size_t stack_bytes(int C, int depth, int K) {
  return (size_t)C * wave_stack_bytes(depth, K);
}
__host__ __device__ inline size_t lds_bytes(int S, int C, int depth, int cap_m, int K) {
  size_t b = 2 * (size_t)C * cap_m * 16 * 8;
  b += stack_bytes(C, depth, K);
  b += ((size_t)S * WAVE * K + 15) / 16 * 16;
  return b;
}

// Buffer resource for the workgroup's scratch region: buffer loads past
// num_records return zeros without touching memory, which lets the reverse
// pass issue its prefetch unconditionally (tip children get an out-of-range
// offset) -- no divergent-looking load paths for the waitcnt pass.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
  void* p = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)n, 0x00020000);
}

// s_waitcnt vmcnt(0) that the compiler's waitcnt pass sees (an inline-asm
// wait would be invisible to it): clears loads left pending by staging /
// flush loops so the step loops are not charged a loop-carried vmcnt(0).
#define WAIT_VMCNT0() __builtin_amdgcn_s_waitcnt(0x0F70)

// Chunk staging and dL/dP flushes (run at chunk switches only).
#ifndef PHY_OUTLINE
#define PHY_OUTLINE 0  // 1: out-of-line calls (measured slower on MI355X)
#endif
#if PHY_OUTLINE
#define PHY_CHUNK_FN __device__ __noinline__
#else
#define PHY_CHUNK_FN __device__ __forceinline__
#endif

// P-matrices [lo, lo+n) of every category -> LDS (one contiguous run of n*16
// doubles per category, 8 loads in flight per thread before the writes).
PHY_CHUNK_FN void stage_chunk(double* pl, const double* pmat_d, int C, int cap_m, int nmat, int lo, int n) {
  const int nthreads = blockDim.x;
  const int q2 = n * 8;  // double2 per category
  for (int cc = 0; cc < C; ++cc) {
    const double2* src = reinterpret_cast<const double2*>(pmat_d + ((size_t)cc * nmat + lo) * 16);
    double2* dst = reinterpret_cast<double2*>(pl + (size_t)cc * cap_m * 16);
    for (int k0 = threadIdx.x; k0 < q2; k0 += nthreads * 8) {
      double2 buf[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u * nthreads;
        buf[u] = (k < q2) ? src[k] : make_double2(0.0, 0.0);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u * nthreads;
        if (k < q2) dst[k] = buf[u];
      }
    }
  }
  WAIT_VMCNT0();  // no staging load may look pending inside the step loops
}

// Hand the LDS dL/dP chunk (matrices [m0, m0+q/16)) to the workgroup's slot
// and zero it: a plain store the first time (g_first), else load-add-store,
// contiguous in program order.  With fin (one workgroup per draw, its last
// pattern block) the totals go to the draw's output rows in branch order
// and each 16-thread group -- one matrix -- also reduces <G, Q P> into
// inner[c][b] (the chain rule dP/dt = Q P), from the P chunk still in LDS.
PHY_CHUNK_FN void flush_chunk(double* gl, const double* pl, double* gslot_wg, double* gout, double* inner_d,
                              const double* Qd, const int* mat_branch, int C, int cap_m, int nmat, int B, int m0,
                              int q, bool g_first, bool fin) {
  const int nthreads = blockDim.x;
  for (int cc = 0; cc < C; ++cc) {
    double* gp = gslot_wg + ((size_t)cc * nmat + m0) * 16;
    double* lp = gl + (size_t)cc * cap_m * 16;
    const double* pp = pl + (size_t)cc * cap_m * 16;
    for (int k0 = threadIdx.x; k0 < q; k0 += nthreads * 8) {
      double old[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u * nthreads;
        old[u] = (!g_first && k < q) ? gp[k] : 0.0;
      }
      if (!fin) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = k0 + u * nthreads;
          if (k < q) {
            gp[k] = old[u] + lp[k];
            lp[k] = 0.0;
          }
        }
        continue;
      }
      // 16 consecutive threads hold one matrix (q and the thread count are
      // multiples of 16), so the groups are uniformly active
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u * nthreads;
        if (k < q) {
          const int mm = k >> 4, e16 = k & 15, j = e16 >> 2, kk = e16 & 3;
          const double g = old[u] + lp[k];
          lp[k] = 0.0;
          const int b = mat_branch[m0 + mm];
          double qp = 0.0;
#pragma unroll
          for (int l = 0; l < 4; ++l) qp = fma(Qd[j * 4 + l], pp[mm * 16 + l * 4 + kk], qp);
          double s = g * qp;
          s += __shfl_xor(s, 8, 16);
          s += __shfl_xor(s, 4, 16);
          s += __shfl_xor(s, 2, 16);
          s += __shfl_xor(s, 1, 16);
          if (b >= 0) {
            gout[((size_t)cc * B + b) * 16 + e16] = g;
            if (e16 == 0) inner_d[(size_t)cc * B + b] = s;  // dlogL/dt_{b,c}
          }
        }
      }
    }
  }
  WAIT_VMCNT0();
}

// K mat-vecs sharing one read of the (wave-uniform, LDS-broadcast) matrix.
template <int K>
__device__ __forceinline__ void matvec_k(const double* __restrict__ M, const V4 (&v)[K], V4 (&r)[K]) {
  const double2 m01 = *reinterpret_cast<const double2*>(M + 0), m23 = *reinterpret_cast<const double2*>(M + 2);
  const double2 m45 = *reinterpret_cast<const double2*>(M + 4), m67 = *reinterpret_cast<const double2*>(M + 6);
  const double2 m89 = *reinterpret_cast<const double2*>(M + 8), mab = *reinterpret_cast<const double2*>(M + 10);
  const double2 mcd = *reinterpret_cast<const double2*>(M + 12), mef = *reinterpret_cast<const double2*>(M + 14);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const V4 x = v[k];
    r[k].x = fma(m23.y, x.w, fma(m23.x, x.z, fma(m01.y, x.y, m01.x * x.x)));
    r[k].y = fma(m67.y, x.w, fma(m67.x, x.z, fma(m45.y, x.y, m45.x * x.x)));
    r[k].z = fma(mab.y, x.w, fma(mab.x, x.z, fma(m89.y, x.y, m89.x * x.x)));
    r[k].w = fma(mef.y, x.w, fma(mef.x, x.z, fma(mcd.y, x.y, mcd.x * x.x)));
  }
}
template <int K>
__device__ __forceinline__ void matTvec_k(const double* __restrict__ M, const V4 (&v)[K], V4 (&r)[K]) {
  const double2 m01 = *reinterpret_cast<const double2*>(M + 0), m23 = *reinterpret_cast<const double2*>(M + 2);
  const double2 m45 = *reinterpret_cast<const double2*>(M + 4), m67 = *reinterpret_cast<const double2*>(M + 6);
  const double2 m89 = *reinterpret_cast<const double2*>(M + 8), mab = *reinterpret_cast<const double2*>(M + 10);
  const double2 mcd = *reinterpret_cast<const double2*>(M + 12), mef = *reinterpret_cast<const double2*>(M + 14);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const V4 x = v[k];
    r[k].x = fma(mcd.x, x.w, fma(m89.x, x.z, fma(m45.x, x.y, m01.x * x.x)));
    r[k].y = fma(mcd.y, x.w, fma(m89.y, x.z, fma(m45.y, x.y, m01.y * x.x)));
    r[k].z = fma(mef.x, x.w, fma(mab.x, x.z, fma(m67.x, x.y, m23.x * x.x)));
    r[k].w = fma(mef.y, x.w, fma(mab.y, x.z, fma(m67.y, x.y, m23.y * x.x)));
  }
}

// `prog`, `chunk_of` and `chunk_m0` are separate __restrict__ const
// arguments so the backend proves them read-only and uses scalar loads.
//
// K columns per lane: lane l of the category-c wave owns patterns
// blk*64K + k*64 + l, k < K.  The columns share every matrix read, the
// program/stack control flow and -- the main saving -- one wave reduction
// of the summed outer products per branch.
// Register budget: two waves per SIMD (<= 256 VGPRs) -- the occupancy the
// default 80 KiB LDS plan allows.  PHY_WPE overrides it in diagnostic builds.
#ifndef PHY_WPE
#define PHY_WPE 2
#endif
template <int MAXT, int K>
__global__ void __launch_bounds__(MAXT) __attribute__((amdgpu_waves_per_eu(PHY_WPE)))
    sweep_kernel(SweepArgs a, const int* __restrict__ prog, const int* __restrict__ chunk_of,
                 const int* __restrict__ chunk_m0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  const int lane = threadIdx.x & (WAVE - 1);
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nthreads = blockDim.x;
  const int draw = blockIdx.y;
  const int wg = blockIdx.y * gridDim.x + blockIdx.x;
  const int C = a.C, nsteps = a.nsteps, nmat = a.nmat, cap_m = a.cap_m;
  const int ncolwg = C * WAVE;
  const bool one_chunk = chunk_of[0] == chunk_of[nsteps - 1];
  bool blk0 = true;  // first pattern block of this workgroup (diagnostic stamps)
  if (PHY_STAMP && a.stamps && lane == 0) {
    a.stamps[((size_t)wg * C + c) * 8 + 6] = __builtin_amdgcn_s_memrealtime();
    a.stamps[((size_t)wg * C + c) * 8 + 0] = __builtin_amdgcn_s_memtime();
  }

  double* pl = reinterpret_cast<double*>(lds_raw);  // [C][cap_m][16]
  double* gl = pl + (size_t)C * cap_m * 16;          // [C][cap_m][16]
  unsigned char* region = reinterpret_cast<unsigned char*>(gl + (size_t)C * cap_m * 16);
  const size_t wstk = wave_stack_bytes(a.depth, K);
  double2* stk = reinterpret_cast<double2*>(region + (size_t)c * wstk);
  // root exchange: wave cc's K x 64 values at the start of its own stack
  auto rootL = [&](int cc, int k) -> double* {
    return reinterpret_cast<double*>(region + (size_t)cc * wstk) + k * WAVE + lane;
  };
  unsigned char* tipl = region + stack_bytes(C, a.depth, K);

  const double* mdl = a.model + (size_t)draw * (10 + 2 * C);
  const V4 pi = {mdl[0], mdl[1], mdl[2], mdl[3]};
  const double ps_c = mdl[10 + C + c];
  const double* pmat_d = a.pmat + (size_t)draw * C * nmat * 16;
  double2* scr = a.scratch + (size_t)wg * a.nslots * K * 2 * ncolwg;
  double* gslot_wg = a.gslot + (size_t)wg * C * nmat * 16;
  const uint32_t scr_bytes = (uint32_t)((size_t)a.nslots * K * 2 * ncolwg * 16);
  const __amdgpu_buffer_rsrc_t srd = make_rsrc(scr, scr_bytes);

  const int e = reduce16_entry(lane);
  const bool gowner = (lane & 3) == 0;

  for (int k = threadIdx.x; k < C * cap_m * 16; k += nthreads) gl[k] = 0.0;

  double acc_ll = 0.0, acc_dps = 0.0;
  V4 acc_f = {0.0, 0.0, 0.0, 0.0};

  // ---- P-matrix / dL/dP chunks in LDS ----
  int cur = -1, m0 = 0, mcount = 0;
  // Hand the LDS G chunk to this workgroup's global slot and zero it: a
  // plain store the first time the slot region is written (the workgroup's
  // first pattern block), otherwise load-add-store, 8 loads in flight per
  // thread.
  // Flushes into the workgroup's slot are contiguous (program order).  With
  // one workgroup per draw (g_direct) the workgroup's LAST flush of each
  // chunk instead writes the draw's dL/dP output rows (branch order) and
  // forms the chain-rule inner products <G_cb, Q P_cb> from the P chunk
  // still in LDS, so the finalize pass never re-reads G or P.
  bool g_first = true, g_last = false;
  double* gout = a.out + (size_t)draw * a.outlen + 1 + a.B + 2 * C + 4;
  const double* Qd = a.eig + (size_t)draw * EIG_LEN + EIG_Q;
  double* inner_d = a.inner + (size_t)draw * C * a.B;
  auto flush_g = [&]() {
    if (cur < 0) return;
    flush_chunk(gl, pl, gslot_wg, gout, inner_d, Qd, a.mat_branch, C, cap_m, nmat, a.B, m0, mcount * 16,
                g_first, a.g_direct && g_last);
  };
  auto ensure_chunk = [&](int s, bool reverse) {
    const int ch = chunk_of[s];
    if (ch == cur) return;  // workgroup-uniform
    __syncthreads();
    if (reverse) flush_g();
    const int lo = chunk_m0[ch], n = chunk_m0[ch + 1] - lo;
    stage_chunk(pl, pmat_d, C, cap_m, nmat, lo, n);
    __syncthreads();
    cur = ch;
    m0 = lo;
    mcount = n;
  };
  auto pm = [&](int m) -> const double* { return pl + ((size_t)c * cap_m + (m - m0)) * 16; };

  // Pending-vector stack: the most recent entry stays in registers (most
  // pushes are popped by the very next step), older ones live in LDS,
  // [entry][k][half][lane] double2.
  int sp = 0;
  bool has_top = false;
  // top of stack: named scalars (a captured struct or array would be
  // demoted to scratch)
  double ta0 = 0.0, ta1 = 0.0, ta2 = 0.0, ta3 = 0.0, tb0 = 0.0, tb1 = 0.0, tb2 = 0.0, tb3 = 0.0;
  auto spill = [&](int k, double v0, double v1, double v2, double v3) {
    stk[((sp * K + k) * 2 + 0) * WAVE + lane] = make_double2(v0, v1);
    stk[((sp * K + k) * 2 + 1) * WAVE + lane] = make_double2(v2, v3);
  };
  auto push = [&](const V4 (&v)[K]) {
    if (has_top) {
      spill(0, ta0, ta1, ta2, ta3);
      if constexpr (K == 2) spill(1, tb0, tb1, tb2, tb3);
      ++sp;
    }
    ta0 = v[0].x;
    ta1 = v[0].y;
    ta2 = v[0].z;
    ta3 = v[0].w;
    if constexpr (K == 2) {
      tb0 = v[1].x;
      tb1 = v[1].y;
      tb2 = v[1].z;
      tb3 = v[1].w;
    }
    has_top = true;
  };
  auto pop = [&](V4 (&v)[K]) {
    if (has_top) {
      has_top = false;
      v[0] = {ta0, ta1, ta2, ta3};
      if constexpr (K == 2) v[1] = {tb0, tb1, tb2, tb3};
      return;
    }
    --sp;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double2 lo = stk[((sp * K + k) * 2 + 0) * WAVE + lane];
      const double2 hi = stk[((sp * K + k) * 2 + 1) * WAVE + lane];
      v[k] = {lo.x, lo.y, hi.x, hi.y};
    }
  };
  // dL/dP_m += sum_k r_k (x) p_k, reduced over the wave; the lane owning
  // entry e adds it to the LDS G chunk (one lane per address).
  auto gacc = [&](int m, const V4 (&r)[K], const V4 (&p)[K]) {
    double v[16];
    v[0] = r[0].x * p[0].x;  v[1] = r[0].x * p[0].y;  v[2] = r[0].x * p[0].z;  v[3] = r[0].x * p[0].w;
    v[4] = r[0].y * p[0].x;  v[5] = r[0].y * p[0].y;  v[6] = r[0].y * p[0].z;  v[7] = r[0].y * p[0].w;
    v[8] = r[0].z * p[0].x;  v[9] = r[0].z * p[0].y;  v[10] = r[0].z * p[0].z; v[11] = r[0].z * p[0].w;
    v[12] = r[0].w * p[0].x; v[13] = r[0].w * p[0].y; v[14] = r[0].w * p[0].z; v[15] = r[0].w * p[0].w;
#pragma unroll
    for (int k = 1; k < K; ++k) {
      v[0] = fma(r[k].x, p[k].x, v[0]);   v[1] = fma(r[k].x, p[k].y, v[1]);
      v[2] = fma(r[k].x, p[k].z, v[2]);   v[3] = fma(r[k].x, p[k].w, v[3]);
      v[4] = fma(r[k].y, p[k].x, v[4]);   v[5] = fma(r[k].y, p[k].y, v[5]);
      v[6] = fma(r[k].y, p[k].z, v[6]);   v[7] = fma(r[k].y, p[k].w, v[7]);
      v[8] = fma(r[k].z, p[k].x, v[8]);   v[9] = fma(r[k].z, p[k].y, v[9]);
      v[10] = fma(r[k].z, p[k].z, v[10]); v[11] = fma(r[k].z, p[k].w, v[11]);
      v[12] = fma(r[k].w, p[k].x, v[12]); v[13] = fma(r[k].w, p[k].y, v[13]);
      v[14] = fma(r[k].w, p[k].z, v[14]); v[15] = fma(r[k].w, p[k].w, v[15]);
    }
    if (PHY_ABLATE & 1) {
      asm volatile("" ::"v"(v[0]), "v"(v[5]), "v"(v[10]), "v"(v[15]));
      return;
    }
    const double sum = reduce16(v, lane);
    if (gowner) gl[((size_t)c * cap_m + (m - m0)) * 16 + e] += sum;
  };
  auto tip_code = [&](int t, int k) -> unsigned { return tipl[(t * K + k) * WAVE + lane]; };

  for (int blk = blockIdx.x; blk < a.nblk; blk += gridDim.x) {
    g_last = blk + (int)gridDim.x >= a.nblk;
    // stage this block's tip codes in LDS: S rows x 64K bytes, shared by the
    // C category-waves and by both passes (8 loads in flight per thread)
    {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(a.tips);
      uint32_t* dst = reinterpret_cast<uint32_t*>(tipl);
      const int rowq = a.Ppad / 4;
      constexpr int wq = WAVE * K / 4;  // words per tip row
      const int nq = a.S * wq;
      for (int k0 = threadIdx.x; k0 < nq; k0 += nthreads * 8) {
        uint32_t buf[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = k0 + u * nthreads;
          buf[u] = (k < nq) ? src[(size_t)(k / wq) * rowq + blk * wq + (k % wq)] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = k0 + u * nthreads;
          if (k < nq) dst[k] = buf[u];
        }
      }
    }
    __syncthreads();
    WAIT_VMCNT0();

    STAMP(1);
    // ------------------------------ forward ------------------------------
    sp = 0;
    has_top = false;
    V4 proot[K];
    for (int s = 0; s < nsteps; ++s) {
      ensure_chunk(s, false);
      const int* st = prog + s * STEP_INTS;
      const int x = st[0], y = st[1], mx = st[2], my = st[3], mv = st[4], vs = st[5], fl = st[6];
      V4 ax[K], ay[K], pv[K];
      if (y >= 0) {
        V4 tv[K];
#pragma unroll
        for (int k = 0; k < K; ++k) tv[k] = tipvec(tip_code(y, k));
        matvec_k<K>(pm(my), tv, ay);
      } else {
        pop(ay);
      }
      if (x >= 0) {
        V4 tv[K];
#pragma unroll
        for (int k = 0; k < K; ++k) tv[k] = tipvec(tip_code(x, k));
        matvec_k<K>(pm(mx), tv, ax);
      } else {
        pop(ax);
      }
#pragma unroll
      for (int k = 0; k < K; ++k) pv[k] = vmul(ax[k], ay[k]);
      if (vs >= 0) {
        V4 av[K];
        if (fl & 1) {
          matvec_k<K>(pm(mv), pv, av);
        } else {  // merged root branch: identity
#pragma unroll
          for (int k = 0; k < K; ++k) av[k] = pv[k];
        }
        if (!(PHY_ABLATE & 4)) {
#pragma unroll
          for (int k = 0; k < K; ++k) {
            double2* dst = scr + (size_t)((vs * K + k) * 2) * ncolwg + c * WAVE + lane;
            dst[0] = make_double2(av[k].x, av[k].y);
            dst[ncolwg] = make_double2(av[k].z, av[k].w);
          }
        }
        push(av);
      } else {
#pragma unroll
        for (int k = 0; k < K; ++k) proot[k] = pv[k];
      }
    }

    STAMP(2);
    // ------------------------- root / site log L -------------------------
    double fp[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      fp[k] = vdot(pi, proot[k]);  // pi . p_root,c
      *rootL(c, k) = ps_c * fp[k];
    }
    __syncthreads();
    double L[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      L[k] = 0.0;
      for (int cc = 0; cc < C; ++cc) L[k] += *rootL(cc, k);
    }
    __syncthreads();  // rootL is stack space again from here on
    V4 qroot[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = blk * WAVE * K + k * WAVE + lane;  // pattern of this column
      const double w = a.weights[i];
      const double lnL = log(L[k]);
      if (c == 0) {
        acc_ll += w * lnL;
        if (a.site_ll != nullptr && i < a.P) a.site_ll[(size_t)draw * a.P + i] = lnL;
      }
      const double sc = w / L[k];
      const double s_c = sc * ps_c;
      acc_dps = fma(sc, fp[k], acc_dps);
      acc_f.x = fma(s_c, proot[k].x, acc_f.x);
      acc_f.y = fma(s_c, proot[k].y, acc_f.y);
      acc_f.z = fma(s_c, proot[k].z, acc_f.z);
      acc_f.w = fma(s_c, proot[k].w, acc_f.w);
      // upper partials are carried pre-scaled by w_i ps_c / L_i, so every
      // outer product below is already a dlogL/dP term
      qroot[k] = vscale(pi, s_c);
    }

    STAMP(3);
    // ------------------------------ reverse ------------------------------
    // Upper partials r travel down the stack (the root's q is pushed first;
    // the root step's own "branch" is the identity).
    sp = 0;
    has_top = false;
    push(qroot);
    const uint32_t col_off = (uint32_t)((c * WAVE + lane) * 16);
    auto ld_partial = [&](uint32_t off) -> V4 {
      const auto lo = __builtin_amdgcn_raw_buffer_load_b128(srd, off, 0, 0);
      const auto hi = __builtin_amdgcn_raw_buffer_load_b128(srd, off + (uint32_t)ncolwg * 16u, 0, 0);
      V4 r;
      r.x = __hiloint2double((int)lo[1], (int)lo[0]);
      r.y = __hiloint2double((int)lo[3], (int)lo[2]);
      r.z = __hiloint2double((int)hi[1], (int)hi[0]);
      r.w = __hiloint2double((int)hi[3], (int)hi[2]);
      return r;
    };
    if (!(PHY_ABLATE & 2)) {
      // The children of step s: codes, stored partials (zeros for tips:
      // out-of-range buffer offset), tip masks.  Requested PHY_PF steps
      // ahead into one of PHY_PF+1 register sets that rotate by name (the
      // loop is unrolled PHY_PF+1 times): no register copy of an in-flight
      // load, so nothing waits before the data is consumed.
      struct CSet {
        int x, y;
        V4 lx[K], ly[K];
        unsigned tx[K], ty[K];
      };
      auto load_set = [&](int s) -> CSet {
        CSet r;
        const int* sp_ = prog + max(s, 0) * STEP_INTS;
        r.x = (s >= 0) ? sp_[0] : 0;
        r.y = (s >= 0) ? sp_[1] : 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const uint32_t kx = (s >= 0 && r.x < 0) ? (uint32_t)(((-r.x - 1) * K + k) * 2 * ncolwg) * 16u + col_off
                                                  : scr_bytes;
          const uint32_t ky = (s >= 0 && r.y < 0) ? (uint32_t)(((-r.y - 1) * K + k) * 2 * ncolwg) * 16u + col_off
                                                  : scr_bytes;
          r.lx[k] = ld_partial(kx);
          r.ly[k] = ld_partial(ky);
          r.tx[k] = tip_code(max(r.x, 0), k);
          r.ty[k] = tip_code(max(r.y, 0), k);
        }
        return r;
      };
      auto rstep = [&](int s, const CSet& cs) {
        ensure_chunk(s, true);
        const int x = cs.x, y = cs.y;
        const int* st = prog + s * STEP_INTS;
        const int mx = st[2], my = st[3], mv = st[4], fl = st[6];
        V4 tvx[K], tvy[K], ax[K], ay[K], rv[K], qv[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          tvx[k] = tipvec(cs.tx[k]);
          tvy[k] = tipvec(cs.ty[k]);
        }
        if (x >= 0) {
          matvec_k<K>(pm(mx), tvx, ax);
        } else {
#pragma unroll
          for (int k = 0; k < K; ++k) ax[k] = cs.lx[k];
        }
        if (y >= 0) {
          matvec_k<K>(pm(my), tvy, ay);
        } else {
#pragma unroll
          for (int k = 0; k < K; ++k) ay[k] = cs.ly[k];
        }
        pop(rv);
        if (fl & 1) {
          V4 pv[K];
#pragma unroll
          for (int k = 0; k < K; ++k) pv[k] = vmul(ax[k], ay[k]);
          matTvec_k<K>(pm(mv), rv, qv);
          gacc(mv, rv, pv);  // dL/dP_v += r_v (x) p_v
        } else {  // root, or the merged root branch: identity
#pragma unroll
          for (int k = 0; k < K; ++k) qv[k] = rv[k];
        }
        V4 rx[K], ry[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          rx[k] = vmul(qv[k], ay[k]);
          ry[k] = vmul(qv[k], ax[k]);
        }
        if (x < 0) push(rx);
        if (y < 0) push(ry);
        if (x >= 0) gacc(mx, rx, tvx);
        if (y >= 0) gacc(my, ry, tvy);
      };
      int s = nsteps - 1;
#if PHY_PF >= 2
      CSet A = load_set(s), Bs = load_set(s - 1), Cs;
      for (;;) {
        Cs = load_set(s - 2);
        rstep(s, A);
        if (--s < 0) break;
        A = load_set(s - 2);
        rstep(s, Bs);
        if (--s < 0) break;
        Bs = load_set(s - 2);
        rstep(s, Cs);
        if (--s < 0) break;
      }
#else
      CSet A = load_set(s), Bs;
      for (;;) {
        Bs = load_set(s - 1);
        rstep(s, A);
        if (--s < 0) break;
        A = load_set(s - 1);
        rstep(s, Bs);
        if (--s < 0) break;
      }
#endif
      if (!one_chunk) {  // hand the last chunk's sums to the slot
        __syncthreads();
        flush_g();
        __syncthreads();
        g_first = false;  // every chunk of the slot has now been written once
      }
    }
    WAIT_VMCNT0();
    STAMP(4);
    blk0 = false;
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
  if (one_chunk) {  // G accumulated in LDS for the workgroup's lifetime
    __syncthreads();
    g_last = true;
    flush_g();
  }
  if (PHY_STAMP && a.stamps && lane == 0) {
    a.stamps[((size_t)wg * C + c) * 8 + 5] = __builtin_amdgcn_s_memtime();
    a.stamps[((size_t)wg * C + c) * 8 + 7] = __builtin_amdgcn_s_memrealtime();
  }
}

// ---------------------------------------------------------------------------
// P-matrices (generate_script.py:755-892)
// ---------------------------------------------------------------------------

struct PmatArgs {
  const double* model;    // [draw][10+2C]
  const double* blens;    // [draw][B]
  const int* mat_branch;  // [nmat] branch (node id) of matrix m, -1 = identity
  double* eig;            // [draw][EIG_LEN]
  double* pmat;           // [draw][C][nmat][16]  program-use order
  int C, B, kind, nmat, n;
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
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int q = p + 1; q < 4; ++q) {
        const double apq = A[p][q];
        if (apq == 0.0) continue;
        const double theta = (A[q][q] - A[p][p]) / (2.0 * apq);
        const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double cs = 1.0 / sqrt(t * t + 1.0);
        const double sn = t * cs;
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // A <- A R   (columns p, q)
          const double akp = A[k][p], akq = A[k][q];
          A[k][p] = cs * akp - sn * akq;
          A[k][q] = sn * akp + cs * akq;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // A <- R^T A (rows p, q)
          const double apk = A[p][k], aqk = A[q][k];
          A[p][k] = cs * apk - sn * aqk;
          A[q][k] = sn * apk + cs * aqk;
        }
        A[p][q] = A[q][p] = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // V <- V R
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = cs * vkp - sn * vkq;
          V[k][q] = sn * vkp + cs * vkq;
        }
      }
  }
  for (int i = 0; i < 4; ++i) lam[i] = A[i][i];
}

// One thread per draw: normalised Q and its eigensystem.
__global__ void __launch_bounds__(64) eig_kernel(PmatArgs a) {
  const int draw = blockIdx.x * blockDim.x + threadIdx.x;
  if (draw >= a.n) return;
  const int C = a.C;
  const double* mdl = a.model + (size_t)draw * (10 + 2 * C);
  double* out = a.eig + (size_t)draw * EIG_LEN;
  if (a.kind == PHY_JC69) {  // generate_script.py:765-769 (closed form; Q for dP/dt only)
    for (int j = 0; j < 4; ++j)
      for (int k = 0; k < 4; ++k) out[EIG_Q + j * 4 + k] = (j == k) ? -1.0 : 1.0 / 3.0;
    return;
  }
  const double f[4] = {mdl[0], mdl[1], mdl[2], mdl[3]};
  const double* r = mdl + 4;  // AC AG AT CG CT GT  (generate_script.py:855-858)
  const double R[4][4] = {{0.0, r[0], r[1], r[2]}, {r[0], 0.0, r[3], r[4]}, {r[1], r[3], 0.0, r[5]},
                          {r[2], r[4], r[5], 0.0}};
  double q[4][4];
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // Q = R diag(pi), zero-sum rows (:862-867)
    double row = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      q[j][k] = (j == k) ? 0.0 : R[j][k] * f[k];
      row += q[j][k];
    }
    q[j][j] = -row;
    s -= q[j][j] * f[j];
  }
  double A[4][4], V[4][4], l[4], sq[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) sq[j] = sqrt(f[j]);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      q[j][k] /= s;  // :868
      out[EIG_Q + j * 4 + k] = q[j][k];
    }
#pragma unroll
  for (int j = 0; j < 4; ++j)  // A = Pi^1/2 Q Pi^-1/2, symmetrised (:870)
#pragma unroll
    for (int k = 0; k < 4; ++k)
      A[j][k] = (j == k) ? q[j][j] : 0.5 * (sq[j] * q[j][k] / sq[k] + sq[k] * q[k][j] / sq[j]);
  jacobi4(A, V, l);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    out[EIG_LAM + j] = l[j];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      out[EIG_M1 + j * 4 + k] = V[j][k] / sq[j];  // Pi^-1/2 V      (:875)
      out[EIG_M2 + j * 4 + k] = V[k][j] * sq[k];  // V^T Pi^1/2     (:876)
    }
  }
}

// One thread per (draw, category, matrix): P in program-use order.
__global__ void __launch_bounds__(256) pmat_kernel(PmatArgs a) {
  __shared__ double e[EIG_LEN];
  const int draw = blockIdx.y;
  const int C = a.C, nmat = a.nmat;
  if (threadIdx.x < EIG_LEN) e[threadIdx.x] = a.eig[(size_t)draw * EIG_LEN + threadIdx.x];
  __syncthreads();
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= C * nmat) return;
  const int c = idx / nmat, m = idx - c * nmat;
  const int br = a.mat_branch[m];
  double2* po = reinterpret_cast<double2*>(a.pmat + (((size_t)draw * C + c) * nmat + m) * 16);
  double P[16];
  if (br < 0) {  // the merged root branch of an unrooted tree (generate_script.py:1019)
#pragma unroll
    for (int k = 0; k < 16; ++k) P[k] = (k % 5 == 0) ? 1.0 : 0.0;
  } else {
    const double* mdl = a.model + (size_t)draw * (10 + 2 * C);
    const double t = a.blens[(size_t)draw * a.B + br] * mdl[10 + c];
    if (a.kind == PHY_JC69) {  // generate_script.py:765-769
      const double ex = exp(-t / 0.75);
      const double off = 0.25 - 0.25 * ex, d = 0.25 + 0.75 * ex;
#pragma unroll
      for (int k = 0; k < 16; ++k) P[k] = (k % 5 == 0) ? d : off;
    } else {  // m1 diag(exp(lam t)) m2   (:880)
      double E[4];
#pragma unroll
      for (int l = 0; l < 4; ++l) E[l] = exp(e[EIG_LAM + l] * t);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          double acc = 0.0;
#pragma unroll
          for (int l = 0; l < 4; ++l) acc = fma(e[EIG_M1 + j * 4 + l] * E[l], e[EIG_M2 + l * 4 + k], acc);
          P[j * 4 + k] = acc;
        }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) po[k] = make_double2(P[2 * k], P[2 * k + 1]);
}

// ---------------------------------------------------------------------------
// finalize: fixed-order sums of the per-workgroup slots + chain rule dP/dt
// ---------------------------------------------------------------------------
struct FinArgs {
  const double* gslot;  // [wg][C][nmat][16]  program-use order
  const double* sslot;  // [wg][C][8]
  const double* pmat;   // [draw][C][nmat][16]
  const double* eig;    // [draw][EIG_LEN]
  const double* blens;  // [draw][B]
  const double* model;  // [draw][10+2C]
  const int* gpos;      // [B] matrix index of branch b
  const double* inner;  // [draw][C][B] <G, Q P> from the sweep when g_direct
  double* out;          // [draw][outlen]
  int C, B, nmat, gx, outlen, g_direct;
};

// dL/dP of a draw spread over several workgroups: out[draw][og + (c*B+b)*16
// + k] = sum of the draw's workgroup slots, in slot order (bitwise
// deterministic).  64 entries x 4 slot strides per workgroup, 8 loads in
// flight per thread.
__global__ void __launch_bounds__(256) gsum_kernel(FinArgs a) {
  __shared__ double part[4][64];
  const int draw = blockIdx.y;
  const int C = a.C, B = a.B;
  const int ng = C * B * 16;
  const int idx = blockIdx.x * 64 + (threadIdx.x & 63);
  const int grp = threadIdx.x >> 6;
  const size_t per_wg = (size_t)C * a.nmat * 16;
  const size_t wg0 = (size_t)draw * a.gx;
  double acc = 0.0;
  if (idx < ng) {
    const int c = idx / (B * 16), rem = idx - c * B * 16;
    const int b = rem >> 4, k = rem & 15;
    const double* src = a.gslot + wg0 * per_wg + ((size_t)c * a.nmat + a.gpos[b]) * 16 + k;
    for (int w0 = grp; w0 < a.gx; w0 += 4 * 8) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int w = w0 + 4 * u;
        v[u] = (w < a.gx) ? src[(size_t)w * per_wg] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
  }
  part[grp][threadIdx.x & 63] = acc;
  __syncthreads();
  if (grp == 0 && idx < ng) {
    const double s = ((part[0][threadIdx.x] + part[1][threadIdx.x]) + part[2][threadIdx.x]) + part[3][threadIdx.x];
    a.out[(size_t)draw * a.outlen + 1 + B + 2 * C + 4 + idx] = s;
  }
}

// One workgroup per draw (dL/dP rows already in place: sweep or gsum).
//   scalars log L, dlogL/dps, root-frequency term: wave 0, lane-strided
//           over slots + a fixed-shape wave reduction;
//   chain rule  dlogL/dt_{b,c} = <G_bc, Q P_bc>,  dlogL/db = sum_c r_c (.),
//           dlogL/dr_c = sum_b b (.)   (generate_script.py:663-671 blens).
__global__ void __launch_bounds__(256) finalize_kernel(FinArgs a) {
  extern __shared__ double fsh[];  // inner[C*B], Q[16]
  const int draw = blockIdx.x;
  const int C = a.C, B = a.B;
  double* inner = fsh;
  double* Q = fsh + (size_t)C * B;
  double* out = a.out + (size_t)draw * a.outlen;
  const size_t wg0 = (size_t)draw * a.gx;
  const int og = 1 + B + 2 * C + 4;
  if (threadIdx.x < 16) Q[threadIdx.x] = a.eig[(size_t)draw * EIG_LEN + EIG_Q + threadIdx.x];
  if (threadIdx.x < WAVE) {
    // scalar partials per slot: [c][8] = ll (c = 0 only), dps_c, dfreq[4]
    const int lane = threadIdx.x;
    const int nq = 2 + C + 4;  // ll, dps_0..C-1, dfreq_0..3 (+1 spare)
    for (int q = 0; q < nq - 1; ++q) {
      double acc = 0.0;
      for (int w = lane; w < a.gx; w += WAVE) {
        const double* ss = a.sslot + (wg0 + w) * C * 8;
        if (q == 0) {
          acc += ss[0];
        } else if (q <= C) {
          acc += ss[(q - 1) * 8 + 1];
        } else {
          double t = 0.0;
          for (int c = 0; c < C; ++c) t += ss[c * 8 + 2 + (q - 1 - C)];
          acc += t;
        }
      }
      acc = wave_sum(acc);
      if (lane == 0) {
        if (q == 0)
          out[0] = isfinite(acc) ? acc : -INFINITY;
        else if (q <= C)
          out[1 + B + C + (q - 1)] = acc;
        else
          out[1 + B + 2 * C + (q - 1 - C)] = acc;
      }
    }
  }
  __syncthreads();  // dL/dP rows and Q visible to the whole workgroup
  const double* pm = a.pmat + (size_t)draw * C * a.nmat * 16;
  for (int idx = threadIdx.x; idx < C * B; idx += blockDim.x) {
    if (a.g_direct) {  // formed by the sweep's last flush
      inner[idx] = a.inner[(size_t)draw * C * B + idx];
      continue;
    }
    const int c = idx / B, b = idx - c * B;
    const double* g = out + og + (size_t)idx * 16;
    const double* P = pm + ((size_t)c * a.nmat + a.gpos[b]) * 16;
    double gv[16], pv[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      gv[k] = g[k];
      pv[k] = P[k];
    }
    double s = 0.0;  // <G, Q P>
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        double qp = 0.0;
#pragma unroll
        for (int l = 0; l < 4; ++l) qp = fma(Q[j * 4 + l], pv[l * 4 + k], qp);
        s = fma(gv[j * 4 + k], qp, s);
      }
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
  int nsteps, nslots, depth, nblk, nmat;
  int wg_budget, cols_pref, wg_cap, lds_budget;
  int cu_count = 256, wg_resident = 512;  // resident workgroups of the current plan
  int K = 1;                   // columns per lane of the current plan
  int cap_m = 0, nchunks = 0;  // current LDS plan
  hipStream_t stream;
  std::vector<int> prog;  // host copy of the program
  uint8_t* d_tips = nullptr;
  double* d_w = nullptr;
  int* d_prog = nullptr;
  int* d_gpos = nullptr;
  int* d_mat_branch = nullptr;
  int* d_chunk_of = nullptr;
  int* d_chunk_m0 = nullptr;
  double* d_pmat = nullptr;
  double* d_eig = nullptr;
  double* d_inner = nullptr;
  double* d_model = nullptr;
  double* d_blens = nullptr;
  double* d_out = nullptr;
  double* d_site = nullptr;
  double2* d_scratch = nullptr;
  double* d_gslot = nullptr;
  double* d_sslot = nullptr;
  unsigned long long* d_stamps = nullptr;
  bool timing = false;
  std::vector<hipEvent_t> ev;  // pairs
  int ev_used = 0;
  double timed_ms = 0.0;
  int timed_n = 0;
};

namespace {

void free_ctx(phy_ctx* c) {
  if (!c) return;
  int dev_old = 0;
  (void)hipGetDevice(&dev_old);
  (void)hipSetDevice(c->device);
  void* ptrs[] = {c->d_tips,  c->d_w,     c->d_prog,    c->d_gpos,    c->d_mat_branch, c->d_chunk_of,
                  c->d_chunk_m0, c->d_pmat, c->d_eig, c->d_inner,    c->d_model,   c->d_blens,      c->d_out,
                  c->d_site,  c->d_scratch, c->d_gslot, c->d_sslot,   c->d_stamps};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  (void)hipSetDevice(dev_old);
  delete c;
}

// Build the traversal program (see DESIGN.md "Traversal program"):
// post-order with the child needing the deeper stack first, every stored
// moved partial in a slot, every branch matrix numbered in order of use.
int build_program(int S, const int32_t* peel, int rooted, std::vector<int>& prog,
                  std::vector<int>& mat_branch, int& nslots, int& depth) {
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
    if (merged < S) return fail(PHY_EINVAL, "unrooted peel: node 2S-3 must be internal");
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
  prog.assign((size_t)(S - 1) * STEP_INTS, -1);
  mat_branch.clear();
  for (int s = 0; s < S - 1; ++s) {
    const int v = steps[s];
    const int x = first[v], y = second[v];
    int* p = &prog[(size_t)s * STEP_INTS];
    p[0] = x < S ? x : -(slot[x] + 1);
    p[1] = y < S ? y : -(slot[y] + 1);
    p[2] = p[3] = p[4] = -1;
    if (x < S) {  // tip children: their matrices are used at this step
      p[2] = (int)mat_branch.size();
      mat_branch.push_back(x);
    }
    if (y < S) {
      p[3] = (int)mat_branch.size();
      mat_branch.push_back(y);
    }
    if (v != root) {  // the step's own branch (identity for the merged one)
      p[4] = (int)mat_branch.size();
      mat_branch.push_back(v == merged ? -1 : v);
    }
    p[5] = (v == root) ? -1 : slot[v];
    p[6] = (v != root && v != merged) ? 1 : 0;
    p[7] = v;
  }
  // simulate both passes to size the LDS stack exactly
  int sp = 0, mx = 0;
  for (int s = 0; s < S - 1; ++s) {
    const int* p = &prog[(size_t)s * STEP_INTS];
    if (p[1] < 0) --sp;
    if (p[0] < 0) --sp;
    if (sp < 0) return fail(PHY_EINVAL, "internal: forward stack underflow");
    if (p[5] >= 0) mx = std::max(mx, ++sp);
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

constexpr size_t LDS_CAP = 160 * 1024;

constexpr int MIN_CAP_K2 = 24;  // two columns per lane only if chunks stay this large

int nblk_for(int P, int K) { return (P + WAVE * K - 1) / (WAVE * K); }

// Columns per lane, matrices per LDS chunk and the chunk boundaries over the
// program.  A plan is (K, LDS budget); a chunk holds >= 3 matrices (one step
// uses up to three).  With the automatic budget (lds_budget 0) and columns
// (cols_pref 0) the first plan that keeps chunks of >= MIN_CAP_K2 matrices
// (or the whole program) wins, in this order (measured on MI355X):
//   K=2 at 80 KiB (2 workgroups per CU), K=2 at 160 KiB, K=1 at 80 KiB.
int plan_chunks(phy_ctx* c) {
  auto cap_for = [&](int K, size_t budget) {
    int cap = c->nmat;
    while (cap > 3 && lds_bytes(c->S, c->C, c->depth, cap, K) > budget) --cap;
    return cap;
  };
  auto good = [&](int K, size_t budget) {
    const int cap = cap_for(K, budget);
    return lds_bytes(c->S, c->C, c->depth, cap, K) <= budget && cap >= std::min(c->nmat, MIN_CAP_K2);
  };
  const size_t dflt = 80 * 1024;
  // two columns only up to 512-thread workgroups (C <= 8): at 1024 threads
  // the register budget is 128 VGPRs and the K=2 body would spill
  int K = (c->C > 8 && c->cols_pref == 0) ? 1 : c->cols_pref;
  size_t budget = c->lds_budget > 0 ? std::min<size_t>(LDS_CAP, (size_t)c->lds_budget) : 0;
  if (budget == 0) {
    if (K == 0) {
      if (good(2, dflt)) {
        K = 2, budget = dflt;
      } else if (good(2, LDS_CAP)) {
        K = 2, budget = LDS_CAP;
      } else {
        K = 1, budget = dflt;
      }
    } else {
      budget = (K == 2 && !good(2, dflt)) ? LDS_CAP : dflt;
    }
  } else if (K == 0) {
    K = good(2, budget) ? 2 : 1;
  }
  const int cap = cap_for(K, budget);
  if (lds_bytes(c->S, c->C, c->depth, cap, K) > LDS_CAP) return fail(PHY_EINVAL, "tree too deep for LDS");
  c->K = K;
  c->nblk = nblk_for(c->P, K);
  {
    // resident workgroups per CU: LDS-limited, and at most two waves per
    // SIMD (the kernel's register budget), C waves per workgroup
    const size_t lds = lds_bytes(c->S, c->C, c->depth, cap, K);
    const int by_lds = (int)std::max<size_t>(1, LDS_CAP / std::max<size_t>(lds, 1));
    const int by_waves = std::max(1, 8 / c->C);
    c->wg_resident = c->cu_count * std::min({by_lds, by_waves, 4});
  }
  if (cap == c->cap_m && c->d_chunk_of) return PHY_OK;
  std::vector<int> chunk_of(c->nsteps), m0{0};
  int used = 0, ch = 0;
  for (int s = 0; s < c->nsteps; ++s) {
    const int* p = &c->prog[(size_t)s * STEP_INTS];
    const int n = (p[2] >= 0) + (p[3] >= 0) + (p[4] >= 0);
    if (used + n > cap) {
      m0.push_back(m0.back() + used);
      used = 0;
      ++ch;
    }
    chunk_of[s] = ch;
    used += n;
  }
  m0.push_back(m0.back() + used);
  if (m0.back() != c->nmat) return fail(PHY_EINVAL, "internal: chunk plan does not cover the matrices");
  if (c->d_chunk_of) (void)hipFree(c->d_chunk_of);
  if (c->d_chunk_m0) (void)hipFree(c->d_chunk_m0);
  c->d_chunk_of = nullptr;
  c->d_chunk_m0 = nullptr;
  int rc = dalloc(&c->d_chunk_of, chunk_of.size());
  if (!rc) rc = dalloc(&c->d_chunk_m0, m0.size());
  if (rc) return rc;
  HIP_TRY(hipMemcpy(c->d_chunk_of, chunk_of.data(), chunk_of.size() * sizeof(int), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->d_chunk_m0, m0.data(), m0.size() * sizeof(int), hipMemcpyHostToDevice));
  c->cap_m = cap;
  c->nchunks = ch + 1;
  return PHY_OK;
}

int launch(phy_ctx* ctx, int n, const double* d_blens, const double* d_model, double* d_out,
           double* d_site, hipStream_t st) {
  const int C = ctx->C, B = ctx->B;
  {
    PmatArgs pa{d_model, d_blens, ctx->d_mat_branch, ctx->d_eig, ctx->d_pmat, C, B, ctx->kind, ctx->nmat, n};
    hipLaunchKernelGGL(eig_kernel, dim3((n + 63) / 64), dim3(64), 0, st, pa);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(pmat_kernel, dim3((C * ctx->nmat + 255) / 256, n), dim3(256), 0, st, pa);
    HIP_TRY(hipGetLastError());
  }
  // persistent workgroups: the explicit budget, else exactly what is resident
  const int budget = ctx->wg_budget > 0 ? ctx->wg_budget : ctx->wg_resident;
  const int gx = std::max(1, std::min(ctx->nblk, (budget + n - 1) / n));
  if ((size_t)gx * n > (size_t)ctx->wg_cap) return fail(PHY_ERANGE, "workgroup cap exceeded");
  const size_t lds = lds_bytes(ctx->S, C, ctx->depth, ctx->cap_m, ctx->K);
  const int g_direct = (gx == 1) ? 1 : 0;
  SweepArgs sa{ctx->d_tips,  ctx->d_w,       ctx->d_pmat,         d_model,     ctx->d_scratch,
               ctx->d_gslot, ctx->d_sslot,   d_site,              ctx->d_stamps, d_out,
               ctx->d_mat_branch, ctx->d_eig, ctx->d_inner, ctx->S,    ctx->P,              ctx->Ppad,   C,
               ctx->nsteps,  ctx->nslots,    ctx->nblk,           ctx->depth,  ctx->nmat,
               ctx->cap_m,   B,              phy_output_len(ctx), g_direct};
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
#define PHY_LAUNCH(T, K_)                                                                       \
  hipLaunchKernelGGL((sweep_kernel<T, K_>), dim3(gx, n), dim3(threads), lds, st, sa, ctx->d_prog, \
                     ctx->d_chunk_of, ctx->d_chunk_m0)
  if (ctx->K == 2) {
    if (threads <= 256)
      PHY_LAUNCH(256, 2);
    else if (threads <= 512)
      PHY_LAUNCH(512, 2);
    else
      PHY_LAUNCH(1024, 2);
  } else {
    if (threads <= 256)
      PHY_LAUNCH(256, 1);
    else if (threads <= 512)
      PHY_LAUNCH(512, 1);
    else
      PHY_LAUNCH(1024, 1);
  }
#undef PHY_LAUNCH
  HIP_TRY(hipGetLastError());
  if (ctx->timing) HIP_TRY(hipEventRecord(e1, st));
  FinArgs fa{ctx->d_gslot, ctx->d_sslot, ctx->d_pmat, ctx->d_eig, d_blens, d_model, ctx->d_gpos, ctx->d_inner, d_out,
             C,            B,            ctx->nmat,   gx,          phy_output_len(ctx), g_direct};
  if (!g_direct) {
    hipLaunchKernelGGL(gsum_kernel, dim3((C * B * 16 + 63) / 64, n), dim3(256), 0, st, fa);
    HIP_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(finalize_kernel, dim3(n), dim3(256), ((size_t)C * B + 16) * sizeof(double), st, fa);
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
  c->nblk = nblk_for(P, 1);
  c->Ppad = nblk_for(P, 2) * 2 * WAVE;  // room for either column plan
  c->stream = nullptr;
  std::vector<int> mat_branch;
  int rc = build_program(S, peel, c->rooted, c->prog, mat_branch, c->nslots, c->depth);
  if (rc) {
    delete c;
    return rc;
  }
  c->nsteps = S - 1;
  c->nmat = (int)mat_branch.size();
  c->cols_pref = 0;
  {
    const char* lb = getenv("PHY_LDS_BUDGET");
    c->lds_budget = lb ? std::max(16384, atoi(lb)) : 0;  // 0: automatic plan
    const char* env = getenv("PHY_WG_BUDGET");
    c->wg_budget = env ? std::max(1, atoi(env)) : 0;  // 0: resident workgroups of the plan
    const char* ck = getenv("PHY_COLS");
    c->cols_pref = ck ? std::max(0, std::min(2, atoi(ck))) : 0;
  }
  hipError_t he = hipSetDevice(device);
  if (he != hipSuccess) {
    delete c;
    return fail(PHY_EHIP, std::string("hipSetDevice: ") + hipGetErrorString(he));
  }
  {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
      c->cu_count = cus;
  }
  // workgroup slots: an explicit budget, or up to 4 resident per CU
  c->wg_cap = (int)std::min<long>((long)c->nblk * max_draws,
                                  (long)std::max(c->wg_budget, 4 * c->cu_count) + max_draws);
  // gfx950: one workgroup may use the whole 160 KiB LDS; dynamic LDS above
  // 64 KiB has to be opted into per kernel.
  {
    const void* ks[] = {(const void*)sweep_kernel<256, 1>, (const void*)sweep_kernel<512, 1>,
                        (const void*)sweep_kernel<1024, 1>, (const void*)sweep_kernel<256, 2>,
                        (const void*)sweep_kernel<512, 2>, (const void*)sweep_kernel<1024, 2>};
    for (const void* k : ks) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_CAP);
  }
  if (lds_bytes(S, C, c->depth, 3, 1) > LDS_CAP) {
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
  TRY_C(dalloc(&c->d_prog, c->prog.size()));
  TRY_C(dalloc(&c->d_mat_branch, (size_t)c->nmat));
  TRY_C(dalloc(&c->d_gpos, (size_t)c->B));
  TRY_C(dalloc(&c->d_pmat, (size_t)max_draws * C * c->nmat * 16));
  TRY_C(dalloc(&c->d_eig, (size_t)max_draws * EIG_LEN));
  TRY_C(dalloc(&c->d_inner, (size_t)max_draws * C * c->B));
  TRY_C(dalloc(&c->d_model, (size_t)max_draws * (10 + 2 * C)));
  TRY_C(dalloc(&c->d_blens, (size_t)max_draws * c->B));
  TRY_C(dalloc(&c->d_out, (size_t)max_draws * phy_output_len(c)));
  TRY_C(dalloc(&c->d_site, (size_t)max_draws * P));
  TRY_C(dalloc(&c->d_scratch, (size_t)c->wg_cap * std::max(c->nslots, 1) * 2 * 2 * ncolwg));
  TRY_C(dalloc(&c->d_gslot, (size_t)c->wg_cap * C * c->nmat * 16));
  TRY_C(dalloc(&c->d_sslot, (size_t)c->wg_cap * C * 8));
  if (PHY_STAMP) TRY_C(dalloc(&c->d_stamps, (size_t)c->wg_cap * C * 8));
  {
    std::vector<uint8_t> tips((size_t)S * c->Ppad, 15);
    for (int t = 0; t < S; ++t) std::memcpy(&tips[(size_t)t * c->Ppad], tipcodes + (size_t)t * P, P);
    std::vector<double> w(c->Ppad, 0.0);
    std::memcpy(w.data(), weights, sizeof(double) * P);
    std::vector<int> gpos(c->B, -1);
    for (int m = 0; m < c->nmat; ++m)
      if (mat_branch[m] >= 0) gpos[mat_branch[m]] = m;
    for (int b = 0; b < c->B; ++b)
      if (gpos[b] < 0) {
        std::string m_ = "internal: branch " + std::to_string(b) + " not in the program";
        free_ctx(c);
        return fail(PHY_EINVAL, m_);
      }
    HIP_C(hipMemcpy(c->d_tips, tips.data(), tips.size(), hipMemcpyHostToDevice));
    HIP_C(hipMemcpy(c->d_w, w.data(), w.size() * sizeof(double), hipMemcpyHostToDevice));
    HIP_C(hipMemcpy(c->d_prog, c->prog.data(), c->prog.size() * sizeof(int), hipMemcpyHostToDevice));
    HIP_C(hipMemcpy(c->d_mat_branch, mat_branch.data(), mat_branch.size() * sizeof(int), hipMemcpyHostToDevice));
    HIP_C(hipMemcpy(c->d_gpos, gpos.data(), gpos.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  TRY_C(plan_chunks(c));
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
  HIP_TRY(hipMemcpyAsync(ctx->d_blens, blens, sizeof(double) * n_draws * ctx->B, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(ctx->d_model, model, sizeof(double) * n_draws * ml, hipMemcpyHostToDevice, st));
  int rc = launch(ctx, n_draws, ctx->d_blens, ctx->d_model, ctx->d_out, site_ll ? ctx->d_site : nullptr, st);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out, ctx->d_out, sizeof(double) * n_draws * phy_output_len(ctx), hipMemcpyDeviceToHost,
                         st));
  if (site_ll)
    HIP_TRY(hipMemcpyAsync(site_ll, ctx->d_site, sizeof(double) * n_draws * ctx->P, hipMemcpyDeviceToHost, st));
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

int phy_set_tuning(phy_ctx* ctx, int wg_budget, int cols, int lds_budget) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (wg_budget > 0) {
    const long need = std::min<long>((long)nblk_for(ctx->P, 1) * ctx->max_draws,
                                     (long)std::max(wg_budget, 4 * ctx->cu_count) + ctx->max_draws);
    if (need > ctx->wg_cap) return fail(PHY_ERANGE, "wg_budget larger than allocated at create");
    ctx->wg_budget = wg_budget;
  }
  if (cols < 0 || cols > 2) return fail(PHY_EINVAL, "cols must be 0 (automatic), 1 or 2");
  ctx->cols_pref = cols;
  if (lds_budget > 0) ctx->lds_budget = std::max(16384, std::min(lds_budget, (int)LDS_CAP));
  HIP_TRY(hipSetDevice(ctx->device));
  return plan_chunks(ctx);
}

// Diagnostic builds (-DPHY_STAMP=1): copy the per-wave s_memtime stamps of
// the last launch ([wg][C][8]: start, fwd, root, rev, end-of-block, end,
// realtime start, realtime end).  Returns the number of values copied.
int phy_debug_stamps(phy_ctx* ctx, unsigned long long* out, int n) {
  if (!ctx || !ctx->d_stamps) return 0;
  const int m = std::min(n, ctx->wg_cap * ctx->C * 8);
  if (hipMemcpy(out, ctx->d_stamps, sizeof(unsigned long long) * m, hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  return m;
}

int phy_columns_per_lane(const phy_ctx* ctx) { return ctx ? ctx->K : -1; }

int phy_lds_plan(const phy_ctx* ctx, int* g_in_lds, int* chunk_steps, int* lds_bytes_out) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (g_in_lds) *g_in_lds = ctx->nchunks;  // number of P / dL/dP chunks per pass
  if (chunk_steps) *chunk_steps = ctx->cap_m;
  if (lds_bytes_out) *lds_bytes_out = (int)lds_bytes(ctx->S, ctx->C, ctx->depth, ctx->cap_m, ctx->K);
  return PHY_OK;
}

}  // extern "C"
