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
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "phylo_hip_diag.h"

namespace {

constexpr int WAVE = 64;
// Program step (STEP_INTS ints, host-built by build_program).
constexpr int STEP_INTS = 16;
enum {
  ST_X = 0,  // child x: tip index >= 0, or -1 (internal)
  ST_Y,      // child y: same
  ST_MX,     // matrix of a tip x (its branch), -1 otherwise
  ST_MY,     // matrix of a tip y
  ST_MV,     // matrix of the step's own branch (-1: root / merged branch)
  ST_VSLOT,  // scratch slot of a_v (-1 at the root)
  ST_FLAGS,  // F_* below
  ST_XSLOT,  // scratch slot of an internal x
  ST_YSLOT,  // scratch slot of an internal y
  ST_XDPOS,  // deep-stack entry of x when both children are internal
  ST_VDPOS,  // deep-stack entry of v when F_VDEEP
  ST_CHUNK,  // LDS chunk holding the step's matrices
  ST_M0,     // first matrix of that chunk
  ST_MN,     // matrices in that chunk
  ST_NODE,   // node id
  ST_RD,     // rebuild depth of the previous-step child (F_PREVREC): 1 cherry, 2.. chain
};
constexpr int F_MV = 1;     // the step's branch has a matrix (else identity)
constexpr int F_XDEEP = 2;  // both children internal: x's operand is on the deep stack
constexpr int F_VDEEP = 4;  // v is the x child of a both-internal parent
// Recomputed cherries (set per LDS plan, plan_chunks): a node whose children
// are both tips is not stored when it is the previous step of its parent and
// shares the parent's LDS chunk -- the parent's reverse step rebuilds it from
// the tips and matrices already in LDS (its step record is the one the
// reverse loaded a step ahead).
constexpr int F_NOSTORE = 8;   // this step's a_v is not written to scratch
constexpr int F_PREVREC = 16;  // the child computed at the previous step is rebuilt, not loaded
#ifndef PHY_EPI_U
#define PHY_EPI_U 4  // dL/dP slot items in flight per lane in the per-draw epilogue
#endif
#ifndef PHY_RD_MAX
#define PHY_RD_MAX 4
#endif
constexpr int RD_MAX = PHY_RD_MAX;  // deepest rebuild chain: a cherry plus up to RD_MAX-1 one-tip nodes above it

// The device copy of the program packs a step into 8 ints (pack_program):
//   w0 x | y<<16   w1 mx | my<<16   w2 mv | vslot<<16   w3 xslot | yslot<<16
//   w4 flags | xdpos<<8 | vdpos<<16 (8-bit fields)      w5 chunk | m0<<16
//   w6 mn | node<<16                                    w7 unused
// 16-bit fields are signed (-1 = none).  One s_load_dwordx8 per step, issued
// a step ahead, replaces a chain of dependent scalar loads.
constexpr int PSTEP = 8;
// The two-column kernel (K = 2, the batched throughput plan) reads the
// host's 16-int steps as they are (one s_load_dwordx16, no field
// extraction): measured 6.07-6.09 against 6.14 ms per fluA launch; the
// one-column latency kernel keeps the packed form (64-draw calls 181
// against 191 us with unpacked records).
constexpr int USTEP = STEP_INTS;
struct Step {
  int x, y, mx, my, mv, vs, fl, xs, ys, xd, vd, ch, m0, mn, rd;
};
__device__ __forceinline__ int lo16(int w) { return (int)(short)(w & 0xFFFF); }
__device__ __forceinline__ int hi16(int w) { return w >> 16; }
__device__ __forceinline__ int b8(int w, int k) { return (int)(signed char)((w >> (8 * k)) & 0xFF); }
template <bool UNP>
__device__ __forceinline__ Step ld_step(const int* __restrict__ prog, int s) {
  if constexpr (UNP) {
    const int4* q = reinterpret_cast<const int4*>(prog + s * USTEP);
    const int4 a = q[0], b = q[1], c = q[2], d = q[3];
    Step t;
    t.x = a.x; t.y = a.y; t.mx = a.z; t.my = a.w;   // ST_X .. ST_MY
    t.mv = b.x; t.vs = b.y; t.fl = b.z; t.xs = b.w;  // ST_MV .. ST_XSLOT
    t.ys = c.x; t.xd = c.y; t.vd = c.z; t.ch = c.w;  // ST_YSLOT .. ST_CHUNK
    t.m0 = d.x; t.mn = d.y; t.rd = d.w;              // ST_M0, ST_MN, (ST_NODE), ST_RD
    return t;
  }
  const int4 a = *reinterpret_cast<const int4*>(prog + s * PSTEP);
  const int4 b = *reinterpret_cast<const int4*>(prog + s * PSTEP + 4);
  Step t;
  t.x = lo16(a.x);
  t.y = hi16(a.x);
  t.mx = lo16(a.y);
  t.my = hi16(a.y);
  t.mv = lo16(a.z);
  t.vs = hi16(a.z);
  t.xs = lo16(a.w);
  t.ys = hi16(a.w);
  t.fl = b.x & 0xFF;
  t.xd = b8(b.x, 1);
  t.vd = b8(b.x, 2);
  t.ch = lo16(b.y);
  t.m0 = hi16(b.y);
  t.mn = lo16(b.z);
  t.rd = b.w;
  return t;
}
// Per-draw eigensystem record: P(t) = m1 diag(exp(lam t)) m2, plus Q.
constexpr int EIG_LEN = 56;  // m1[16] lam[4] m2[16] Q[16] s (+pad)
constexpr int EIG_M1 = 0, EIG_LAM = 16, EIG_M2 = 20, EIG_Q = 36, EIG_S = 52;

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
// Field-wise copies: an aggregate copy becomes a 32-B memcpy, and memcpys
// on both sides of a branch get merged into one from a phi of the source
// addresses, which pins the arrays in scratch.  Copying fields keeps every
// V4 in registers.
struct V4 {
  double x, y, z, w;
  __host__ __device__ V4() = default;
  __host__ __device__ __forceinline__ V4(double a, double b, double c, double d) : x(a), y(b), z(c), w(d) {}
  __host__ __device__ __forceinline__ V4(const V4& o) : x(o.x), y(o.y), z(o.z), w(o.w) {}
  __host__ __device__ __forceinline__ V4& operator=(const V4& o) {
    x = o.x;
    y = o.y;
    z = o.z;
    w = o.w;
    return *this;
  }
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

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, WAVE);
  return v;
}

// Cross-lane moves on doubles (two 32-bit halves each).
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  // every lane has a valid source for the controls used here, so the old
  // value is dead: mov_dpp leaves it undefined (no zeroing v_mov per half)
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
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
  const uint8_t* tips;    // [S][Ppad/2] tip nibbles: record vector index, pattern 2j+1 in the high nibble
  const double* weights;  // [Ppad]   (0 on padding)
  const double* pmat;     // [draw][C][nmat][R][4]  matrix records, program-use order
  const double* model;    // [draw][10+2C]
  double2* scratch;       // [wg][nslots][K][2][C*64]  stored moved partials
  double2* dstk;          // [wg][ndeep][K][2][C*64]   deep-stack entries
  double* gslot;          // [wg][C][nmat][16]  dL/dP partial sums (per-wave store / atomic adds)
  double* sslot;          // [wg][C][8]
  double* site_ll;        // [draw][P] or null
  double* out;            // [draw][outlen]: dL/dP rows written in place when g_direct
  const int* mat_branch;  // [nmat] branch of matrix m
  const double* eig;      // [draw][EIG_LEN] (Q for the chain rule)
  double* inner;          // [draw][C][B] <G, Q P> when g_direct
  int S, P, Ppad, C, nsteps, nslots, ndeep, ndl, nblk, nmat, R, cap_m;  // ndl: deep entries in LDS
  int B, outlen, g_direct;  // g_direct: one workgroup per draw
  unsigned long long extra;  // tip masks of record vectors 4..R-1, 4 bits each
  int fin;  // g_direct and the finalize fits in LDS: the sweep writes the whole output row
  const double* blens;  // [draw][B] (fin)
  double* grows;        // dL/dP rows of draw d at grows + d * grows_stride (in `out`, or scratch when compact)
  long long grows_stride;
  // qfused (fin only): the Q-parameter chain rule (qgrad_kernel's work,
  // qgrad_body) runs after the finalize, in the same workgroup
  int qfused, kind;
};

// LDS carve (16-B aligned pieces), K columns per lane:
//   tips   S x 64K nibbles            record indices, shared by the C category waves
//   mats   C x cap_m x R x 4 doubles  wave c's chunk of matrix records
//   tail   per wave: ndl deep entries of K x 2 x 64 double2 (the deep
//          entries [0, ndl) kept in LDS), or K x 64 doubles when ndl = 0;
//          wave c's root-exchange slice (K x 64 doubles) sits at the start
//          of its own tail, whose deep entries are all free at the root
// tips: the block's nibbles, then the 0/1 state vectors of the 16 record
// indices (the t of dL/dP += r (x) t for a tip child: two LDS reads instead
// of unpacking and converting its mask bits per column)
__host__ __device__ inline size_t tip_nib_bytes(int S, int K) { return ((size_t)S * WAVE * K / 2 + 15) / 16 * 16; }
__host__ __device__ inline size_t tip_lds_bytes(int S, int K) { return tip_nib_bytes(S, K) + 16 * 4 * sizeof(double); }
__host__ __device__ inline size_t tail_doubles(int K, int ndl) {  // per wave
  return ndl > 0 ? (size_t)ndl * K * 2 * WAVE * 2 : (size_t)K * WAVE;
}
__host__ __device__ inline size_t lds_bytes(int S, int C, int R, int cap_m, int K, int ndl) {
  return tip_nib_bytes(S, K) + 16 * 4 * sizeof(double) + (size_t)C * cap_m * R * 32 +
         (size_t)C * tail_doubles(K, ndl) * 8;
}

// Buffer resource over a workgroup's scratch / deep-stack region: loads past
// num_records return zeros without touching memory, so operand prefetches
// are issued unconditionally (an unused operand gets an out-of-range offset)
// and the waitcnt pass never sees a load on only one side of a branch.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
  void* p = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)n, 0x00020000);
}
// One stored 4-vector: two 16-B halves `half` bytes apart (the wave-uniform
// `half` rides in the instruction's soffset: no per-lane add; an
// out-of-range `off` is out of range with or without it).  Every stored
// partial is read exactly once, so the loads are non-temporal (aux 2 = nt):
// measured +13% (fluA) / +3% (synthetic) over the default policy, with the
// stores left at the default (nt or sc1 stores measured no better).
constexpr int LOAD_NT = 2;
#ifndef PHY_STORE_AUX
#define PHY_STORE_AUX 0
#endif
constexpr int STORE_AUX = PHY_STORE_AUX;  // cache policy of the moved-partial stores (0: default)
constexpr uint32_t OOB = 0x40000000u;  // out-of-range offset part (regions are < 2^30 bytes, checked at plan time)
__device__ __forceinline__ V4 ld_v4(__amdgpu_buffer_rsrc_t srd, uint32_t off, uint32_t half) {
  const auto lo = __builtin_amdgcn_raw_buffer_load_b128(srd, off, 0, LOAD_NT);
  const auto hi = __builtin_amdgcn_raw_buffer_load_b128(srd, off, half, LOAD_NT);  // half in soffset
  V4 r;
  r.x = __hiloint2double((int)lo[1], (int)lo[0]);
  r.y = __hiloint2double((int)lo[3], (int)lo[2]);
  r.z = __hiloint2double((int)hi[1], (int)hi[0]);
  r.w = __hiloint2double((int)hi[3], (int)hi[2]);
  return r;
}

// One 4-vector stored as two 16-B halves `half` bytes apart (dropped by the
// buffer range check when `off` is out of range).
__device__ __forceinline__ void st_v4(__amdgpu_buffer_rsrc_t srd, uint32_t off, uint32_t half, const V4& v) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  const u4 lo = {(unsigned)__double2loint(v.x), (unsigned)__double2hiint(v.x), (unsigned)__double2loint(v.y),
                 (unsigned)__double2hiint(v.y)};
  const u4 hi = {(unsigned)__double2loint(v.z), (unsigned)__double2hiint(v.z), (unsigned)__double2loint(v.w),
                 (unsigned)__double2hiint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(lo, srd, off, 0, STORE_AUX);
  __builtin_amdgcn_raw_buffer_store_b128(hi, srd, off, half, STORE_AUX);
}

// s_waitcnt vmcnt(0) that the compiler's waitcnt pass sees (an inline-asm
// wait would be invisible to it): clears loads left pending by staging
// loops so the step loops are not charged a loop-carried vmcnt(0).
#define WAIT_VMCNT0() __builtin_amdgcn_s_waitcnt(0x0F70)

// Matrix records (pmat_kernel): R 4-vectors per matrix -- the four columns
// of P, then P t for every non-one-hot tip mask t present in the data (the
// reference's tips are one-hot or all-ones, phylostan/utils.py:180-187).
// A tip child's moved partial P t is therefore one indexed LDS read.
//   P v   = sum_j col_j v_j   (row i: P_i0 v0 + P_i1 v1 + P_i2 v2 + P_i3 v3)
//   P^T v = (col_j . v)_j
// K products share one read of the (wave-uniform: LDS broadcast) columns.
template <int K>
__device__ __forceinline__ void pvec_k(const double* __restrict__ M, const V4 (&v)[K], V4 (&r)[K]) {
  const double2 a01 = *reinterpret_cast<const double2*>(M + 0), a23 = *reinterpret_cast<const double2*>(M + 2);
  const double2 b01 = *reinterpret_cast<const double2*>(M + 4), b23 = *reinterpret_cast<const double2*>(M + 6);
  const double2 c01 = *reinterpret_cast<const double2*>(M + 8), c23 = *reinterpret_cast<const double2*>(M + 10);
  const double2 d01 = *reinterpret_cast<const double2*>(M + 12), d23 = *reinterpret_cast<const double2*>(M + 14);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const V4 x = v[k];
    r[k].x = fma(d01.x, x.w, fma(c01.x, x.z, fma(b01.x, x.y, a01.x * x.x)));
    r[k].y = fma(d01.y, x.w, fma(c01.y, x.z, fma(b01.y, x.y, a01.y * x.x)));
    r[k].z = fma(d23.x, x.w, fma(c23.x, x.z, fma(b23.x, x.y, a23.x * x.x)));
    r[k].w = fma(d23.y, x.w, fma(c23.y, x.z, fma(b23.y, x.y, a23.y * x.x)));
  }
}
template <int K>
__device__ __forceinline__ void ptvec_k(const double* __restrict__ M, const V4 (&v)[K], V4 (&r)[K]) {
  const double2 a01 = *reinterpret_cast<const double2*>(M + 0), a23 = *reinterpret_cast<const double2*>(M + 2);
  const double2 b01 = *reinterpret_cast<const double2*>(M + 4), b23 = *reinterpret_cast<const double2*>(M + 6);
  const double2 c01 = *reinterpret_cast<const double2*>(M + 8), c23 = *reinterpret_cast<const double2*>(M + 10);
  const double2 d01 = *reinterpret_cast<const double2*>(M + 12), d23 = *reinterpret_cast<const double2*>(M + 14);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const V4 x = v[k];
    r[k].x = fma(a23.y, x.w, fma(a23.x, x.z, fma(a01.y, x.y, a01.x * x.x)));
    r[k].y = fma(b23.y, x.w, fma(b23.x, x.z, fma(b01.y, x.y, b01.x * x.x)));
    r[k].z = fma(c23.y, x.w, fma(c23.x, x.z, fma(c01.y, x.y, c01.x * x.x)));
    r[k].w = fma(d23.y, x.w, fma(d23.x, x.z, fma(d01.y, x.y, d01.x * x.x)));
  }
}

// 0/1 state vector of a tip's record index b: the one-hot columns 0..3, then
// the extra masks (4 bits each in `extra`).
__device__ __forceinline__ V4 tipvec_b(unsigned b, unsigned long long extra) {
  const unsigned m = b < 4 ? (1u << b) : (unsigned)(extra >> (4 * (b - 4))) & 15u;
  return {(double)(m & 1u), (double)((m >> 1) & 1u), (double)((m >> 2) & 1u), (double)((m >> 3) & 1u)};
}
// The same, from the sweep's LDS table.
__device__ __forceinline__ V4 tipvec_l(const double* tvec, unsigned b) {
  const double2 lo = *reinterpret_cast<const double2*>(tvec + (b & 15u) * 4);
  const double2 hi = *reinterpret_cast<const double2*>(tvec + (b & 15u) * 4 + 2);
  return {lo.x, lo.y, hi.x, hi.y};
}

// One matrix record (R 4-vectors): the four columns of P(t), then P t for
// every extra tip mask (pmat_kernel).  Building the records inside the sweep
// instead (verdict item 4c) was measured: the extra code in the chunk
// staging path pushed the K=2 kernel into scratch spills and cost 7 % even
// when unused, 11 % when used (fluA 6.67 ms against 6.0).
//   e: the draw's eigensystem record (EIG_LEN doubles), t = r_c b.
__device__ __forceinline__ void build_record(const double* __restrict__ e, double t, int kind, int R,
                                             unsigned long long extra, double2* po) {
  double P[16];
  if (kind == PHY_JC69) {  // generate_script.py:765-769
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
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // column j
    po[2 * j] = make_double2(P[j], P[4 + j]);
    po[2 * j + 1] = make_double2(P[8 + j], P[12 + j]);
  }
  for (int v = 4; v < R; ++v) {
    const unsigned tm = (unsigned)(extra >> (4 * (v - 4))) & 15u;
    double r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      double acc = P[i * 4] * (double)(tm & 1u);
#pragma unroll
      for (int j = 1; j < 4; ++j) acc = fma(P[i * 4 + j], (double)((tm >> j) & 1u), acc);
      r[i] = acc;
    }
    po[2 * v] = make_double2(r[0], r[1]);
    po[2 * v + 1] = make_double2(r[2], r[3]);
  }
}

// dlogL / d(exchangeabilities[6], freqs[4]) through the eigendecomposition:
// the device form of models.q_param_gradients_batch (Q = V diag(lam) V^-1,
// V = m1 = Pi^-1/2 U, V^-1 = m2 = U^T Pi^1/2, t = r_c b):
//   H_cb = V^T G_cb V^-T,  Phi_cb[k][l] = (e^{lam_k t} - e^{lam_l t}) / (lam_k - lam_l)
//   (t e^{lam_k t} on ties),  M = sum_cb H_cb .* Phi_cb,  W = V^-T M V^T,
//   qw = <Q, W>,  s = the normaliser of Q (generate_script.py:862-868);
//   rate (i,j): (f_j W_ij + f_i W_ji - f_j W_ii - f_i W_jj - 2 f_i f_j qw) / s
//   freq m:     (sum_{j != m} R_jm (W_jm - W_jj) - qw sum_{j != m} 2 R_mj f_j) / s
//               + the explicit root term.
// One workgroup per draw; per-thread partial M over (c, b) (the per-draw
// V, V^-1, lambda and 1/(lambda_k - lambda_l) in LDS, so a thread holds only
// M, G and one row of V^T G: ~100 VGPRs instead of 200, twice the resident
// waves), a wave reduction of the 16 partials, then the waves in order:
// deterministic.  JC69 has no Q parameters: zeros.
// qgrad_body: the work of a QG_THREADS-thread workgroup (QG_THREADS / 64
// "virtual" waves; a smaller workgroup runs them in turn), so qgrad_kernel
// and the sweep's fused epilogue give the same bits;
// every thread of the workgroup must call it (it holds barriers).
// sh: QG_SHARED doubles of LDS.
struct QgArgs {
  const double* eig;    // [draw][EIG_LEN]
  const double* model;  // [draw][10+2C]
  const double* blens;  // [draw][B]
  const double* grows;  // dL/dP rows of draw d at grows + d * grows_stride
  long long grows_stride;
  double* out;          // [draw][outlen]
  int outlen, C, B, kind;
};
constexpr int QG_THREADS = 1024;  // 256 (c, b) quads per pass (the synthetic config: 1016 in 4 passes, not 16)
constexpr int QG_SHARED = 16 * 3 + 4 + (QG_THREADS / 64) * 16 + 16 * 2;  // V, V^-1, 1/(lam_k - lam_l), lam,
                                                                          // wave partials, M, W
// Row k of the (c, b) item's dL/dP block G (row-major 4x4) for lane k of the
// item's quad in qgrad_body (the other rows come by quad broadcast): by
// default from the draw's dL/dP row.
struct RowsG {
  const double* rows;
  __device__ __forceinline__ void operator()(int idx, int k, double (&g)[4]) const {
    const double2* g2 = reinterpret_cast<const double2*>(rows + (size_t)idx * 16 + k * 4);
    const double2 lo = g2[0], hi = g2[1];
    g[0] = lo.x;
    g[1] = lo.y;
    g[2] = hi.x;
    g[3] = hi.y;
  }
};
// The Q-parameter tail every epilogue ends with (one thread): from
// W = V^-T M V^T the exchangeability gradients oq[4..9] and the frequency
// gradients oq[10..13] (plus the root-frequency term rt[0..3]) through
// Q = S^-1 R diag(f) with S the normaliser (generate_script.py's GTR / HKY
// rate matrix; models.q_param_gradients is the host statement).
__device__ void q_tail(const double (&W)[16], const double* Q, double sn, const double* mdl, const double* rt,
                       double* oq) {
  double qw = 0.0;
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) qw = fma(Q[kk], W[kk], qw);
  const double f[4] = {mdl[0], mdl[1], mdl[2], mdl[3]};
  const double* r = mdl + 4;  // AC AG AT CG CT GT
  const int pi_[6] = {0, 0, 0, 1, 1, 2}, pj_[6] = {1, 2, 3, 2, 3, 3};
  double Rm[16];
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) Rm[kk] = 0.0;
#pragma unroll
  for (int kk = 0; kk < 6; ++kk) {
    const int i = pi_[kk], j = pj_[kk];
    Rm[i * 4 + j] = Rm[j * 4 + i] = r[kk];
    const double dq = f[j] * W[i * 4 + j] + f[i] * W[j * 4 + i] - f[j] * W[i * 4 + i] - f[i] * W[j * 4 + j];
    oq[4 + kk] = (dq - 2.0 * f[i] * f[j] * qw) / sn;
  }
#pragma unroll
  for (int mm = 0; mm < 4; ++mm) {
    double dq = 0.0, ds = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j != mm) {
        dq += Rm[j * 4 + mm] * (W[j * 4 + mm] - W[j * 4 + j]);
        ds += 2.0 * Rm[mm * 4 + j] * f[j];
      }
    oq[10 + mm] = (dq - ds * qw) / sn + rt[mm];
  }
}

// W = V^-T M V^T, entry t = (i, j) (every epilogue's order)
__device__ __forceinline__ double w_entry(const double* M, const double* V, const double* Vi, int t) {
  const int i = t >> 2, j = t & 3;
  double acc = 0.0;
  for (int kk = 0; kk < 4; ++kk) {
    double ml = 0.0;
    for (int l = 0; l < 4; ++l) ml = fma(M[kk * 4 + l], V[j * 4 + l], ml);
    acc = fma(Vi[kk * 4 + i], ml, acc);
  }
  return acc;
}

template <typename GP>
__device__ void qgrad_body(const QgArgs& a, int draw, int tid, double* sh, const GP& getG);
__device__ __forceinline__ void qgrad_body(const QgArgs& a, int draw, int tid, double* sh) {
  qgrad_body(a, draw, tid, sh, RowsG{a.grows + (size_t)draw * a.grows_stride});
}
template <typename GP>
__device__ void qgrad_body(const QgArgs& a, int draw, int tid, double* sh, const GP& getG) {
  double* sV = sh;
  double* sVi = sh + 16;
  double* srinv = sh + 32;
  double* slam = sh + 48;
  double* part = sh + 52;  // [QG_THREADS / 64][16]
  double* sM = part + (QG_THREADS / 64) * 16;
  double* sW = sM + 16;
  const int lane = tid & 63, wave = tid >> 6;
  const int nwr = max(1, (int)(blockDim.x >> 6));  // the workgroup's waves
  const int C = a.C, B = a.B;
  double* out = a.out + (size_t)draw * a.outlen;
  const int o = 1 + B + 2 * C;
  if (a.kind == PHY_JC69) {  // workgroup-uniform
    if (tid < 10) out[o + 4 + tid] = 0.0;
    return;
  }
  const double* e = a.eig + (size_t)draw * EIG_LEN;
  if (tid < 16) {
    sV[tid] = e[EIG_M1 + tid];
    sVi[tid] = e[EIG_M2 + tid];
    // 1 / (lam_k - lam_l) once per draw (0 marks a tie: t e^{lam_k t} there)
    const double lk = e[EIG_LAM + (tid >> 2)], ll = e[EIG_LAM + (tid & 3)];
    const double d = lk - ll;
    srinv[tid] = fabs(d) < 1e-12 * fmax(1.0, fabs(lk)) ? 0.0 : 1.0 / d;
    if (tid < 4) slam[tid] = e[EIG_LAM + tid];
  }
  __syncthreads();
  const double* mdl = a.model + (size_t)draw * (10 + 2 * C);
  const double* bl = a.blens + (size_t)draw * B;
  // a quad of lanes per (c, b): lane k forms row k of H = V^T G V^-T and
  // accumulates row k of M (4 values); e^{lam_k t} comes from lane k
  const int k = tid & 3;
  for (int vw = wave; vw < QG_THREADS / 64; vw += nwr) {  // virtual wave vw: threads vw*64 + lane
    const int vt = vw * 64 + lane;
    double m[4] = {0.0, 0.0, 0.0, 0.0};
    // two items per trip, their loads and exps side by side (the
    // accumulation stays in item order: the same bits as one at a time)
    constexpr int QS = QG_THREADS / 4;
    for (int idx = vt >> 2; idx < C * B; idx += 2 * QS) {
      const bool two = idx + QS < C * B;  // (quad-uniform)
      double t2[2], Ek2[2], g2[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ix = h && two ? idx + QS : idx;
        const int c = ix / B, b = ix - c * B;
        t2[h] = mdl[10 + c] * bl[b];
        getG(ix, k, g2[h]);  // row k of G; G[i][j] = row i's g[j], broadcast from lane i of the quad
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) Ek2[h] = exp(slam[k] * t2[h]);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h && !two) break;
        const double t = t2[h], Ek = Ek2[h];
        const double(&g)[4] = g2[h];
        double E[4];
        E[0] = dpp_d<0x00>(Ek);
        E[1] = dpp_d<0x55>(Ek);
        E[2] = dpp_d<0xAA>(Ek);
        E[3] = dpp_d<0xFF>(Ek);
        double T[4];  // row k of V^T G
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const double g0 = dpp_d<0x00>(g[j]), g1 = dpp_d<0x55>(g[j]), gg2 = dpp_d<0xAA>(g[j]),
                       g3 = dpp_d<0xFF>(g[j]);
          T[j] = fma(sV[12 + k], g3, fma(sV[8 + k], gg2, fma(sV[4 + k], g1, fma(sV[k], g0, 0.0))));
        }
#pragma unroll
        for (int l = 0; l < 4; ++l) {
          double hh = 0.0;  // (V^T G V^-T)[k][l]
#pragma unroll
          for (int j = 0; j < 4; ++j) hh = fma(T[j], sVi[l * 4 + j], hh);
          const double ri = srinv[k * 4 + l];
          const double phi = ri == 0.0 ? t * Ek : (Ek - E[l]) * ri;
          m[l] = fma(hh, phi, m[l]);
        }
      }
    }
    // sum over the wave's 16 quads (lane bits 2..5): lanes with bits 2, 3
    // clear end with M[k][2 b5 + b4]
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      swap32(m[u], m[u + 2]);
      m[u] += m[u + 2];
    }
    swap16(m[0], m[1]);
    m[0] += m[1];
    m[0] += dpp_d<DPP_ROW_ROR8>(m[0]);
    m[0] += dpp_d<0x124>(m[0]);  // row_ror:4 (symmetric after the ror:8 stage)
    if ((lane & 12) == 0) part[vw * 16 + k * 4 + ((lane >> 5) & 1) * 2 + ((lane >> 4) & 1)] = m[0];
  }
  __syncthreads();
  // M = the waves' partials in order; W = V^-T M V^T, one entry per thread:
  // W[i][j] = sum_kl Vi[k][i] M[k][l] V[j][l]
  if (tid < 16) {
    double acc = part[tid];
    for (int w = 1; w < QG_THREADS / 64; ++w) acc += part[w * 16 + tid];
    sM[tid] = acc;
  }
  __syncthreads();
  if (tid < 16) sW[tid] = w_entry(sM, sV, sVi, tid);
  __syncthreads();
  if (tid != 0) return;
  double W[16];
  for (int kk = 0; kk < 16; ++kk) W[kk] = sW[kk];
  q_tail(W, e + EIG_Q, e[EIG_S], mdl, out + o, out + o);
}

// The sweep.  `prog` is a separate __restrict__ const argument so the
// backend proves it read-only and uses scalar loads.
//
// K columns per lane: lane l of the category-c wave owns patterns
// blk*64K + k*64 + l, k < K.  The columns share every matrix read, the
// program control flow and -- the main saving -- one wave reduction of the
// summed outer products per branch.
//
// Stack discipline of the post-order program (build_program): the operand a
// step pops is the previous step's result (`top`, in registers) except for
// the first child x of a node whose children are both internal; those live
// on a small per-workgroup "deep stack" in global memory (L2-resident),
// at entries the host assigns statically, and are prefetched one step ahead.
// The reverse pass mirrors this for the upper partials r.  No LDS stack:
// LDS holds only tips, the root exchange and the matrix chunks.
//
// Register budget: K=2 targets two waves per SIMD (<= 256 VGPRs), K=1 four.
// DL: the deep stack lives in LDS (no VMEM traffic or prefetch for it),
// else in the per-workgroup global region behind a buffer descriptor.
#ifdef PHY_STEPTIME
// Diagnostic build only (tools/steptime.py): the shader clock (s_memtime) of
// lane 0 of every category wave of draws [TT_DRAW0, TT_DRAW0 + TT_DRAWS) at
// each program step and phase boundary, one slot per event.
#ifndef TT_DRAW0
#define TT_DRAW0 0
#endif
constexpr int TT_DRAWS = 64, TT_EV = 1024;
__device__ unsigned long long g_tt[TT_DRAWS * 16][TT_EV];
#define TT_MARK(i)                                                                   \
  do {                                                                               \
    if (draw >= TT_DRAW0 && draw < TT_DRAW0 + TT_DRAWS && lane == 0)                 \
      g_tt[(draw - TT_DRAW0) * 16 + wv][(i)] = __builtin_amdgcn_s_memtime();         \
  } while (0)
#else
#define TT_MARK(i) do {} while (0)
#endif
#ifndef PHY_WPE2
#define PHY_WPE2 2  // waves per SIMD the K=2 kernel is register-budgeted for
#endif
template <int MAXT, int K, bool DL>
__global__ void __launch_bounds__(MAXT) __attribute__((amdgpu_waves_per_eu(MAXT <= 512 ? PHY_WPE2 : 4)))
    sweep_kernel(SweepArgs a, const int* __restrict__ prog) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  const int lane = threadIdx.x & (WAVE - 1);
  const int C = a.C, nsteps = a.nsteps, nmat = a.nmat;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = wv;  // category
  const int nthreads = blockDim.x;
  const int draw = blockIdx.y;
  const int wg = blockIdx.y * gridDim.x + blockIdx.x;
  const int rec = a.R * 4;  // doubles per matrix record
  const int ncolwg = C * WAVE;

  unsigned char* tipl = lds_raw;  // the block's tips
  double* tvec = reinterpret_cast<double*>(lds_raw + tip_nib_bytes(a.S, K));  // [16][4]
  double* mats0 = tvec + 64;
  if (threadIdx.x < 64) {  // published by the block loop's first barrier
    const unsigned b = threadIdx.x >> 2, j = threadIdx.x & 3;
    const unsigned m = b < 4 ? (1u << b) : (unsigned)(a.extra >> (4 * (b - 4))) & 15u;
    tvec[threadIdx.x] = (double)((m >> j) & 1u);
  }
  double* mats = mats0 + (size_t)c * a.cap_m * rec;
  const int ndl = DL ? a.ndeep : a.ndl;  // deep entries [0, ndl) live in LDS
  double* tail0 = mats0 + (size_t)C * a.cap_m * rec;
  const size_t tstride = tail_doubles(K, ndl);

  const double* mdl = a.model + (size_t)draw * (10 + 2 * C);
  const V4 pi = {mdl[0], mdl[1], mdl[2], mdl[3]};
  const double ps_c = mdl[10 + C + c];
  const double* pmat_c = a.pmat + ((size_t)draw * C + c) * nmat * rec;
  const size_t entry2 = (size_t)K * 2 * ncolwg;  // double2 per scratch / deep-stack entry
  double2* scr = a.scratch + (size_t)wg * a.nslots * entry2;
  double2* dsk = a.dstk + (size_t)wg * a.ndeep * entry2;
  const uint32_t scr_bytes = (uint32_t)((size_t)a.nslots * entry2 * 16);
  const uint32_t dsk_bytes = (uint32_t)((size_t)a.ndeep * entry2 * 16);
  const __amdgpu_buffer_rsrc_t srd_scr = make_rsrc(scr, scr_bytes);
  const __amdgpu_buffer_rsrc_t srd_dsk = make_rsrc(dsk, dsk_bytes);
  const int colw = c * WAVE + lane;  // this lane's column inside an entry half
  const uint32_t half_bytes = (uint32_t)ncolwg * 16u;
  // Byte offset of (entry e, column k), half 0 = a per-lane column part plus
  // the wave-uniform e * estr.  An operand that is not loaded gets the
  // uniform part OOB instead (>= every region's size, so the sum is out of
  // range and the load returns zeros): the choice is one scalar select, no
  // per-lane select or exec masking.
  const uint32_t estr = (uint32_t)(K * 2 * ncolwg * 16);
  uint32_t lcol[K];  // this lane's column part
#pragma unroll
  for (int k = 0; k < K; ++k) lcol[k] = (uint32_t)((k * 2 * ncolwg + colw) * 16);
  auto ent = [&](bool use, int e) __attribute__((always_inline)) -> uint32_t {  // uniform part
    return use ? (uint32_t)e * estr : OOB;
  };
  // Scratch offsets of this lane's live columns only: padding columns
  // (pattern >= P) get the column part OOB, so they neither store nor load
  // moved partials -- the range check drops their stores and zero-fills
  // their loads, so they stay finite and their weight-0 upper partials are
  // exactly zero.
  uint32_t lofs[K];  // per block: lcol[k], or OOB on a padding column
  auto soff = [&](int e, int k) __attribute__((always_inline)) -> uint32_t {
    return lofs[k] + (uint32_t)e * estr;
  };
  auto put = [&](double2* base, int e, int k, const V4& v) __attribute__((always_inline)) {
    double2* d = base + ((size_t)e * K + k) * 2 * ncolwg + colw;
    d[0] = make_double2(v.x, v.y);
    d[ncolwg] = make_double2(v.z, v.w);
  };
  // this wave's LDS deep entries: ndl x K x 2 halves x 64 double2
  double2* dlw = reinterpret_cast<double2*>(tail0 + (size_t)wv * tstride);
  auto dput = [&](int e, int k, const V4& v) __attribute__((always_inline)) {
    double2* d = dlw + (size_t)(e * K + k) * 2 * WAVE + lane;
    d[0] = make_double2(v.x, v.y);
    d[WAVE] = make_double2(v.z, v.w);
  };
  auto dget = [&](int e, int k) __attribute__((always_inline)) -> V4 {
    const double2* d = dlw + (size_t)(e * K + k) * 2 * WAVE + lane;
    const double2 lo = d[0], hi = d[WAVE];
    return V4(lo.x, lo.y, hi.x, hi.y);
  };

  // this wave's dL/dP slot: a plain store per (branch, entry) in the
  // workgroup's first block, then one atomic add per later block, all from
  // this wave only -- same-address program order, so the sums are bitwise
  // reproducible and the slot needs no zeroing
  double* gs = a.gslot + ((size_t)wg * C + c) * nmat * 16;
  bool gfirst = true;  // wave-uniform

  const int e = reduce16_entry(lane);
  const bool gowner = (lane & 3) == 0;

  double acc_ll = 0.0, acc_dps = 0.0;
  V4 acc_f = {0.0, 0.0, 0.0, 0.0};

  // ---- this wave's chunk of matrix records in LDS (no barrier: private) ----
  int cur = -1, m0 = 0;
  auto ensure_chunk = [&](const Step& st) {
    const int ch = st.ch;
    if (ch == cur) return;  // wave-uniform
    const int lo = st.m0, n = st.mn;
    const double2* src = reinterpret_cast<const double2*>(pmat_c + (size_t)lo * rec);
    double2* dst = reinterpret_cast<double2*>(mats);
    const int q2 = n * rec / 2;
    for (int k0 = lane; k0 < q2; k0 += WAVE * 8) {
      double2 buf[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u * WAVE;
        buf[u] = (k < q2) ? src[k] : make_double2(0.0, 0.0);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u * WAVE;
        if (k < q2) dst[k] = buf[u];
      }
    }
    WAIT_VMCNT0();  // no staging load may look pending inside the step loops
    cur = ch;
    m0 = lo;
  };
  auto mrec = [&](int m) __attribute__((always_inline)) -> const double* { return mats + (size_t)(m - m0) * rec; };
  // record index of tip t, column k: a nibble (two lanes share a byte)
  auto tipb = [&](int t, int k) __attribute__((always_inline)) -> unsigned {
    return (tipl[(t * K + k) * (WAVE / 2) + (lane >> 1)] >> ((lane & 1) * 4)) & 15u;
  };
  auto look = [&](int m, unsigned b) __attribute__((always_inline)) -> V4 {  // P t of a tip: one record vector
    const double* p = mrec(m) + (b & 15u) * 4;
    const double2 lo = *reinterpret_cast<const double2*>(p);
    const double2 hi = *reinterpret_cast<const double2*>(p + 2);
    return {lo.x, lo.y, hi.x, hi.y};
  };
  // dL/dP_m += sum_k r_k (x) p_k, reduced over the wave; the lane owning
  // entry e adds it to this wave's slot.
  auto gacc = [&](int m, const V4 (&r)[K], const V4 (&p)[K]) __attribute__((always_inline)) {
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
    const double sum = reduce16(v, lane);
    if (gowner) {
      if (gfirst)
        gs[(size_t)m * 16 + e] = sum;
      else
        unsafeAtomicAdd(gs + (size_t)m * 16 + e, sum);
    }
  };

  // blocks: the workgroup takes blocks blockIdx.x, + gridDim.x, ... of its
  // draw (the launch keeps gridDim.x <= nblk: every workgroup has a block)
  const int VG = gridDim.x, vg = blockIdx.x;
  const int trips = (a.nblk - vg + VG - 1) / VG;
  for (int trip = 0; trip < trips; ++trip) {
    const int blk = vg + trip * VG;
    TT_MARK(trip * 320 + 0);
#pragma unroll
    for (int k = 0; k < K; ++k) lofs[k] = (blk * WAVE * K + k * WAVE + lane < a.P) ? lcol[k] : OOB;
    __syncthreads();  // the previous block's tip / root-exchange reads are done
    // stage this block's tip bytes in LDS: S rows x 64K bytes, shared by the
    // C category-waves and by both passes (8 loads in flight per thread)
    {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(a.tips);
      uint32_t* dst = reinterpret_cast<uint32_t*>(tipl);
      const int rowq = a.Ppad / 8;
      constexpr int wq = WAVE * K / 8;  // words per tip row of this block
      const int nq = a.S * wq;
      const int nthr = C * WAVE, t0 = c * WAVE + lane;
      for (int k0 = t0; k0 < nq; k0 += nthr * 8) {
        uint32_t buf[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = k0 + u * nthr;
          buf[u] = (k < nq) ? src[(size_t)(k / wq) * rowq + blk * wq + (k % wq)] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = k0 + u * nthr;
          if (k < nq) dst[k] = buf[u];
        }
      }
    }
    __syncthreads();
    WAIT_VMCNT0();
    TT_MARK(trip * 320 + 1);

    // ------------------------------ forward ------------------------------
    // Step s: a_y = P t_y (tip) or top; a_x = P t_x (tip), top (y a tip) or
    // the deep operand; p_v = a_x * a_y; a_v = P_v p_v -> scratch slot (and
    // the deep stack when v is a deep x child); top = a_v.
    V4 top[K], proot[K];
#pragma unroll
    for (int k = 0; k < K; ++k) top[k] = proot[k] = {0.0, 0.0, 0.0, 0.0};
    // dcur: this step's deep operand (loaded one step ahead into dnext,
    // alternating by name across an unrolled pair of steps: no register
    // copy of an in-flight load)
    #define FSTEP(s, dcur, dnext, st, sn) do {                                            \
      {                                                                                   \
        const bool more = s + 1 < nsteps;                                                 \
        sn = ld_step<K == 2>(prog, more ? s + 1 : s); /* next step's record, a step ahead */      \
        /* an x operand whose deep entry is global is read back from x's scratch slot */  \
        const bool need = more && (sn.fl & F_XDEEP) && sn.xd >= ndl;                      \
        if (!DL)                                                                                                      \
      _Pragma("unroll")                                                                                               \
        for (int k = 0; k < K; ++k) dnext[k] = ld_v4(srd_scr, lofs[k] + ent(need, sn.xs), half_bytes);         \
      }                                                                                                               \
      ensure_chunk(st);                                                                                               \
      const int x = st.x, y = st.y, fl = st.fl, vs = st.vs;                        \
      V4 ax[K], ay[K], pv[K];                                                                                         \
      if (y >= 0) {                                                                                                   \
        const int my = st.my;                                                                                     \
      _Pragma("unroll")                                                                                               \
        for (int k = 0; k < K; ++k) ay[k] = look(my, tipb(y, k));                                                     \
      } else {                                                                                                        \
      _Pragma("unroll")                                                                                               \
        for (int k = 0; k < K; ++k) ay[k] = top[k];                                                                   \
      }                                                                                                               \
      if (x >= 0) {                                                                                                   \
        const int mx = st.mx;                                                                                     \
      _Pragma("unroll")                                                                                               \
        for (int k = 0; k < K; ++k) ax[k] = look(mx, tipb(x, k));                                                     \
      } else if (y >= 0) {                                                                                            \
      _Pragma("unroll")                                                                                               \
        for (int k = 0; k < K; ++k) ax[k] = top[k];                                                                   \
      } else {                                                                                                        \
        {                                                                                                             \
          const int xd = st.xd;                                                                                \
          if (DL || xd < ndl) {                                                                                       \
      _Pragma("unroll")                                                                                               \
            for (int k = 0; k < K; ++k) ax[k] = dget(xd, k);                                                          \
          } else {                                                                                                    \
      _Pragma("unroll")                                                                                               \
            for (int k = 0; k < K; ++k) ax[k] = dcur[k];                                                              \
          }                                                                                                           \
        }                                                                                                             \
      }                                                                                                               \
      _Pragma("unroll")                                                                                               \
      for (int k = 0; k < K; ++k) pv[k] = vmul(ax[k], ay[k]);                                                         \
      if (vs >= 0) {                                                                                                  \
        V4 av[K];                                                                                                     \
        if (fl & F_MV) {                                                                                              \
          pvec_k<K>(mrec(st.mv), pv, av);                                                                         \
        } else { /* merged root branch of an unrooted tree: identity */                                                \
      _Pragma("unroll")                                                                                               \
          for (int k = 0; k < K; ++k) av[k] = pv[k];                                                                  \
        }                                                                                                             \
      _Pragma("unroll")                                                                                               \
        for (int k = 0; k < K; ++k) if (!(fl & F_NOSTORE)) st_v4(srd_scr, soff(vs, k), half_bytes, av[k]);                                    \
        if (fl & F_VDEEP) {                                                                                           \
          const int dp = st.vd;                                                                                \
          if (DL || dp < ndl)  /* a global entry is x's scratch slot itself */                                        \
          for (int k = 0; k < K; ++k) dput(dp, k, av[k]);                                                             \
        }                                                                                                             \
      _Pragma("unroll")                                                                                               \
        for (int k = 0; k < K; ++k) top[k] = av[k];                                                                   \
      } else {                                                                                                        \
      _Pragma("unroll")                                                                                               \
        for (int k = 0; k < K; ++k) proot[k] = pv[k];                                                                 \
      }                                                                                                               \
    } while (0)
    {
      V4 dA[K], dB[K];
#pragma unroll
      for (int k = 0; k < K; ++k) dA[k] = {0.0, 0.0, 0.0, 0.0};  // step 0 has no internal child
      Step sA = ld_step<K == 2>(prog, 0), sB;
      for (int s = 0;;) {
        TT_MARK(trip * 320 + 2 + s);
        FSTEP(s, dA, dB, sA, sB);
        if (++s >= nsteps) break;
        TT_MARK(trip * 320 + 2 + s);
        FSTEP(s, dB, dA, sB, sA);
        if (++s >= nsteps) break;
      }
    }
    TT_MARK(trip * 320 + 152);

    // ------------------------- root / site log L -------------------------
    // (the C category waves exchange through their tails)
    double fp[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      fp[k] = vdot(pi, proot[k]);  // pi . p_root,c
      tail0[(size_t)wv * tstride + k * WAVE + lane] = ps_c * fp[k];
    }
    __syncthreads();
    double L[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      L[k] = 0.0;
      for (int cc = 0; cc < C; ++cc) L[k] += tail0[(size_t)cc * tstride + k * WAVE + lane];
    }
    __syncthreads();  // every wave has read the exchange before deep entries are rewritten
    TT_MARK(trip * 320 + 153);
    V4 topr[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = blk * WAVE * K + k * WAVE + lane;  // pattern of this column
      const bool live = i < a.P;  // padding columns contribute exactly nothing
      const double wt = a.weights[i];
      const double lnL = live ? log(L[k]) : 0.0;
      if (c == 0) {
        acc_ll += wt * lnL;
        if (a.site_ll != nullptr && live) a.site_ll[(size_t)draw * a.P + i] = lnL;
      }
      const double sc = live ? wt / L[k] : 0.0;
      const double s_c = sc * ps_c;
      acc_dps = fma(sc, fp[k], acc_dps);
      acc_f.x = fma(s_c, proot[k].x, acc_f.x);
      acc_f.y = fma(s_c, proot[k].y, acc_f.y);
      acc_f.z = fma(s_c, proot[k].z, acc_f.z);
      acc_f.w = fma(s_c, proot[k].w, acc_f.w);
      // upper partials are carried pre-scaled by w_i ps_c / L_i, so every
      // outer product below is already a dlogL/dP term
      topr[k] = vscale(pi, s_c);
    }

    // ------------------------------ reverse ------------------------------
    // Step s (program backwards) with upper partial r_v (top, or the deep
    // stack when v is a deep x child): q_v = P_v^T r_v, r_x = q_v * a_y,
    // r_y = q_v * a_x, dL/dP_v += r_v (x) (a_x * a_y), and for tip children
    // dL/dP += r (x) t.  Children's stored a come back from scratch, loaded
    // one step ahead (zeros for tips: out-of-range offset).
    struct CSet {
      V4 lx[K], ly[K], lr[K];
      Step st;  // the step's record, loaded with its operands
    };
    #define LOAD_SET(s, r) do {                                                  \
      const bool ok = s >= 0;                                                    \
      r.st = ld_step<K == 2>(prog, ok ? s : 0);                                   \
      const int x = r.st.x, y = r.st.y, fl = r.st.fl;                     \
      /* a rebuilt cherry (F_PREVREC) is the previous-step child: y when y is       \
         internal, else x -- its operand is not loaded */                           \
      const bool rec_ = fl & F_PREVREC;                 \
      const bool lx = ok && x < 0 && !(rec_ && y >= 0), ly = ok && y < 0 && !rec_;  \
      const bool lr = ok && (fl & F_VDEEP) && r.st.vd >= ndl;             \
      const int xs = r.st.xs, ys = r.st.ys, vd = r.st.vd;                 \
      _Pragma("unroll")                                                          \
      for (int k = 0; k < K; ++k) {                                              \
        r.lx[k] = ld_v4(srd_scr, lofs[k] + ent(lx, xs), half_bytes);             \
        r.ly[k] = ld_v4(srd_scr, lofs[k] + ent(ly, ys), half_bytes);             \
        if constexpr (!DL)                                                       \
          r.lr[k] = ld_v4(srd_dsk, lcol[k] + ent(lr, vd), half_bytes);            \
      }                                                                          \
    } while (0)
    #define REBUILD(cst, out) do { /* a_c of a cherry c from LDS, as its forward step formed it */  \
      V4 p_[K];                                                                                     \
      _Pragma("unroll")                                                                             \
      for (int k = 0; k < K; ++k)                                                                   \
        p_[k] = vmul(look(cst.mx, tipb(cst.x, k)), look(cst.my, tipb(cst.y, k)));                   \
      pvec_k<K>(mrec(cst.mv), p_, out);                                                             \
    } while (0)
    /* one level up a rebuilt chain: a_v of v (one tip child, the other the
       rebuilt a_in), in the forward's operand order */
    #define CHAIN_UP(vst, in, out) do {                                                   \
      V4 pu_[K];                                                                          \
      if (vst.x >= 0) {                                                                   \
      _Pragma("unroll")                                                                   \
        for (int k = 0; k < K; ++k) pu_[k] = vmul(look(vst.mx, tipb(vst.x, k)), in[k]);   \
      } else {                                                                            \
      _Pragma("unroll")                                                                   \
        for (int k = 0; k < K; ++k) pu_[k] = vmul(in[k], look(vst.my, tipb(vst.y, k)));  \
      }                                                                                   \
      pvec_k<K>(mrec(vst.mv), pu_, out);                                                  \
    } while (0)
    /* the previous-step child of step s, rebuilt from the chain of depth d
       below it: its cherry at step s-d, then one-tip nodes up to vst (s-1) */
    #define REBUILDN(vst, s, d, out) do {                                                 \
      if (d == 1) {                                                                       \
        REBUILD(vst, out);                                                                \
      } else {                                                                            \
        const Step cb_ = ld_step<K == 2>(prog, s - d);                                            \
        V4 acc_[K];                                                                       \
        REBUILD(cb_, acc_);                                                               \
        for (int j_ = d - 1; j_ >= 2; --j_) {                                             \
          const Step v_ = ld_step<K == 2>(prog, s - j_);                                          \
          CHAIN_UP(v_, acc_, acc_);                                                       \
        }                                                                                 \
        CHAIN_UP(vst, acc_, out);                                                         \
      }                                                                                   \
    } while (0)
    #define RSTEP_V(s, cs, cn, XT, YT) do {                                               \
      const Step& st = cs.st;                                                     \
      ensure_chunk(st);                                                           \
      const int fl = st.fl;                                                       \
      V4 rv[K], ax[K], ay[K], q[K], rx[K], ry[K];                                 \
      unsigned bx[K], by[K];                                                      \
      if (fl & F_VDEEP) {                                                         \
        const int vd = st.vd;                                                     \
        if (DL || vd < ndl) {                                                     \
      _Pragma("unroll")                                                           \
          for (int k = 0; k < K; ++k) rv[k] = dget(vd, k);                        \
        } else {                                                                  \
      _Pragma("unroll")                                                           \
          for (int k = 0; k < K; ++k) rv[k] = cs.lr[k];                           \
        }                                                                         \
      } else {                                                                    \
      _Pragma("unroll")                                                           \
        for (int k = 0; k < K; ++k) rv[k] = topr[k];                              \
      }                                                                           \
      if (XT) {                                                                   \
        const int mx = st.mx, x = st.x;                                           \
      _Pragma("unroll")                                                           \
        for (int k = 0; k < K; ++k) {                                             \
          bx[k] = tipb(x, k);                                                     \
          ax[k] = look(mx, bx[k]);                                                \
        }                                                                         \
      } else if (YT && (fl & F_PREVREC)) { /* x is the rebuilt previous-step child */  \
        REBUILDN(cn.st, s, st.rd, ax);                                                 \
      } else {                                                                         \
      _Pragma("unroll")                                                                \
        for (int k = 0; k < K; ++k) ax[k] = cs.lx[k];                                  \
      }                                                                           \
      if (YT) {                                                                   \
        const int my = st.my, y = st.y;                                           \
      _Pragma("unroll")                                                           \
        for (int k = 0; k < K; ++k) {                                             \
          by[k] = tipb(y, k);                                                     \
          ay[k] = look(my, by[k]);                                                \
        }                                                                         \
      } else if (fl & F_PREVREC) { /* y is the rebuilt previous-step child */  \
        REBUILDN(cn.st, s, st.rd, ay);                                         \
      } else {                                                                 \
      _Pragma("unroll")                                                        \
        for (int k = 0; k < K; ++k) ay[k] = cs.ly[k];                          \
      }                                                                           \
      if (fl & F_MV) {                                                            \
        const int mv = st.mv;                                                     \
        V4 pv[K];                                                                 \
      _Pragma("unroll")                                                           \
        for (int k = 0; k < K; ++k) pv[k] = vmul(ax[k], ay[k]);                   \
        ptvec_k<K>(mrec(mv), rv, q);                                              \
        gacc(mv, rv, pv); /* dL/dP_v += r_v (x) p_v */                            \
      } else { /* root, or the merged root branch: identity */                    \
      _Pragma("unroll")                                                           \
        for (int k = 0; k < K; ++k) q[k] = rv[k];                                 \
      }                                                                           \
      _Pragma("unroll")                                                           \
      for (int k = 0; k < K; ++k) {                                               \
        rx[k] = vmul(q[k], ay[k]);                                                \
        ry[k] = vmul(q[k], ax[k]);                                                \
      }                                                                           \
      if (XT) {                                                                   \
        V4 tv[K];                                                                 \
      _Pragma("unroll")                                                           \
        for (int k = 0; k < K; ++k) tv[k] = tipvec_l(tvec, bx[k]);                \
        gacc(st.mx, rx, tv);                                                      \
      }                                                                           \
      if (YT) {                                                                   \
        V4 tv[K];                                                                 \
      _Pragma("unroll")                                                           \
        for (int k = 0; k < K; ++k) tv[k] = tipvec_l(tvec, by[k]);                \
        gacc(st.my, ry, tv);                                                      \
      }                                                                           \
      if (!XT && !YT) { /* r_x waits on the deep stack while y's subtree runs */  \
        const int dp = st.xd;                                                     \
      _Pragma("unroll")                                                           \
        for (int k = 0; k < K; ++k) {                                             \
          if (DL || dp < ndl) dput(dp, k, rx[k]); else put(dsk, dp, k, rx[k]);    \
          topr[k] = ry[k];                                                        \
        }                                                                         \
      } else if (!YT) {                                                           \
      _Pragma("unroll")                                                           \
        for (int k = 0; k < K; ++k) topr[k] = ry[k];                              \
      } else if (!XT) {                                                           \
      _Pragma("unroll")                                                           \
        for (int k = 0; k < K; ++k) topr[k] = rx[k];                              \
      }                                                                           \
    } while (0)
    /* one straight-line body per child kind (tip / internal), so the
       independent LDS reads and dL/dP reductions of a step share a basic
       block and the scheduler can interleave them */
    #define RSTEP(s, cs, cn) do {                        \
      const int xt_ = cs.st.x >= 0, yt_ = cs.st.y >= 0;  \
      if (xt_ && yt_) RSTEP_V(s, cs, cn, true, true);    \
      else if (xt_) RSTEP_V(s, cs, cn, true, false);     \
      else if (yt_) RSTEP_V(s, cs, cn, false, true);     \
      else RSTEP_V(s, cs, cn, false, false);             \
    } while (0)
    {
      int s = nsteps - 1;
      CSet A, Bs;
      LOAD_SET(s, A);
      for (;;) {
        TT_MARK(trip * 320 + 154 + (nsteps - 1 - s));
        LOAD_SET(s - 1, Bs);
        RSTEP(s, A, Bs);
        if (--s < 0) break;
        TT_MARK(trip * 320 + 154 + (nsteps - 1 - s));
        LOAD_SET(s - 1, A);
        RSTEP(s, Bs, A);
        if (--s < 0) break;
      }
    }
    WAIT_VMCNT0();
    TT_MARK(trip * 320 + 310);
    gfirst = false;
  }

  // per-wave scalar partials: [ll, dps, dfreq0..3]
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
  if (a.g_direct) {
    // One workgroup per draw: this wave's slot is the draw's dL/dP for
    // category c.  Write the output rows (branch order) and the chain-rule
    // inner products <G_cb, Q P_cb> (dP/dt = Q P), 16 lanes per matrix.
    // The atomics were performed at L2 once vmcnt drains; the slot is read
    // back with agent-scope loads (past L1, same XCD's L2).  No device fence:
    // a release fence here would write back the whole L2 per workgroup.
    WAIT_VMCNT0();
    // fin: the finalize runs here; its LDS (inner products [C][B], then the
    // waves' scalar partials [C][8], then qgrad's) reuses the sweep's, once
    // every wave is done
    TT_MARK(990);
    double* innerL = mats0;
    double* scalL = mats0 + (size_t)C * a.B;
    if (a.fin) __syncthreads();
    const double* Qd = a.eig + (size_t)draw * EIG_LEN + EIG_Q;
    double* gout = a.grows + (size_t)draw * a.grows_stride;
    double* inner_d = a.inner + (size_t)draw * C * a.B;
    // k = lane (mod 64): every item of this lane has the same entry e16 =
    // (j, kk), so the Q row is loaded once
    const int e16 = lane & 15, j = e16 >> 2, kk = e16 & 3;
    const double q0 = Qd[j * 4 + 0], q1 = Qd[j * 4 + 1], q2 = Qd[j * 4 + 2], q3 = Qd[j * 4 + 3];
    const int tot = nmat * 16;  // a multiple of 16: 16-lane groups are whole
    constexpr int U = PHY_EPI_U;
    for (int k0 = lane; k0 < tot; k0 += WAVE * U) {
      double g[U], qp[U];
      int bb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {  // all loads in flight before any use
        const int k = k0 + u * WAVE;
        const int kc = k < tot ? k : lane;
        const int mm = kc >> 4;
        g[u] = __hip_atomic_load(gs + kc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const double2* col = reinterpret_cast<const double2*>(pmat_c + (size_t)mm * rec + kk * 4);  // column kk of P
        const double2 c01 = col[0], c23 = col[1];
        qp[u] = fma(q3, c23.y, fma(q2, c23.x, fma(q1, c01.y, q0 * c01.x)));
        bb[u] = a.mat_branch[mm];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + u * WAVE;
        if (k < tot) {
          // the 16-entry butterfly (xor 8, 4, 2, 1) in DPP: after the first
          // stage lanes i and i^8 hold the same sum, so row_ror:4 reads the
          // value xor 4 would -- the __shfl_xor butterfly's bits, no LDS trips
          double sv = g[u] * qp[u];
          sv += dpp_d<DPP_ROW_ROR8>(sv);
          sv += dpp_d<0x124>(sv);  // row_ror:4
          sv += dpp_d<DPP_QUAD_XOR2>(sv);
          sv += dpp_d<DPP_QUAD_XOR1>(sv);
          gout[((size_t)c * a.B + bb[u]) * 16 + e16] = g[u];
          if (e16 == 0) {
            inner_d[(size_t)c * a.B + bb[u]] = sv;
            if (a.fin) innerL[(size_t)c * a.B + bb[u]] = sv;
          }
        }
      }
    }
    TT_MARK(991);
    if (a.fin) {
      if (lane == 0) {
        double* sl = scalL + (size_t)wv * 8;
        sl[0] = acc_ll;
        sl[1] = acc_dps;
        sl[2] = acc_f.x;
        sl[3] = acc_f.y;
        sl[4] = acc_f.z;
        sl[5] = acc_f.w;
      }
      __syncthreads();
      // finalize_kernel's sums, in its order (bitwise the same results)
      const int B = a.B;
      double* out = a.out + (size_t)draw * a.outlen;
      const double* rs = mdl + 10;
      const double* bl = a.blens + (size_t)draw * B;
      for (int b = threadIdx.x; b < B; b += nthreads) {
        double sacc = 0.0;
        for (int cc = 0; cc < C; ++cc) sacc = fma(rs[cc], innerL[cc * B + b], sacc);
        out[1 + b] = sacc;
      }
      for (int cc = threadIdx.x; cc < C; cc += nthreads) {
        double sacc = 0.0;
        for (int b = 0; b < B; ++b) sacc = fma(bl[b], innerL[cc * B + b], sacc);
        out[1 + B + cc] = sacc;
      }
      if (threadIdx.x == 0) {
        auto tot8 = [&](int cc, int jj) { return scalL[(size_t)cc * 8 + jj]; };
        const double ll = tot8(0, 0);
        out[0] = isfinite(ll) ? ll : -INFINITY;
        for (int cc = 0; cc < C; ++cc) out[1 + B + C + cc] = tot8(cc, 1);
        for (int q = 0; q < 4; ++q) {
          double t = 0.0;
          for (int cc = 0; cc < C; ++cc) t += tot8(cc, 2 + q);
          out[1 + B + 2 * C + q] = t;
        }
      }
      TT_MARK(992);
      if (a.qfused) {  // the Q-parameter chain rule (qgrad_kernel's work, same bits)
        double* qsh = scalL + (size_t)C * 8;
        const QgArgs q{a.eig, a.model, a.blens, a.grows, a.grows_stride, a.out, a.outlen, C, B, a.kind};
        __syncthreads();  // dL/dP rows and the root term visible to the workgroup
        qgrad_body(q, draw, threadIdx.x, qsh);
      }
    }
  }
  TT_MARK(1000);
}

#include "quad_engine.inc"

// ---------------------------------------------------------------------------
// P-matrices (generate_script.py:755-892)
// ---------------------------------------------------------------------------

struct PmatArgs {
  const double* model;    // [draw][10+2C]
  const double* blens;    // [draw][B]
  const int* mat_branch;  // [nmat] branch (node id) of matrix m
  double* eig;            // [draw][EIG_LEN]
  double* pmat;           // [draw][C][nmat][R][4]  records, program-use order
  int C, B, kind, nmat, n, R;
  unsigned long long extra;  // tip masks of record vectors 4..R-1, 4 bits each
  int with_eig;  // pmat_kernel forms the draw's eigensystem itself (small batches: no eig launch)
};

// Jacobi eigendecomposition of a symmetric 4x4 (A overwritten) in the
// parallel ordering: each sweep is three rounds of two rotations on disjoint
// index pairs -- {(0,1),(2,3)}, {(0,2),(1,3)}, {(0,3),(1,2)}.  A round's two
// rotation parameters read entries the other rotation does not change, so
// their chains (square root, square root, division: the latency of the
// solve on one GPU thread) run side by side -- three chains
// per sweep instead of six.  Then A <- J^T A J and V <- V J for the round's
// combined rotation J.  No FMA contraction here or in eig_record, and every
// operation in the C oracle's order (oracle/cpu_pruner.c jacobi4): the same
// bits -- the gradients' agreement with the oracle at 10^5-10^6 sites rests
// on it (an independent eigensolver moves dL/dP by ~1e-9 relative there).
__host__ __device__ inline void jacobi_rot(double app, double aqq, double apq, double& cs, double& sn) {
#pragma clang fp contract(off)
  if (apq == 0.0) {  // the identity
    cs = 1.0;
    sn = 0.0;
    return;
  }
  // t = sgn(theta) / (|theta| + sqrt(theta^2 + 1)), theta = d / e, with the
  // divisions folded: cs = 1 / sqrt(t^2 + 1) = den / w, sn = t cs =
  // sgn(theta) |e| / w, den = |d| + sqrt(d^2 + e^2), w = sqrt(den^2 + e^2)
  // (two square roots and one division on the chain instead of three)
  const double d = aqq - app, e = 2.0 * apq;
  const double den = fabs(d) + sqrt(d * d + e * e);
  const double inv = 1.0 / sqrt(den * den + e * e);
  const double ae = fabs(e);
  cs = den * inv;
  sn = ((d == 0.0 || (d > 0.0) == (e > 0.0)) ? ae : -ae) * inv;  // sgn(theta): + at theta = 0
}
__host__ __device__ void jacobi4(double A[4][4], double V[4][4], double lam[4]) {
#pragma clang fp contract(off)
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
    for (int r = 0; r < 3; ++r) {
      const int p1 = 0, q1 = r + 1;                       // (0,1) (0,2) (0,3)
      const int p2 = r == 0 ? 2 : 1, q2 = r == 2 ? 2 : 3;  // (2,3) (1,3) (1,2)
      double c1, s1, c2, s2;
      jacobi_rot(A[p1][p1], A[q1][q1], A[p1][q1], c1, s1);
      jacobi_rot(A[p2][p2], A[q2][q2], A[p2][q2], c2, s2);
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // A <- A J   (columns)
        const double a1 = A[k][p1], b1 = A[k][q1], a2 = A[k][p2], b2 = A[k][q2];
        A[k][p1] = c1 * a1 - s1 * b1;
        A[k][q1] = s1 * a1 + c1 * b1;
        A[k][p2] = c2 * a2 - s2 * b2;
        A[k][q2] = s2 * a2 + c2 * b2;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // A <- J^T A (rows)
        const double a1 = A[p1][k], b1 = A[q1][k], a2 = A[p2][k], b2 = A[q2][k];
        A[p1][k] = c1 * a1 - s1 * b1;
        A[q1][k] = s1 * a1 + c1 * b1;
        A[p2][k] = c2 * a2 - s2 * b2;
        A[q2][k] = s2 * a2 + c2 * b2;
      }
      A[p1][q1] = A[q1][p1] = 0.0;
      A[p2][q2] = A[q2][p2] = 0.0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // V <- V J
        const double a1 = V[k][p1], b1 = V[k][q1], a2 = V[k][p2], b2 = V[k][q2];
        V[k][p1] = c1 * a1 - s1 * b1;
        V[k][q1] = s1 * a1 + c1 * b1;
        V[k][p2] = c2 * a2 - s2 * b2;
        V[k][q2] = s2 * a2 + c2 * b2;
      }
    }
  }
  for (int i = 0; i < 4; ++i) lam[i] = A[i][i];
}

// Normalised Q and its eigensystem of one draw's model vector (the
// EIG_LEN record: P(t) = m1 diag(exp(lam t)) m2, Q, the normaliser):
// eig_kernel runs it one thread per draw for batches, lane 0 of each pmat
// wave for small ones (a serial chain of one thread either way).
__host__ __device__ void eig_record(const double* mdl, int kind, double* out) {
#pragma clang fp contract(off)
  if (kind == PHY_JC69) {  // generate_script.py:765-769 (closed form; Q for dP/dt only)
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
  out[EIG_S] = s;  // the normaliser, for the Q-parameter chain rule
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

// eig_record for one wave (pmat_kernel<true>: a small device batch, where
// the one-lane chain of eig_record was most of the launch): lane (j, k),
// j, k < 4, owns element [j][k] of Q, A and V; the Jacobi rotation
// parameters are formed by every lane from the same LDS values, each pass of
// a round updates the 16 elements in parallel through LDS.  Every element
// sees exactly eig_record's operations in eig_record's order (no FMA
// contraction), so the record is bitwise eig_record's (tested against the
// host-formed eigensystems).  All 64 lanes must call it; `sh` is 48 doubles
// of LDS; the result lands in `out` (LDS, EIG_LEN doubles).
__device__ void eig_record_wave(const double* mdl, int kind, double* out, double* sh, int lane) {
#pragma clang fp contract(off)
  const int j = (lane >> 2) & 3, k = lane & 3;
  const bool own = lane < 16;
  double* A = sh;       // [4][4]
  double* V = sh + 16;  // [4][4]
  if (kind == PHY_JC69) {
    if (own) out[EIG_Q + j * 4 + k] = (j == k) ? -1.0 : 1.0 / 3.0;
    __syncthreads();
    return;
  }
  const double f[4] = {mdl[0], mdl[1], mdl[2], mdl[3]};
  const double* r = mdl + 4;
  const double R[4][4] = {{0.0, r[0], r[1], r[2]}, {r[0], 0.0, r[3], r[4]}, {r[1], r[3], 0.0, r[5]},
                          {r[2], r[4], r[5], 0.0}};
  // Q = R diag(pi) with zero-sum rows and the normaliser s, in eig_record's
  // order (every lane: a few dozen operations)
  double q[4][4];
  double sn = 0.0;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    double row = 0.0;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      q[jj][kk] = (jj == kk) ? 0.0 : R[jj][kk] * f[kk];
      row += q[jj][kk];
    }
    q[jj][jj] = -row;
    sn -= q[jj][jj] * f[jj];
  }
  double sq[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) sq[jj] = sqrt(f[jj]);
  // this lane's element: q[j][k] / s, q[k][j] / s, then A[j][k]
  double qjk = 0.0, qkj = 0.0;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (jj == j && kk == k) qjk = q[jj][kk];
      if (jj == k && kk == j) qkj = q[jj][kk];
    }
  qjk /= sn;
  qkj /= sn;
  const double sqj = j == 0 ? sq[0] : j == 1 ? sq[1] : j == 2 ? sq[2] : sq[3];
  const double sqk = k == 0 ? sq[0] : k == 1 ? sq[1] : k == 2 ? sq[2] : sq[3];
  if (own) {
    out[EIG_Q + j * 4 + k] = qjk;
    A[j * 4 + k] = (j == k) ? qjk : 0.5 * (sqj * qjk / sqk + sqk * qkj / sqj);
    V[j * 4 + k] = (j == k) ? 1.0 : 0.0;
  }
  if (lane == 0) out[EIG_S] = sn;
  __syncthreads();
  for (int sweep = 0; sweep < 50; ++sweep) {
    double off = 0.0, tot = 0.0;
    for (int i = 0; i < 4; ++i)
      for (int jj = 0; jj < 4; ++jj) {
        tot += A[i * 4 + jj] * A[i * 4 + jj];
        if (i != jj) off += A[i * 4 + jj] * A[i * 4 + jj];
      }
    if (off <= 1e-32 * tot || off == 0.0) break;  // wave-uniform
#pragma unroll
    for (int rr = 0; rr < 3; ++rr) {
      const int p1 = 0, q1 = rr + 1;
      const int p2 = rr == 0 ? 2 : 1, q2 = rr == 2 ? 2 : 3;
      double c1, s1, c2, s2;
      jacobi_rot(A[p1 * 4 + p1], A[q1 * 4 + q1], A[p1 * 4 + q1], c1, s1);
      jacobi_rot(A[p2 * 4 + p2], A[q2 * 4 + q2], A[p2 * 4 + q2], c2, s2);
      // element (j, k)'s rotation: the pair {p, q} holding k (columns) / j (rows)
      auto rot = [&](const double* M, int row, int col, bool by_col) __attribute__((always_inline)) -> double {
        const int x = by_col ? col : row;
        const bool first = x == p1 || x == q1;
        const int p = first ? p1 : p2, qq = first ? q1 : q2;
        const double cc = first ? c1 : c2, ss = first ? s1 : s2;
        const double av = by_col ? M[row * 4 + p] : M[p * 4 + col];
        const double bv = by_col ? M[row * 4 + qq] : M[qq * 4 + col];
        return x == p ? cc * av - ss * bv : ss * av + cc * bv;
      };
      // A <- J^T (A J): the two column-rotated entries of k's column that
      // row j's rotation combines, (A J)[p][k] and (A J)[q][k] ({p, q} = j's
      // pair), formed by this lane from A itself -- the same operations as
      // the two-pass form, without the intermediate's LDS round trip and barrier
      double na = 0.0, nv = 0.0;
      if (own) {
        const bool first = j == p1 || j == q1;
        const int p = first ? p1 : p2, qq = first ? q1 : q2;
        const double cc = first ? c1 : c2, ss = first ? s1 : s2;
        const double tp = rot(A, p, k, true), tq = rot(A, qq, k, true);  // (A J)[p][k], (A J)[qq][k]
        na = j == p ? cc * tp - ss * tq : ss * tp + cc * tq;
        if ((j == p1 && k == q1) || (j == q1 && k == p1) || (j == p2 && k == q2) || (j == q2 && k == p2)) na = 0.0;
        nv = rot(V, j, k, true);   // V <- V J
      }
      __syncthreads();  // every lane has read A and V
      if (own) {
        A[j * 4 + k] = na;
        V[j * 4 + k] = nv;
      }
      __syncthreads();
    }
  }
  if (own) {
    if (k == 0) out[EIG_LAM + j] = A[j * 4 + j];
    out[EIG_M1 + j * 4 + k] = V[j * 4 + k] / sqj;  // Pi^-1/2 V
    out[EIG_M2 + j * 4 + k] = V[k * 4 + j] * sqk;  // V^T Pi^1/2
  }
  __syncthreads();
}

// One thread per draw.
__global__ void __launch_bounds__(64) eig_kernel(PmatArgs a) {
  const int draw = blockIdx.x * blockDim.x + threadIdx.x;
  if (draw >= a.n) return;
  eig_record(a.model + (size_t)draw * (10 + 2 * a.C), a.kind, a.eig + (size_t)draw * EIG_LEN);
}

// One thread per (draw, category, matrix): the matrix record in program-use
// order -- the four columns of P, then P t for each extra tip mask t (the
// 0/1 sum of P's columns, in column order: bitwise what a mat-vec with the
// 0/1 vector gives).
// One wave per 64 consecutive records of a draw (record idx = c*nmat + m,
// contiguous in memory): each lane builds its record in LDS, then the wave
// copies the 64 records out as one contiguous run (whole-line stores; a
// record per lane straight to HBM would scatter every store instruction).
constexpr int PMAT_WAVE_RECS = 64;
constexpr int EIG_FUSE_MAX = 32;  // draws per launch up to which pmat_kernel forms the eigensystems
// WITH_EIG is a template parameter, not a runtime flag: the inlined Jacobi's
// registers would otherwise be allocated in the batched kernel too (round 3:
// 0.158 -> 0.249 ms per fluA launch of 8192 draws when it was a runtime flag).
template <bool WITH_EIG>
__global__ void __launch_bounds__(64) pmat_kernel(PmatArgs a) {
  __shared__ double e[EIG_LEN];
  extern __shared__ __attribute__((aligned(16))) double recl[];  // [64][R*4]
  const int draw = blockIdx.y;
  const int C = a.C, nmat = a.nmat;
  const int lane = threadIdx.x;
  if constexpr (WITH_EIG) {  // every wave of the draw forms it, lane-parallel (no eig launch)
    __shared__ double esh[48];
    eig_record_wave(a.model + (size_t)draw * (10 + 2 * C), a.kind, e, esh, lane);
    if (blockIdx.x == 0 && lane < EIG_LEN) a.eig[(size_t)draw * EIG_LEN + lane] = e[lane];
  } else if (lane < EIG_LEN) {
    e[lane] = a.eig[(size_t)draw * EIG_LEN + lane];
  }
  __syncthreads();
  const int total = C * nmat;
  const int idx0 = blockIdx.x * PMAT_WAVE_RECS;
  const int nrec = min(PMAT_WAVE_RECS, total - idx0);
  const int rlen = a.R * 4;  // doubles per record
  const int idx = idx0 + lane;
  if (lane < nrec) {
    const int c = idx / nmat, m = idx - c * nmat;
    const int br = a.mat_branch[m];
    double2* po = reinterpret_cast<double2*>(recl + (size_t)lane * rlen);
    const double* mdl = a.model + (size_t)draw * (10 + 2 * C);
    build_record(e, a.blens[(size_t)draw * a.B + br] * mdl[10 + c], a.kind, a.R, a.extra, po);
  }
  __syncthreads();
  const double2* src = reinterpret_cast<const double2*>(recl);
  double2* dst = reinterpret_cast<double2*>(a.pmat + ((size_t)draw * total + idx0) * rlen);
  const int n2 = nrec * rlen / 2;
  for (int k = lane; k < n2; k += 64) dst[k] = src[k];
}

// ---------------------------------------------------------------------------
// finalize: fixed-order sums of the per-workgroup slots + chain rule dP/dt
// ---------------------------------------------------------------------------
struct FinArgs {
  const double* gslot;  // [wg][C][nmat][16]  program-use order
  const double* sslot;  // [wg][C][8]
  const double* pmat;   // [draw][C][nmat][R][4]  records (columns of P first)
  const double* eig;    // [draw][EIG_LEN]
  const double* blens;  // [draw][B]
  const double* model;  // [draw][10+2C]
  const int* gpos;      // [B] matrix index of branch b
  const double* inner;  // [draw][C][B] <G, Q P> from the sweep when g_direct
  double* out;          // [draw][outlen]
  int C, B, nmat, gx, outlen, g_direct, R;
  double* grows;        // dL/dP rows (see SweepArgs)
  long long grows_stride;
  int kind;
  int gsum_in;  // finalize_kernel first sums the gx per-workgroup dL/dP slots itself (few slots per draw)
  int qf;       // finalize_kernel then runs the Q-parameter chain rule (qgrad_body)
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
    a.grows[(size_t)draw * a.grows_stride + idx] = s;
  }
}

// One 1,024-thread workgroup per draw (dL/dP rows already in place: sweep or
// gsum, or summed here first when a draw spans few workgroups -- gsum_in),
// so the slot sums are a few rounds of loads in flight instead of a long
// latency chain (the synthetic workload's 2,063 root chunks: 38 us with 256
// threads); then, with qf, the Q-parameter chain rule: one launch for the
// whole epilogue of a small batch.
//   scalars log L, dlogL/dps, root-frequency term: wave 0, lane-strided
//           over slots + a fixed-shape wave reduction;
//   chain rule  dlogL/dt_{b,c} = <G_bc, Q P_bc>,  dlogL/db = sum_c r_c (.),
//           dlogL/dr_c = sum_b b (.)   (generate_script.py:663-671 blens).
// The fused epilogue's dL/dP provider (finalize_kernel with the chain rule):
// lane k of the (c, b) item's quad forms row k of G -- the sum of the gx
// workgroup slots (gsum_in; written out as the dL/dP row) or the row
// itself -- qgrad_body broadcasts the rows inside the quad, and its share of <G, Q P>
// goes to inner[idx] after a quad sum.  One pass over the items instead of
// slot sums -> HBM -> <G, QP> -> HBM -> the chain rule's reads.
struct FusedG {
  const FinArgs& a;
  int draw;
  double* inner;    // LDS [C*B]
  const double* Q;  // LDS [16]
  __device__ __forceinline__ void operator()(int idx, int k, double (&g)[4]) const {
    const int C = a.C, B = a.B;
    const int c = idx / B, b = idx - c * B;
    const int mm = a.gpos[b];
    double* grow = a.grows + (size_t)draw * a.grows_stride + (size_t)idx * 16 + k * 4;
    double r[4];
    if (a.gsum_in) {
      const size_t per_wg = (size_t)C * a.nmat * 16;
      const double* src = a.gslot + (size_t)draw * a.gx * per_wg + ((size_t)c * a.nmat + mm) * 16 + k * 4;
      double2 lo = *reinterpret_cast<const double2*>(src), hi = *reinterpret_cast<const double2*>(src + 2);
      r[0] = lo.x; r[1] = lo.y; r[2] = hi.x; r[3] = hi.y;
      for (int w0 = 1; w0 < a.gx; w0 += 4) {  // 4 slots (8 loads) in flight, summed in slot order
        double2 l8[4], h8[4];  // (8 slots spill at 1,024 threads)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int w = w0 + u < a.gx ? w0 + u : 0;
          l8[u] = *reinterpret_cast<const double2*>(src + (size_t)w * per_wg);
          h8[u] = *reinterpret_cast<const double2*>(src + (size_t)w * per_wg + 2);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (w0 + u < a.gx) {
            r[0] += l8[u].x; r[1] += l8[u].y; r[2] += h8[u].x; r[3] += h8[u].y;
          }
      }
      *reinterpret_cast<double2*>(grow) = make_double2(r[0], r[1]);
      *reinterpret_cast<double2*>(grow + 2) = make_double2(r[2], r[3]);
    } else {
      const double2 lo = *reinterpret_cast<const double2*>(grow), hi = *reinterpret_cast<const double2*>(grow + 2);
      r[0] = lo.x; r[1] = lo.y; r[2] = hi.x; r[3] = hi.y;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) g[j] = r[j];
    // row k of <G, Q P>: sum_j G[k][j] (Q P)[k][j]; P column-major in its record
    const double* P = a.pmat + ((size_t)draw * C * a.nmat + (size_t)c * a.nmat + mm) * a.R * 4;
    double sv = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double2 p01 = *reinterpret_cast<const double2*>(P + j * 4);
      const double2 p23 = *reinterpret_cast<const double2*>(P + j * 4 + 2);
      const double qp = fma(Q[k * 4 + 3], p23.y, fma(Q[k * 4 + 2], p23.x, fma(Q[k * 4 + 1], p01.y, Q[k * 4] * p01.x)));
      sv = fma(r[j], qp, sv);
    }
    sv += dpp_d<0xB1>(sv);  // quad_perm [1,0,3,2]
    sv += dpp_d<0x4E>(sv);  // quad_perm [2,3,0,1]
    if (k == 0) inner[idx] = sv;
  }
};

__global__ void __launch_bounds__(1024) finalize_kernel(FinArgs a) {
  extern __shared__ double fsh[];  // inner[C*B], Q[16]
  const int draw = blockIdx.x;
  const int C = a.C, B = a.B;
  double* inner = fsh;
  double* Q = fsh + (size_t)C * B;
  double* out = a.out + (size_t)draw * a.outlen;
  const size_t wg0 = (size_t)draw * a.gx;
  // the chain rule's pass also sums the slots and forms <G, QP> (FusedG)
  const bool fused = a.qf && !a.g_direct && a.kind != PHY_JC69 && blockDim.x == QG_THREADS;
  if (a.gsum_in && !fused) {
    // the draw's dL/dP rows from its gx workgroup slots, summed in slot
    // order (gsum_kernel's work, for draws spread over a few workgroups);
    // made visible to the workgroup by the barriers below
    const size_t per_wg = (size_t)C * a.nmat * 16;
    const double* base = a.gslot + (size_t)draw * a.gx * per_wg;
    for (int idx = threadIdx.x; idx < C * B * 16; idx += blockDim.x) {
      const int c = idx / (B * 16), rem = idx - c * B * 16;
      const int b = rem >> 4, k = rem & 15;
      const double* src = base + ((size_t)c * a.nmat + a.gpos[b]) * 16 + k;
      double s = src[0];
      for (int w0 = 1; w0 < a.gx; w0 += 8) {  // 8 slots in flight, summed in slot order
        double v8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v8[u] = src[(size_t)(w0 + u < a.gx ? w0 + u : 0) * per_wg];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (w0 + u < a.gx) s += v8[u];
      }
      a.grows[(size_t)draw * a.grows_stride + idx] = s;
    }
  }
  if (threadIdx.x < 16) Q[threadIdx.x] = a.eig[(size_t)draw * EIG_LEN + EIG_Q + threadIdx.x];
  {
    // scalar partials per slot: [c][8] = ll (c = 0 only), dps_c, dfreq[4].
    // Thread t owns element k = t % (8C) of the slot records and sums it over
    // the slots of its group g = t / (8C) (slots g, g + G, ...: one
    // coalesced 8C-double record per group per step, 16 in flight), then
    // thread k sums the G group partials in group order -- a fixed order,
    // and with a single slot (one workgroup per draw) exactly that slot.
    const int E = 8 * C;
    const int G = max(1, (int)blockDim.x / E);
    double* red = fsh + (size_t)C * B + 16;  // blockDim.x doubles past inner[C*B] and Q[16]
    const int g = threadIdx.x / E, k = threadIdx.x - g * E;
    double acc = 0.0;
    if (g < G && E <= (int)blockDim.x) {
      const double* ss = a.sslot + wg0 * E + k;
      constexpr int U = 16;  // loads in flight: thousands of slots are a latency chain otherwise
      for (int w0 = g; w0 < a.gx; w0 += U * G) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int w = w0 + u * G;
          v[u] = (w < a.gx) ? ss[(size_t)w * E] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
      }
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    double tot = 0.0;
    if ((int)threadIdx.x < E) {
      for (int gg = 0; gg < G; ++gg) tot += red[gg * E + threadIdx.x];
    }
    __syncthreads();
    if ((int)threadIdx.x < E) red[threadIdx.x] = tot;
    __syncthreads();
    if (threadIdx.x == 0) {
      const double ll = red[0];
      out[0] = isfinite(ll) ? ll : -INFINITY;
      for (int c = 0; c < C; ++c) out[1 + B + C + c] = red[c * 8 + 1];
      for (int f = 0; f < 4; ++f) {
        double t = 0.0;
        for (int c = 0; c < C; ++c) t += red[c * 8 + 2 + f];
        out[1 + B + 2 * C + f] = t;
      }
    }
  }
  __syncthreads();  // dL/dP rows and Q visible to the whole workgroup
  if (fused) {
    const QgArgs q{a.eig, a.model, a.blens, a.grows, a.grows_stride, a.out, a.outlen, C, B, a.kind};
    qgrad_body(q, draw, threadIdx.x, fsh + (size_t)C * B + 16 + blockDim.x, FusedG{a, draw, inner, Q});
    __syncthreads();  // inner[] complete (and the chain rule's tail done)
  }
  const int rec = a.R * 4;
  const double* pm = a.pmat + (size_t)draw * C * a.nmat * rec;
  for (int idx = threadIdx.x; idx < C * B && !fused; idx += blockDim.x) {
    if (a.g_direct) {  // formed by the sweep's last flush
      inner[idx] = a.inner[(size_t)draw * C * B + idx];
      continue;
    }
    const int c = idx / B, b = idx - c * B;
    const double* g = a.grows + (size_t)draw * a.grows_stride + (size_t)idx * 16;
    const double* P = pm + ((size_t)c * a.nmat + a.gpos[b]) * rec;  // column-major
    double gv[16], pv[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      gv[k] = g[k];
      pv[k] = P[(k & 3) * 4 + (k >> 2)];  // row-major P[l][k] = column k, entry l
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
  if (!fused) __syncthreads();
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
  if (a.qf && !fused) {  // the Q-parameter chain rule (qgrad_kernel's work, same bits)
    __syncthreads();  // the finalize's root term visible to thread 0 of qgrad_body
    const QgArgs q{a.eig, a.model, a.blens, a.grows, a.grows_stride, a.out, a.outlen, C, B, a.kind};
    qgrad_body(q, draw, threadIdx.x, fsh + (size_t)C * B + 16 + blockDim.x);
  }
}

__global__ void __launch_bounds__(QG_THREADS) qgrad_kernel(FinArgs a) {
  __shared__ double sh[QG_SHARED];
  const QgArgs q{a.eig, a.model, a.blens, a.grows, a.grows_stride, a.out, a.outlen, a.C, a.B, a.kind};
  qgrad_body(q, blockIdx.x, threadIdx.x, sh);
}

// The small call's epilogue split over workgroups (the quad sweep's, <= 16
// draws of <= 16 workgroup slots each).  One 1,024-thread workgroup per draw
// (finalize_kernel) reads the draw's ~1 MB of slots (fluA: 15 x C x nmat x
// 16 doubles, written by workgroups on other XCDs: L2 misses) through ONE
// CU, 16 dependent rounds: 25 us of a 125 us sampler call (r04f SQ: 67% of
// the waves' cycles waiting).  Here workgroup s of a draw owns branches
// [s bper, (s + 1) bper) in every category, a quad of lanes per (c, b)
// item with every slot load of the item in flight at once:
//   * row k of G_cb = the slots summed in slot order -> the dL/dP row;
//   * <G_cb, Q P_cb> (finalize's order) -> dlogL/db = sum_c r_c (.) for the
//     owned branches directly, sum_b b (.) per category as a hand-off;
//   * the item's share of M = sum_cb (V^T G V^-T) o Phi (qgrad_body's
//     terms), summed over the workgroup's items in a fixed tree -> hand-off;
//   * workgroup 0 also sums the scalar slots (log L, dlogL/dps, the root
//     frequency term).
// Hand-offs are write-through agent-scope stores; the draw's last workgroup
// (a ticket) takes one acquire and sums the hand-offs in workgroup order,
// then W = V^-T M V^T and q_tail.  Deterministic: every sum has a fixed
// order (not finalize_kernel's bits: M and sum_b b (.) are summed per
// workgroup first).
constexpr int QFIN_THREADS = 256;
constexpr int QFIN_ITEMS = QFIN_THREADS / 4;  // (c, b) items per workgroup
constexpr int QFIN_SLOTS = 16;                // workgroup slots per draw it takes
// HANDOFF.  The sampler's split epilogue (qfin_kernel) hands per-
// workgroup partials to the draw's last-arriving workgroup inside one launch
// (the class sweep's epilogue did too until round 6; it is two launches now):
// every hand-off byte is stored write-through (sc1: __hip_atomic_store
// relaxed/agent), every storing wave drains vmcnt, a workgroup barrier, then
// ONE lane's relaxed agent-scope ticket add; the workgroup whose add returns
// the last ticket reads the hand-offs with sc1 loads only (relaxed agent-scope
// atomic loads).  On gfx950 that is the sc1 form of cdna_hip_programming.md
// Guideline 16 / MI355X_MICROARCH.md "Valid forms" row 1: sc1 stores leave
// the producer's L2 at once, sc1 loads bypass the reader's L1, and the add is
// issued after the drain -- the reader cannot see a stale copy.  On top of
// that the last workgroup takes ONE agent-scope acquire after its ticket (the
// guide's Consumer recipe: relaxed ticket -> agent acquire -> vmcnt wait ->
// barrier), so the hand-off does not rest on the sc1-load argument alone; the
// producers' sc1 payload + drain needs no release fence (MI355X_MICROARCH
// "Valid forms", Consumer (2)-(3)).  Measured on one box, alternating: fluA
// 4-draw call 103.8 / 103.8 us without / with, 1-draw 99.1 / 100.6, shard of 8
// 3,984 / 3,986 evals/s (profiles/r05_handoff_acquire_ab.txt) -- within noise,
// so it is the default; PHY_HANDOFF_ACQUIRE=0 at build time gives the
// sc1-only form.  tests/test_gpu_quad.py / test_gpu_class.py stress tests run
// 10^4 calls with rows compared bitwise, in one process.
#ifndef PHY_HANDOFF_ACQUIRE
#define PHY_HANDOFF_ACQUIRE 1
#endif
__device__ __forceinline__ void handoff_acquire(bool last) {
  if (PHY_HANDOFF_ACQUIRE && last) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate done before the barrier releases the others
  }
}

struct QfinArgs {
  FinArgs f;
  double* part;              // [draw][nspl][16 + C] hand-offs: M partial, sum_b b <G, QP> per category
  unsigned long long* cnt;   // [draw] tickets (modulo nspl; zeroed at allocation)
  int bper, nspl;
};
__global__ void __launch_bounds__(QFIN_THREADS) qfin_kernel(QfinArgs qa) {
  const FinArgs& a = qa.f;
  __shared__ double sV[16], sVi[16], sQ[16], srinv[16], slam[4];
  __shared__ double sinner[QFIN_ITEMS];
  __shared__ double wpart[QFIN_THREADS / 64][16];
  __shared__ double sred[8 * 16];
  __shared__ double sM[16];
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int sp = blockIdx.x, draw = blockIdx.y;
  const int C = a.C, B = a.B, bper = qa.bper, nspl = qa.nspl, gx = a.gx;
  const int b0 = sp * bper, nb = min(bper, B - b0);
  const bool qp = a.kind != PHY_JC69;
  const double* eg = a.eig + (size_t)draw * EIG_LEN;
  const double* mdl = a.model + (size_t)draw * (10 + 2 * C);
  const double* blv = a.blens + (size_t)draw * B;
  double* out = a.out + (size_t)draw * a.outlen;
  const int o = 1 + B + 2 * C;
  const int li = tid >> 2, k = tid & 3;
  const int c = li / bper, bl = li - c * bper;
  const bool live = c < C && bl < nb;  // quad-uniform
  const int b = b0 + (live ? bl : 0), idx = c * B + b, mm = a.gpos[b];
  // every global load of the item first (slots, P record), then the
  // eigensystem's staging barrier: one memory round trip, not three
  double2 lo[QFIN_SLOTS], hi[QFIN_SLOTS], p01[4], p23[4];
  if (live) {
    const size_t per_wg = (size_t)C * a.nmat * 16;
    const double* src = a.gslot + (size_t)draw * gx * per_wg + ((size_t)c * a.nmat + mm) * 16 + k * 4;
#pragma unroll
    for (int w = 0; w < QFIN_SLOTS; ++w)
      if (w < gx) {
        lo[w] = *reinterpret_cast<const double2*>(src + (size_t)w * per_wg);
        hi[w] = *reinterpret_cast<const double2*>(src + (size_t)w * per_wg + 2);
      }
    const double* P = a.pmat + ((size_t)draw * C * a.nmat + (size_t)c * a.nmat + mm) * a.R * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p01[j] = *reinterpret_cast<const double2*>(P + j * 4);
      p23[j] = *reinterpret_cast<const double2*>(P + j * 4 + 2);
    }
  }
  if (tid < 16) {
    sV[tid] = eg[EIG_M1 + tid];
    sVi[tid] = eg[EIG_M2 + tid];
    sQ[tid] = eg[EIG_Q + tid];
    const double lk = eg[EIG_LAM + (tid >> 2)], ll = eg[EIG_LAM + (tid & 3)];
    const double d = lk - ll;
    srinv[tid] = fabs(d) < 1e-12 * fmax(1.0, fabs(lk)) ? 0.0 : 1.0 / d;  // 0: tie (qgrad_body's rule)
    if (tid < 4) slam[tid] = eg[EIG_LAM + tid];
  }
  __syncthreads();
  double m[4] = {0.0, 0.0, 0.0, 0.0};
  if (live) {
    double r[4] = {lo[0].x, lo[0].y, hi[0].x, hi[0].y};
#pragma unroll
    for (int w = 1; w < QFIN_SLOTS; ++w)
      if (w < gx) {
        r[0] += lo[w].x;
        r[1] += lo[w].y;
        r[2] += hi[w].x;
        r[3] += hi[w].y;
      }
    double* grow = a.grows + (size_t)draw * a.grows_stride + (size_t)idx * 16 + k * 4;
    *reinterpret_cast<double2*>(grow) = make_double2(r[0], r[1]);
    *reinterpret_cast<double2*>(grow + 2) = make_double2(r[2], r[3]);
    // row k of <G, Q P> (FusedG's order), then the quad's sum
    double sv = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double qpv = fma(sQ[k * 4 + 3], p23[j].y,
                             fma(sQ[k * 4 + 2], p23[j].x, fma(sQ[k * 4 + 1], p01[j].y, sQ[k * 4] * p01[j].x)));
      sv = fma(r[j], qpv, sv);
    }
    sv += dpp_d<0xB1>(sv);  // quad_perm [1,0,3,2]
    sv += dpp_d<0x4E>(sv);  // quad_perm [2,3,0,1]
    if (k == 0) sinner[li] = sv;
    if (qp) {  // row k of this item's M term (qgrad_body's arithmetic)
      const double t = mdl[10 + c] * blv[b];
      const double Ek = exp(slam[k] * t);
      double E[4];
      E[0] = dpp_d<0x00>(Ek);
      E[1] = dpp_d<0x55>(Ek);
      E[2] = dpp_d<0xAA>(Ek);
      E[3] = dpp_d<0xFF>(Ek);
      double T[4];  // row k of V^T G
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double g0 = dpp_d<0x00>(r[j]), g1 = dpp_d<0x55>(r[j]), g2 = dpp_d<0xAA>(r[j]), g3 = dpp_d<0xFF>(r[j]);
        T[j] = fma(sV[12 + k], g3, fma(sV[8 + k], g2, fma(sV[4 + k], g1, fma(sV[k], g0, 0.0))));
      }
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        double hh = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) hh = fma(T[j], sVi[l * 4 + j], hh);
        const double ri = srinv[k * 4 + l];
        const double phi = ri == 0.0 ? t * Ek : (Ek - E[l]) * ri;
        m[l] = hh * phi;
      }
    }
  }
  // the wave's 16 quads (qgrad_body's butterfly), then the waves in order
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    swap32(m[u], m[u + 2]);
    m[u] += m[u + 2];
  }
  swap16(m[0], m[1]);
  m[0] += m[1];
  m[0] += dpp_d<DPP_ROW_ROR8>(m[0]);
  m[0] += dpp_d<0x124>(m[0]);
  if ((lane & 12) == 0) wpart[wave][k * 4 + ((lane >> 5) & 1) * 2 + ((lane >> 4) & 1)] = m[0];
  if (sp == 0 && tid < 8 * C) {  // scalar slots, in slot order (finalize_kernel's bits)
    const double* ss = a.sslot + (size_t)draw * gx * 8 * C + tid;
    double acc = ss[0];
    for (int w = 1; w < gx; ++w) acc += ss[(size_t)w * 8 * C];
    sred[tid] = acc;
  }
  __syncthreads();
  const double* rs = mdl + 10;
  if (tid < nb) {  // dlogL/db of the owned branches (finalize's order over c)
    double sv = 0.0;
    for (int cc = 0; cc < C; ++cc) sv = fma(rs[cc], sinner[cc * bper + tid], sv);
    out[1 + b0 + tid] = sv;
  }
  double* hp = qa.part + ((size_t)draw * nspl + sp) * (16 + C);
  if (tid >= 64 && tid < 80) {
    const int t = tid - 64;
    double acc = wpart[0][t];
    for (int w = 1; w < QFIN_THREADS / 64; ++w) acc += wpart[w][t];
    __hip_atomic_store(hp + t, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid >= 128 && tid < 128 + C) {
    const int cc = tid - 128;
    double acc = 0.0;
    for (int j = 0; j < nb; ++j) acc = fma(blv[b0 + j], sinner[cc * bper + j], acc);
    __hip_atomic_store(hp + 16 + cc, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (sp == 0 && tid == 0) {
    const double ll = sred[0];
    out[0] = isfinite(ll) ? ll : -INFINITY;
    for (int cc = 0; cc < C; ++cc) out[1 + B + C + cc] = sred[cc * 8 + 1];
    for (int f = 0; f < 4; ++f) {
      double t = 0.0;
      for (int cc = 0; cc < C; ++cc) t += sred[cc * 8 + 2 + f];
      __hip_atomic_store(out + o + f, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its write-through hand-offs
  __syncthreads();
  if (tid == 0) {
    const unsigned long long old = __hip_atomic_fetch_add(qa.cnt + draw, 1ull, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
    const bool last = ((old + 1) % (unsigned long long)nspl) == 0;
    handoff_acquire(last);
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  // the draw's last workgroup: every hand-off was stored sc1 and drained
  // before its ticket, and EVERY load of one here is an sc1 load (HANDOFF
  // note above handoff_acquire); the other loads read launch inputs
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const double* pp = qa.part + (size_t)draw * nspl * (16 + C);
  auto ld1 = [](const double* q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  if (tid < 16) {
    double u[8];  // 8 hand-offs in flight, summed in workgroup order
    double acc = 0.0;
    for (int q0 = 0; q0 < nspl; q0 += 8) {
#pragma unroll
      for (int v = 0; v < 8; ++v) u[v] = q0 + v < nspl ? ld1(pp + (size_t)(q0 + v) * (16 + C) + tid) : 0.0;
#pragma unroll
      for (int v = 0; v < 8; ++v)
        if (q0 + v < nspl) acc = (q0 + v == 0) ? u[v] : acc + u[v];
    }
    sM[tid] = acc;
  }
  if (tid >= 64 && tid < 64 + C) {
    const int cc = tid - 64;
    double u[8];
    double acc = 0.0;
    for (int q0 = 0; q0 < nspl; q0 += 8) {
#pragma unroll
      for (int v = 0; v < 8; ++v) u[v] = q0 + v < nspl ? ld1(pp + (size_t)(q0 + v) * (16 + C) + 16 + cc) : 0.0;
#pragma unroll
      for (int v = 0; v < 8; ++v)
        if (q0 + v < nspl) acc = (q0 + v == 0) ? u[v] : acc + u[v];
    }
    out[1 + B + cc] = acc;
  }
  if (!qp) {
    if (tid < 10) out[o + 4 + tid] = 0.0;
    return;
  }
  __syncthreads();
  if (tid < 16) wpart[0][tid] = w_entry(sM, sV, sVi, tid);
  __syncthreads();
  if (tid != 0) return;
  double W[16];
  for (int t = 0; t < 16; ++t) W[t] = wpart[0][t];
  const double rt[4] = {ld1(out + o), ld1(out + o + 1), ld1(out + o + 2), ld1(out + o + 3)};  // workgroup 0's
  q_tail(W, sQ, eg[EIG_S], mdl, rt, out + o);
}

}  // namespace

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
namespace {
struct ClassEngine;  // class_engine.inc
void free_class_engine(ClassEngine* e);
struct MultiState;  // multi_device.inc
void free_multi(MultiState* m);
}  // namespace

struct phy_ctx {
  int S, P, Ppad, C, B, rooted, kind, max_draws, device;
  int nsteps, nslots, ndeep, nblk, nmat;
  int R = 5;                     // 4-vectors per matrix record (4 columns + extra tip masks)
  unsigned long long extra = 0;  // the extra tip masks, 4 bits each
  int wg_budget, cols_pref, wg_cap, lds_budget;
  int cu_count = 256, wg_resident = 512;  // resident workgroups of the current plan
  int K = 1;                   // columns per lane of the current plan
  bool klat = false;           // K = 1 latency plan (sweep_kernel<512, 1, .>: no register spills)
  // the quad sweep (quad_engine.inc) for calls of <= QUAD_MAX_DRAWS draws
  bool quad_pref = true;       // PHY_QUAD=0: off
  // the multi-wave quad sweep (qmw_kernel): W waves per category share a block
  bool qmw_pref = true;        // PHY_QMW=0: the one-wave quad sweep
  bool qmw_ok = false;
  int qmw_W = 0, qmw_maxst = 0, qmw_nslot = 0, qmw_root = 0, qmw_nst[4] = {0, 0, 0, 0}, qmw_span = 0;
  size_t qmw_lds = 0;
  int* d_mprog = nullptr;
  bool quad_ok = false;        // its LDS plan fits
  size_t quad_lds = 0;
  int* d_qprog = nullptr;      // unpacked program, nothing rebuilt (every moved partial stored)
  double* d_qscr = nullptr;    // [wg][nslots][C][64]
  bool quad_build = false;     // this launch's quad sweep builds its matrix records (no pmat launch)
  double* d_qfpart = nullptr;  // qfin_kernel hand-offs [QUAD_MAX_DRAWS][nspl][16 + C]
  unsigned long long* d_qfcnt = nullptr;  // its tickets [QUAD_MAX_DRAWS]
  long qscr_wgs = 0;
  bool qfuse_pref = true;      // Q-parameter chain rule inside the sweep (PHY_QFUSE=0: off)
  int cap_m = 0, nchunks = 0;  // current LDS plan
  int deep_pref = 0;           // deep stack: 0 automatic, 1 LDS, 2 global
  bool deep_lds = false;       // current plan keeps the whole deep stack in LDS
  int ndl = 0;                 // deep entries in LDS (== ndeep when deep_lds)
  bool recompute = true;       // rebuild cherries in the reverse instead of storing them
  bool fin_pref = true;        // finalize inside the sweep when one workgroup runs a draw (PHY_FIN=0: off)
  int nrec = 0;                // cherries recomputed under the current plan
  // engine: 0 = pattern sweep (sweep_kernel; the quad sweep for small
  // calls), 1 = class sweep (site repeats, class_engine.inc);
  // engine_pref 0 = automatic, 1 = pattern, 2 = class
  int engine = 0, engine_pref = 0;
  ClassEngine* ce = nullptr;
  MultiState* ms = nullptr;  // a multi-device context (phy_create_multi): its shards do the work
  int compact = 0;             // output rows without the dL/dP block (phy_set_output)
  double* d_grows = nullptr;   // dL/dP rows when compact: [max_draws][16 C B]
  std::vector<uint8_t> h_tips;  // host copies of the static data (the class plan is built on demand)
  std::vector<double> h_w;
  std::vector<int32_t> h_peel;
  std::vector<int> vec_of, gpos;
  hipStream_t stream;
  // phy_eval_device on the legacy null stream: the context's stream waits for
  // the null stream's work (nin), the null stream for the evaluation (nout)
  hipEvent_t ev_nin = nullptr, ev_nout = nullptr;
  std::vector<int> prog;  // host copy of the program (chunk fields per plan)
  uint8_t* d_tips = nullptr;
  double* d_w = nullptr;
  int* d_prog = nullptr;
  int* d_gpos = nullptr;
  int* d_mat_branch = nullptr;
  double* d_pmat = nullptr;
  double* d_eig = nullptr;
  const double* eig_cur = nullptr;  // the eigensystems of the launch in flight: d_eig, or host-formed rows in d_in
  double* d_inner = nullptr;
  double* d_model = nullptr;
  double* d_blens = nullptr;
  double* d_out = nullptr;
  double* d_site = nullptr;
  // small host-buffer evaluations (phy_eval with n <= PIN_DRAWS): inputs packed
  // into one pinned staging buffer and one device buffer (one H2D copy), the
  // output rows back through pinned memory (asynchronous DMA both ways); the
  // eigensystems of up to 32 draws are formed on the host (stage_small) and ride along
  double* h_in = nullptr;   // pinned [PIN_DRAWS][B + model_len + EIG_LEN]
  double* h_out = nullptr;  // pinned [PIN_DRAWS][full output row]
  // the small path's kernel-side views of h_in / h_out when the kernels read
  // their operands from / write their rows to pinned host memory directly
  double* d_in = nullptr;   // device [PIN_DRAWS][B + model_len + EIG_LEN]
  int pending = 0;          // draws of a phy_eval_submit not yet collected by phy_eval_wait
  double2* d_scratch = nullptr;
  double2* d_dstk = nullptr;
  double* d_gslot = nullptr;
  double* d_sslot = nullptr;
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
  void* ptrs[] = {c->d_tips,  c->d_w,     c->d_prog,    c->d_gpos,    c->d_mat_branch, c->d_pmat,
                  c->d_eig,   c->d_inner, c->d_model,   c->d_blens,   c->d_out,        c->d_site,
                  c->d_scratch, c->d_dstk, c->d_gslot,  c->d_sslot, c->d_grows, c->d_in, c->d_qprog, c->d_qscr,
                  c->d_qfpart, c->d_qfcnt, c->d_mprog};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (c->h_in) (void)hipHostFree(c->h_in);
  if (c->h_out) (void)hipHostFree(c->h_out);
  for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
  if (c->ev_nin) (void)hipEventDestroy(c->ev_nin);
  if (c->ev_nout) (void)hipEventDestroy(c->ev_nout);
  free_class_engine(c->ce);
  free_multi(c->ms);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  (void)hipSetDevice(dev_old);
  delete c;
}

// Build the traversal program (DESIGN.md "Traversal program"): post-order
// with the child needing the deeper stack first (Strahler order), every
// stored moved partial in a slot (its step index), every branch matrix
// numbered in order of use, and the deep-stack entries.
//
// In this post-order the node computed just before v is v's second child y
// when y is internal, else its first child x when x is internal.  So a step
// pops `top` (the previous step's result) for y, and for x when y is a tip;
// only the first child x of a node whose children are both internal waits
// while y's subtree runs.  Those waits nest, so they live on a stack whose
// entry per wait is fixed here (ST_XDPOS / ST_VDPOS), used by both passes.
// Device layout of the program (see Step / ld_step): 8 packed ints per step.
std::vector<int> pack_program(const std::vector<int>& prog, bool unpacked = false) {
  if (unpacked) return prog;  // the K = 2 kernel's form
  const size_t n = prog.size() / STEP_INTS;
  std::vector<int> out(n * PSTEP, 0);
  auto h = [](int lo, int hi) { return (int)(((unsigned)(lo & 0xFFFF)) | ((unsigned)hi << 16)); };
  for (size_t s = 0; s < n; ++s) {
    const int* p = &prog[s * STEP_INTS];
    int* q = &out[s * PSTEP];
    q[0] = h(p[ST_X], p[ST_Y]);
    q[1] = h(p[ST_MX], p[ST_MY]);
    q[2] = h(p[ST_MV], p[ST_VSLOT]);
    q[3] = h(p[ST_XSLOT], p[ST_YSLOT]);
    q[4] = (int)((unsigned)(p[ST_FLAGS] & 0xFF) | ((unsigned)(p[ST_XDPOS] & 0xFF) << 8) |
                 ((unsigned)(p[ST_VDPOS] & 0xFF) << 16));
    q[5] = h(p[ST_CHUNK], p[ST_M0]);
    q[6] = h(p[ST_MN], p[ST_NODE]);
    q[7] = p[ST_RD];
  }
  return out;
}

int build_program(int S, const int32_t* peel, int rooted, std::vector<int>& prog,
                  std::vector<int>& mat_branch, int& nslots, int& ndeep) {
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
  // deep-stack need per subtree; larger-need child first (Strahler order)
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
  std::vector<int> slot(N, -1), parent(N, -1);
  for (int s = 0; s < S - 1; ++s) {
    if (steps[s] != root) slot[steps[s]] = s;
    parent[first[steps[s]]] = parent[second[steps[s]]] = steps[s];
  }
  nslots = S - 2;
  prog.assign((size_t)(S - 1) * STEP_INTS, -1);
  mat_branch.clear();
  std::vector<int> vdpos(N, -1);
  int cur = 0;
  ndeep = 0;
  for (int s = 0; s < S - 1; ++s) {
    const int v = steps[s];
    const int x = first[v], y = second[v];
    int* p = &prog[(size_t)s * STEP_INTS];
    p[ST_X] = x < S ? x : -1;
    p[ST_Y] = y < S ? y : -1;
    p[ST_MX] = p[ST_MY] = p[ST_MV] = -1;
    if (x < S) {  // tip children: their matrices are used at this step
      p[ST_MX] = (int)mat_branch.size();
      mat_branch.push_back(x);
    }
    if (y < S) {
      p[ST_MY] = (int)mat_branch.size();
      mat_branch.push_back(y);
    }
    int fl = 0;
    if (v != root && v != merged) {  // the step's own branch
      p[ST_MV] = (int)mat_branch.size();
      mat_branch.push_back(v);
      fl |= F_MV;
    }
    p[ST_VSLOT] = (v == root) ? -1 : slot[v];
    p[ST_XSLOT] = x >= S ? slot[x] : -1;
    p[ST_YSLOT] = y >= S ? slot[y] : -1;
    // operand sources (see the comment above), checked here
    if (y >= S && (s == 0 || steps[s - 1] != y)) return fail(PHY_EINVAL, "internal: y is not the previous step");
    if (x >= S && y < S && (s == 0 || steps[s - 1] != x))
      return fail(PHY_EINVAL, "internal: x is not the previous step");
    if (x >= S && y >= S) {
      fl |= F_XDEEP;
      if (vdpos[x] != cur - 1) return fail(PHY_EINVAL, "internal: deep stack out of order");
      p[ST_XDPOS] = vdpos[x];
      --cur;
    }
    if (v != root) {
      const int u = parent[v];
      if (first[u] == v && second[u] >= S) {  // waits for its sibling's subtree
        fl |= F_VDEEP;
        vdpos[v] = cur++;
        ndeep = std::max(ndeep, cur);
        p[ST_VDPOS] = vdpos[v];
      }
    }
    p[ST_FLAGS] = fl;
    p[ST_NODE] = v;
  }
  if (cur != 0) return fail(PHY_EINVAL, "internal: deep stack not empty");
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

#include "class_engine.inc"

constexpr size_t LDS_CAP = 160 * 1024;

constexpr int PIN_DRAWS = 128;  // phy_eval batches up to this size go through pinned staging
                                // (ADVI's elbo_samples = 100 fits: phylostan.py:47)
bool env_flag(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) != 0 : dflt != 0;
}
constexpr int MIN_CAP = 24;  // an occupancy level is taken only if chunks stay this large

int nblk_for(int P, int K) { return (P + WAVE * K - 1) / (WAVE * K); }
// The sweep instantiation of a plan: K columns per lane, deep stack in LDS.
// K = 1 has two register budgets: four waves per SIMD (1,024-thread
// workgroups, 128 VGPRs: spills) for wide launches with C > 8, and the
// sampler's latency plan (a few draws: at most one wave per SIMD is busy)
// at 256 VGPRs without spills (lat).
const void* sweep_kernel_ptr(int K, bool dl, bool lat) {
  if (K == 2) return dl ? (const void*)sweep_kernel<512, 2, true> : (const void*)sweep_kernel<512, 2, false>;
  if (lat) return dl ? (const void*)sweep_kernel<512, 1, true> : (const void*)sweep_kernel<512, 1, false>;
  return dl ? (const void*)sweep_kernel<1024, 1, true> : (const void*)sweep_kernel<1024, 1, false>;
}
int alloc_wg_buffers(phy_ctx* c, long cap);
int waves_per_simd(int K, bool lat) { return (K == 2 || lat) ? PHY_WPE2 : 4; }  // the kernel's register budget

// Columns per lane, matrices per LDS chunk and the chunk boundaries over the
// program.  Occupancy is bounded by registers (two waves per SIMD for K=2,
// four for K=1) and by LDS; the automatic plan takes the most workgroups
// per CU whose LDS share still holds chunks of >= MIN_CAP matrices (or the
// whole program).  An explicit budget (lds_budget) fixes the LDS share.
// A chunk holds >= 3 matrices (one step uses up to three).
int plan_chunks(phy_ctx* c) {
  // automatic: two columns per lane, unless even the one-column plan's
  // largest launch has at most one wave per SIMD (a sampler's few draws):
  // then nothing shares a SIMD, and one column per lane halves each wave's
  // step body (fluA, 4 draws: 182 -> 167 us per call; 100 draws: K = 2 stays
  // ahead, 220 against 235 us)
  int K = c->cols_pref;
  bool lat = false;
  if (!K) {
    K = c->C <= 8 ? 2 : 1;
    if (K == 2 && (long)c->max_draws * nblk_for(c->P, 1) * c->C <= 4L * c->cu_count) {
      K = 1;
      lat = true;
    }
  }
  if (K == 2 && c->C > 8) return fail(PHY_EINVAL, "two columns per lane need C <= 8");
  if ((size_t)std::max(c->nslots, c->ndeep) * K * 2 * c->C * WAVE * 16 >= (size_t)OOB)
    return fail(PHY_EINVAL, "per-workgroup scratch region too large for 32-bit buffer offsets");
  const int nb = nblk_for(c->P, K);
  int ndl = 0;  // deep-stack entries held in LDS
  auto cap_for = [&](size_t budget) {
    int cap = c->nmat;
    while (cap > 3 && lds_bytes(c->S, c->C, c->R, cap, K, ndl) > budget) --cap;
    return cap;
  };
  auto fits = [&](int cap, size_t budget) {
    return lds_bytes(c->S, c->C, c->R, cap, K, ndl) <= budget && cap >= std::min(c->nmat, MIN_CAP);
  };
  const int by_waves = std::max(1, 4 * waves_per_simd(K, lat) / c->C);  // workgroups per CU
  int cap = 0;
  // Deep-stack placement at a given LDS share: the whole stack in LDS if it
  // fits beside chunks of MIN_CAP matrices (mode 0/1), else (mode 0/2) its
  // outermost entries [0, ndl) in LDS and the rest in global memory, with
  // the largest ndl that still fits.
  auto place = [&](size_t budget, bool last) -> bool {
    if (c->deep_pref != 2) {
      ndl = c->ndeep;
      cap = cap_for(budget);
      if (fits(cap, budget) || (c->deep_pref == 1 && last)) return true;
      if (c->deep_pref == 1) return false;
    }
    for (ndl = c->ndeep - 1; ndl >= 0; --ndl) {
      if (c->deep_pref == 2) ndl = 0;
      cap = cap_for(budget);
      if (fits(cap, budget)) return true;
    }
    ndl = 0;
    cap = cap_for(budget);
    return false;
  };
  if (c->lds_budget > 0) {
    place(std::min<size_t>(LDS_CAP, (size_t)c->lds_budget), true);
  } else {
    // most workgroups per CU first
    for (int t = by_waves; t >= 1; --t)
      if (place(LDS_CAP / t, t == 1)) break;
  }
  const size_t lds = lds_bytes(c->S, c->C, c->R, cap, K, ndl);
  if (lds > LDS_CAP) return fail(PHY_EINVAL, "tree too large for LDS (tips of one block)");
  c->K = K;
  c->klat = lat;
  c->nblk = nb;
  c->wg_resident = c->cu_count * std::min<int>(by_waves, (int)(LDS_CAP / lds));
  {
    // workgroup regions the largest launch of this plan may use
    // (launch_pattern's gx per draw), grown here so no launch fails
    const long budget = c->wg_budget > 0 ? c->wg_budget : c->wg_resident;
    const long need = std::min<long>((long)c->max_draws * nb, budget + c->max_draws);
    if (need > c->wg_cap) {
      HIP_TRY(hipStreamSynchronize(c->stream));
      int rc = alloc_wg_buffers(c, need);
      if (rc) return rc;
      c->wg_cap = (int)need;
    }
  }
  // chunk boundaries: matrices are numbered in step order, so a chunk is a
  // run of steps whose matrices fit
  int used = 0, ch = 0, lo = 0;
  std::vector<int> first_step{0};
  for (int s = 0; s < c->nsteps; ++s) {
    const int* p = &c->prog[(size_t)s * STEP_INTS];
    const int n = (p[ST_MX] >= 0) + (p[ST_MY] >= 0) + (p[ST_MV] >= 0);
    if (used + n > cap) {
      first_step.push_back(s);
      lo += used;
      used = 0;
      ++ch;
    }
    int* q = &c->prog[(size_t)s * STEP_INTS];
    q[ST_CHUNK] = ch;
    q[ST_M0] = lo;
    used += n;
  }
  if (lo + used != c->nmat) return fail(PHY_EINVAL, "internal: chunk plan does not cover the matrices");
  first_step.push_back(c->nsteps);
  for (int k = 0; k <= ch; ++k) {
    const int m0 = c->prog[(size_t)first_step[k] * STEP_INTS + ST_M0];
    const int m1 = (k < ch) ? c->prog[(size_t)first_step[k + 1] * STEP_INTS + ST_M0] : c->nmat;
    for (int s = first_step[k]; s < first_step[k + 1]; ++s) c->prog[(size_t)s * STEP_INTS + ST_MN] = m1 - m0;
  }
  // rebuilt chains (F_NOSTORE / F_PREVREC / ST_RD), valid for this chunk plan:
  // step s's previous-step child q is rebuilt at depth d when q is a cherry
  // (d = 1) or has one tip child and itself rebuilds its previous-step child
  // at depth d-1, and steps s-d..s share one LDS chunk
  c->nrec = 0;
  for (int s = 0; s < c->nsteps; ++s) {
    c->prog[(size_t)s * STEP_INTS + ST_FLAGS] &= ~(F_NOSTORE | F_PREVREC);
    c->prog[(size_t)s * STEP_INTS + ST_RD] = 0;
  }
  if (c->recompute) {
    for (int s = 1; s < c->nsteps; ++s) {
      int* p = &c->prog[(size_t)s * STEP_INTS];
      int* q = &c->prog[(size_t)(s - 1) * STEP_INTS];
      const bool has_internal = p[ST_X] < 0 || p[ST_Y] < 0;  // then step s-1 is its top child
      const bool eligible = (q[ST_FLAGS] & F_MV) && q[ST_VSLOT] >= 0 && !(q[ST_FLAGS] & F_VDEEP);
      if (!has_internal || !eligible) continue;
      int d = 0;
      if (q[ST_X] >= 0 && q[ST_Y] >= 0) d = 1;
      else if ((q[ST_X] >= 0) != (q[ST_Y] >= 0) && q[ST_RD] > 0) d = q[ST_RD] + 1;
      if (d == 0 || d > RD_MAX || s - d < 0) continue;
      bool same = true;
      for (int j = 1; j <= d; ++j) same = same && c->prog[(size_t)(s - j) * STEP_INTS + ST_CHUNK] == p[ST_CHUNK];
      if (!same) continue;
      q[ST_FLAGS] |= F_NOSTORE;
      p[ST_FLAGS] |= F_PREVREC;
      p[ST_RD] = d;
      ++c->nrec;
    }
  }
  {
    const std::vector<int> packed = pack_program(c->prog, K == 2);
    HIP_TRY(hipMemcpy(c->d_prog, packed.data(), packed.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  c->cap_m = cap;
  c->nchunks = ch + 1;
  c->deep_lds = ndl > 0 && ndl == c->ndeep;
  c->ndl = ndl;
  return PHY_OK;
}

// Engine choice.  Pattern sweep (sweep_kernel) or class sweep
// (class_engine.inc).  Automatic: the class plan is built only for large
// alignments (P >= 16384 patterns) and kept when its non-root classes are at
// most a quarter of the (node, pattern) work of the pattern sweep -- e.g. the
// synthetic 128 x 1M workload (1.16M classes vs 66.5M); the small configs
// (fluA / HCV / DS1, batched over draws) stay on the pattern sweep.
int ensure_class_plan(phy_ctx* c) {
  if (c->ce) return PHY_OK;
  return build_class_engine(c->S, c->P, c->C, c->rooted, c->h_tips.data(), c->h_w.data(), c->h_peel.data(),
                            c->vec_of, c->R, c->nmat, c->gpos, &c->ce);
}

int select_engine(phy_ctx* c) {
  c->engine = 0;
  if (c->engine_pref == 1) return PHY_OK;
  if (c->engine_pref == 0 && c->P < 16384) return PHY_OK;
  int rc = ensure_class_plan(c);
  if (rc) return rc;
  const double pattern_work = (double)(c->S - 2) * c->P;
  if (c->engine_pref == 2 || (double)c->ce->classes <= 0.25 * pattern_work) {
    c->engine = 1;
  } else {
    free_class_engine(c->ce);
    c->ce = nullptr;
  }
  return PHY_OK;
}

// HIP events around the timed part of one launch (phy_timing_start)
int timing_begin(phy_ctx* ctx, hipStream_t st, hipEvent_t* e0, hipEvent_t* e1) {
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
  *e0 = ctx->ev[ctx->ev_used];
  *e1 = ctx->ev[ctx->ev_used + 1];
  ctx->ev_used += 2;
  HIP_TRY(hipEventRecord(*e0, st));
  return PHY_OK;
}

bool launch_finalize(FinArgs fa, int n, hipStream_t st);

// The class sweep (class_engine.inc): forward levels, root, reverse levels,
// then the ordered dL/dP sums and the shared finalize.  The timed region
// (phy_timing_*) spans the forward through the last reverse level.
int launch_class(phy_ctx* ctx, int n, const double* d_blens, const double* d_model, double* d_out,
                 double* d_site, hipStream_t st, double* grows, long long gstride, bool* qdone) {
  ClassEngine* e = ctx->ce;
  const int C = ctx->C, B = ctx->B;
  if ((long)n * C > 65535) return fail(PHY_ERANGE, "class sweep: n_draws * C must be <= 65535");
  int rc = class_engine_reserve(e, n, st);
  if (rc) return rc;
  ClassArgs a = class_args(e, ctx->d_pmat, d_model, ctx->extra);
  const int dcn = n * C;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (ctx->timing && (rc = timing_begin(ctx, st, &e0, &e1))) return rc;
  if (e->Lc > 0)  // levels 1..Lc: one workgroup per (bottom clade, dc)
    hipLaunchKernelGGL(cls_clade_fwd_kernel, dim3(e->nclade, dcn), dim3(CLADE_THREADS), 0, st, a,
                       (const CladeLevel*)e->d_clade, e->Lc);
  const bool chain = e->chain_m > 0;
  const ChainArgs ca{e->d_link, e->d_ctab, e->d_crep, e->chain_m, e->chain_ntop, e->chain_ntp, e->chain_toff};
  const int chain_wgs = (e->chain_ntp / WAVE + CLS_WPG - 1) / CLS_WPG;
  auto in_chain = [&](int l) { return chain && l >= e->chain_lo && l <= e->chain_hi; };
  for (int l = e->Lc + 1; l < e->levels; ++l) {
    const ClassLevel& L = e->lv[l];
    if (!L.nchunk || in_chain(l) || L.pair == 2) continue;
    a.first = L.chunk0;
    a.count = L.nchunk;
    if (L.pair == 1) {  // this level and the next (its chunks follow): cls_fwd2_kernel
      a.count += e->lv[l + 1].nchunk;
      hipLaunchKernelGGL(cls_fwd2_kernel, dim3((a.count + CLS_WPG - 1) / CLS_WPG, dcn), dim3(CLS_THREADS), 0, st, a,
                         (const int2*)e->d_pair, (const int4*)e->d_gc);
      continue;
    }
    hipLaunchKernelGGL(cls_fwd_kernel, dim3((L.nchunk + CLS_WPG - 1) / CLS_WPG, dcn), dim3(CLS_THREADS), 0, st, a);
  }
  // the root recomputes the chain's top (cls_root_kernel<·, ·, MC>) instead of
  // a chain forward launch storing it (PHY_ROOT_CHAIN=0 at phy_create: the launch)
  const bool root_chain = chain && C <= 4 && e->root_chain_pref;
  if (chain && !root_chain)  // levels lo..hi in one launch
    hipLaunchKernelGGL(e->chain_m <= 4 ? cls_chain_fwd_kernel<4> : e->chain_m == 5 ? cls_chain_fwd_kernel<5>
                       : e->chain_m <= 6 ? cls_chain_fwd_kernel<6> : cls_chain_fwd_kernel<CHAIN_MAX>,
                       dim3(chain_wgs, dcn), dim3(CLS_THREADS), 0, st, a, ca);
  auto rk = C <= 4 ? (e->root_tips ? cls_root_kernel<256, true> : cls_root_kernel<256, false>)
                   : (e->root_tips ? cls_root_kernel<1024, true> : cls_root_kernel<1024, false>);
  if (root_chain) {
    const int m = e->chain_m;
    rk = e->root_tips ? (m <= 4 ? cls_root_kernel<256, true, 4> : m == 5 ? cls_root_kernel<256, true, 5>
                         : m <= 6 ? cls_root_kernel<256, true, 6> : cls_root_kernel<256, true, CHAIN_MAX>)
                      : (m <= 4 ? cls_root_kernel<256, false, 4> : m == 5 ? cls_root_kernel<256, false, 5>
                         : m <= 6 ? cls_root_kernel<256, false, 6> : cls_root_kernel<256, false, CHAIN_MAX>);
  }
  hipLaunchKernelGGL(rk, dim3(e->nrootch, n), dim3(C * WAVE), 0, st, a, ca);
  for (int l = e->levels - 1; l > e->Lc; --l) {
    const ClassLevel& L = e->lv[l];
    if (L.ntile) {
      a.first = L.tile0;
      a.count = L.ntile;
      a.sfirst = L.sec0;
      a.sord = L.sord;
      hipLaunchKernelGGL(cls_red_kernel, dim3((L.ntile + CLS_WPG - 1) / CLS_WPG, dcn), dim3(CLS_THREADS), 0, st, a);
    }
    if (L.nlfix && !L.revfix)  // the level's long spans (the short ones are summed by the REV lanes)
      hipLaunchKernelGGL(cls_fix_list_kernel, dim3((L.nlfix + CLS_WPG - 1) / CLS_WPG, dcn), dim3(CLS_THREADS), 0, st, a,
                         (const int*)e->d_lfix + L.lfix0, L.nlfix);
    if (in_chain(l)) {  // the chain's levels: one reverse launch at its top (levels below hold no staged tiles)
      if (l == e->chain_hi)
        hipLaunchKernelGGL(e->chain_m <= 4 ? cls_chain_rev_kernel<4> : e->chain_m == 5 ? cls_chain_rev_kernel<5>
                           : e->chain_m <= 6 ? cls_chain_rev_kernel<6> : cls_chain_rev_kernel<CHAIN_MAX>,
                           dim3(chain_wgs, dcn), dim3(CLS_THREADS), 0, st, a, ca);
      continue;
    }
    if (L.nchunk) {
      a.first = L.chunk0;
      a.count = L.nchunk;
      if (L.revfix)  // ... the long ones by the chunks' waves
        hipLaunchKernelGGL(cls_rev_ls_kernel, dim3((L.nchunk + CLS_WPG - 1) / CLS_WPG, dcn), dim3(CLS_THREADS), 0, st, a,
                           (const int2*)e->d_clf, (const int*)e->d_clong);
      else
        hipLaunchKernelGGL(cls_rev_kernel, dim3((L.nchunk + CLS_WPG - 1) / CLS_WPG, dcn), dim3(CLS_THREADS), 0, st, a);
    }
  }
  if (e->Lc > 0) {
    if (e->nrtile)
      hipLaunchKernelGGL(cls_red_list_kernel, dim3((e->nrtile + CLS_WPG - 1) / CLS_WPG, dcn), dim3(CLS_THREADS), 0, st, a,
                         (const int*)e->d_rtile, e->nrtile);
    if (e->nrspan)
      hipLaunchKernelGGL(cls_fix_list_kernel, dim3((e->nrspan + CLS_WPG - 1) / CLS_WPG, dcn), dim3(CLS_THREADS), 0, st, a,
                         (const int*)e->d_rspan, e->nrspan);
    hipLaunchKernelGGL(cls_clade_rev_kernel, dim3(e->nclade, dcn), dim3(CLADE_THREADS), 0, st, a,
                       (const CladeLevel*)e->d_clade, e->Lc);
  }
  HIP_TRY(hipGetLastError());
  if (ctx->timing) HIP_TRY(hipEventRecord(e1, st));
  if (d_site)
    hipLaunchKernelGGL(cls_site_kernel, dim3((ctx->P + 255) / 256, n), dim3(256), 0, st,
                       (const double*)e->d_sitecls, (const int*)e->d_pat_root, d_site, ctx->P, e->nroot);
  double* epi = e->d_epi;
  const size_t ncb = (size_t)n * C * B;
  if (e->nsub)  // the long branches' partial rows in sub-ranges first
    hipLaunchKernelGGL(cls_gsum_kernel, dim3(e->nsub, dcn), dim3(256), 0, st, (const double*)e->d_gpart,
                       (const int2*)e->d_gsub, e->d_gpsum, std::max(e->ngs, 1), e->nsub);
  EpiArgs ea{e->d_gpart, e->d_gbase, e->d_gcount, e->d_sslot, ctx->d_pmat, ctx->eig_cur, d_blens, d_model,
             ctx->d_gpos, grows, gstride, d_out, epi, epi + ncb, epi + 17 * ncb,
             C, B, ctx->nmat, ctx->R, std::max(e->ngs, 1), e->nrootch, phy_output_len(ctx), ctx->kind,
             e->d_gpsum, e->d_pbase, std::max(e->nsub, 1)};
  // the per-item part (every workgroup resident at once), then the closing part
  hipLaunchKernelGGL((cls_epi_kernel<EPI_WIDE_THREADS, 1>), dim3(C * B, n), dim3(EPI_WIDE_THREADS), 0, st, ea);
  hipLaunchKernelGGL((cls_epi_kernel<EPI_THREADS, 2>), dim3(n), dim3(EPI_THREADS), 0, st, ea);
  *qdone = true;
  HIP_TRY(hipGetLastError());
  return PHY_OK;
}

int launch_pattern(phy_ctx* ctx, int n, const double* d_blens, const double* d_model, double* d_out,
                   double* d_site, hipStream_t st, double* grows, long long gstride, bool* qdone = nullptr);
// the pattern engine takes the quad sweep for this call (launch_pattern)
bool quad_applies(const phy_ctx* ctx, int n) {
  return ctx->quad_ok && ctx->quad_pref && ctx->cols_pref == 0 && n <= QUAD_MAX_DRAWS;
}

// Returns whether the finalize ran the Q-parameter chain rule too: when its
// LDS ([C][B] inner products, Q, the reduction rows and the chain rule's
// QG_SHARED) would pass the 160 KiB cap the chain rule is left to
// qgrad_kernel (large C*B; finalize_kernel is opted into LDS_CAP at
// phy_create, and phy_create refuses a C*B whose finalize alone cannot fit).
bool launch_finalize(FinArgs fa, int n, hipStream_t st) {
  const int threads = 1024;
  const size_t base = (size_t)fa.C * fa.B + 16 + threads;
  if (fa.qf && (base + QG_SHARED) * sizeof(double) > LDS_CAP) fa.qf = 0;
  hipLaunchKernelGGL(finalize_kernel, dim3(n), dim3(threads), (base + (fa.qf ? QG_SHARED : 0)) * sizeof(double), st,
                     fa);
  return fa.qf != 0;
}

int launch(phy_ctx* ctx, int n, const double* d_blens, const double* d_model, double* d_out,
           double* d_site, hipStream_t st, const double* d_eig_in = nullptr) {
  const int C = ctx->C, B = ctx->B;
  ctx->eig_cur = d_eig_in ? d_eig_in : ctx->d_eig;
  // the quad sweep builds its own records when the eigensystems are given
  ctx->quad_build = d_eig_in && ctx->engine == 0 && quad_applies(ctx, n);
  if (!ctx->quad_build) {
    // eigensystems: given (host-formed, the small host-buffer path); small
    // device batches: each pmat wave forms its draw's (one launch less);
    // large ones: one thread per draw first
    const int with_eig = (!d_eig_in && n <= EIG_FUSE_MAX) ? 1 : 0;
    PmatArgs pa{d_model, d_blens, ctx->d_mat_branch, const_cast<double*>(ctx->eig_cur), ctx->d_pmat, C, B, ctx->kind,
                ctx->nmat, n, ctx->R, ctx->extra, with_eig};
    if (!with_eig && !d_eig_in) {
      hipLaunchKernelGGL(eig_kernel, dim3((n + 63) / 64), dim3(64), 0, st, pa);
      HIP_TRY(hipGetLastError());
    }
    const dim3 pgrid((C * ctx->nmat + PMAT_WAVE_RECS - 1) / PMAT_WAVE_RECS, n);
    const size_t plds = (size_t)PMAT_WAVE_RECS * ctx->R * 4 * sizeof(double);
    if (with_eig)
      hipLaunchKernelGGL(pmat_kernel<true>, pgrid, dim3(64), plds, st, pa);
    else
      hipLaunchKernelGGL(pmat_kernel<false>, pgrid, dim3(64), plds, st, pa);
    HIP_TRY(hipGetLastError());
  }
  double* grows = ctx->compact ? ctx->d_grows : d_out + PHY_OUT_G(B, C);
  const long long gstride = ctx->compact ? (long long)16 * C * B : (long long)phy_output_len(ctx);
  // the chain rule runs inside the sweep (one workgroup per draw) or the
  // finalize kernel unless PHY_QFUSE=0
  bool qdone = false;
  int rc0 = ctx->engine == 1 ? launch_class(ctx, n, d_blens, d_model, d_out, d_site, st, grows, gstride, &qdone)
                             : launch_pattern(ctx, n, d_blens, d_model, d_out, d_site, st, grows, gstride, &qdone);
  if (rc0) return rc0;
  if (!qdone) {
    FinArgs qa{ctx->d_gslot, ctx->d_sslot, ctx->d_pmat, ctx->eig_cur, d_blens, d_model, ctx->d_gpos, ctx->d_inner,
               d_out,        C,            B,           ctx->nmat,   1,       phy_output_len(ctx), 0, ctx->R, grows,
               gstride,      ctx->kind};
    hipLaunchKernelGGL(qgrad_kernel, dim3(n), dim3(QG_THREADS), 0, st, qa);
    HIP_TRY(hipGetLastError());
  }
  return PHY_OK;
}

// The quad sweep (quad_engine.inc) for a small call: one workgroup of C
// waves per 16-column block and draw, as many blocks per workgroup as keep
// the launch within one wave per SIMD; then the pattern sweep's epilogue
// (slot sums, finalize, chain rule).
int launch_quad(phy_ctx* ctx, int n, const double* d_blens, const double* d_model, double* d_out, double* d_site,
                hipStream_t st, double* grows, long long gstride, bool* qdone) {
  const int C = ctx->C, B = ctx->B;
  const int nb = (ctx->P + QCOLS - 1) / QCOLS;
  const int gx = std::max(1, std::min(nb, (4 * ctx->cu_count) / (C * n)));
  const long wgs = (long)gx * n;
  if (wgs > ctx->wg_cap || wgs > ctx->qscr_wgs) {  // grown once per context (the sampler's call size)
    HIP_TRY(hipDeviceSynchronize());
    if (wgs > ctx->wg_cap) {
      int rc = alloc_wg_buffers(ctx, wgs);
      if (rc) return rc;
      ctx->wg_cap = (int)wgs;
    }
    if (wgs > ctx->qscr_wgs) {
      if (ctx->d_qscr) (void)hipFree(ctx->d_qscr);
      ctx->d_qscr = nullptr;
      ctx->qscr_wgs = 0;
      int rc = dalloc(&ctx->d_qscr, (size_t)wgs * std::max(ctx->nslots, 1) * C * WAVE);
      if (rc) return rc;
      ctx->qscr_wgs = wgs;
    }
  }
  // the split epilogue (qfin_kernel): items of bper branches x C categories per workgroup
  const int bper = std::max(1, std::min((B + 15) / 16, QFIN_ITEMS / C));
  const int nspl = (B + bper - 1) / bper;
  if (!ctx->d_qfcnt) {  // once per context: hand-offs and zeroed tickets for QUAD_MAX_DRAWS draws
    HIP_TRY(hipDeviceSynchronize());
    int rc = dalloc(&ctx->d_qfpart, (size_t)QUAD_MAX_DRAWS * nspl * (16 + C));
    if (!rc) rc = dalloc(&ctx->d_qfcnt, (size_t)QUAD_MAX_DRAWS);
    if (rc) return rc;
    HIP_TRY(hipMemset(ctx->d_qfcnt, 0, (size_t)QUAD_MAX_DRAWS * sizeof(unsigned long long)));
    HIP_TRY(hipDeviceSynchronize());
  }
  QuadArgs qa;
  qa.s = SweepArgs{ctx->d_tips,  ctx->d_w,     ctx->d_pmat,  d_model,      ctx->d_scratch, ctx->d_dstk,
                   ctx->d_gslot, ctx->d_sslot, d_site,       d_out,        ctx->d_mat_branch, ctx->eig_cur,
                   ctx->d_inner, ctx->S,       ctx->P,       ctx->Ppad,    C,              ctx->nsteps,
                   ctx->nslots,  ctx->ndeep,   0,            ctx->nblk,    ctx->nmat,    ctx->R,         ctx->nmat,
                   B,            phy_output_len(ctx), 0, ctx->extra, 0, d_blens, grows, gstride, 0, ctx->kind};
  qa.qscr = ctx->d_qscr;
  qa.nblk = nb;
  qa.pmat_out = ctx->d_pmat;
  qa.build = ctx->quad_build ? 1 : 0;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (ctx->timing) {
    int rc = timing_begin(ctx, st, &e0, &e1);
    if (rc) return rc;
  }
  {
    if (ctx->qmw_ok && ctx->qmw_pref) {  // W waves per category
      QmwArgs ma{qa, ctx->d_mprog, ctx->qmw_W, ctx->qmw_maxst, ctx->qmw_nslot, ctx->qmw_root,
                 ctx->qmw_nst[0], ctx->qmw_nst[1], ctx->qmw_nst[2], ctx->qmw_nst[3]};
      void* kargs[] = {(void*)&ma};
      HIP_TRY(hipLaunchKernel((const void*)qmw_kernel, dim3(gx, n), dim3(C * ctx->qmw_W * WAVE), kargs, ctx->qmw_lds,
                              st));
    } else {
      const int* prog = ctx->d_qprog;
      void* kargs[] = {(void*)&qa, (void*)&prog};
      const void* kern = C <= 4 ? (const void*)qsweep_kernel<256> : (const void*)qsweep_kernel<1024>;
      HIP_TRY(hipLaunchKernel(kern, dim3(gx, n), dim3(C * WAVE), kargs, ctx->quad_lds, st));
    }
  }
  HIP_TRY(hipGetLastError());
  if (ctx->timing) HIP_TRY(hipEventRecord(e1, st));
  const int gsum_in = gx <= 16 ? 1 : 0;
  FinArgs fa{ctx->d_gslot, ctx->d_sslot, ctx->d_pmat, ctx->eig_cur, d_blens, d_model, ctx->d_gpos, ctx->d_inner, d_out,
             C,            B,            ctx->nmat,   gx,          phy_output_len(ctx), 0, ctx->R, grows, gstride,
             ctx->kind,    gsum_in,      ctx->qfuse_pref ? 1 : 0};
  if (gx <= QFIN_SLOTS && C * bper <= QFIN_ITEMS && 8 * C <= 128 && ctx->qfuse_pref) {
    hipLaunchKernelGGL(qfin_kernel, dim3(nspl, n), dim3(QFIN_THREADS), 0, st,
                       QfinArgs{fa, ctx->d_qfpart, ctx->d_qfcnt, bper, nspl});
    HIP_TRY(hipGetLastError());
    *qdone = true;
    return PHY_OK;
  }
  if (!gsum_in) {
    hipLaunchKernelGGL(gsum_kernel, dim3((C * B * 16 + 63) / 64, n), dim3(256), 0, st, fa);
    HIP_TRY(hipGetLastError());
  }
  *qdone = launch_finalize(fa, n, st);
  HIP_TRY(hipGetLastError());
  return PHY_OK;
}

// The pattern sweep (sweep_kernel) and its dL/dP sums / finalize.
int launch_pattern(phy_ctx* ctx, int n, const double* d_blens, const double* d_model, double* d_out,
                   double* d_site, hipStream_t st, double* grows, long long gstride, bool* qdone) {
  const int C = ctx->C, B = ctx->B;
  // (an explicit column plan, phy_set_tuning(cols > 0), keeps the one / two column sweeps)
  if (quad_applies(ctx, n) && qdone)
    return launch_quad(ctx, n, d_blens, d_model, d_out, d_site, st, grows, gstride, qdone);
  // persistent workgroups: the explicit budget, else exactly what is resident
  const int budget = ctx->wg_budget > 0 ? ctx->wg_budget : ctx->wg_resident;
  // (at most one workgroup per block, so every workgroup has a block to write its slots)
  const int gx = std::max(1, std::min(ctx->nblk, (budget + n - 1) / n));
  if ((size_t)gx * n > (size_t)ctx->wg_cap) return fail(PHY_ERANGE, "workgroup cap exceeded");
  const size_t lds = lds_bytes(ctx->S, C, ctx->R, ctx->cap_m, ctx->K, ctx->ndl);
  const int g_direct = (gx == 1) ? 1 : 0;
  // finalize inside the sweep when its LDS holds [C][B] + [C][8] doubles
  // past the tips; the chain rule too when QG_SHARED more fit
  const size_t room = lds - tip_nib_bytes(ctx->S, ctx->K) - 16 * 4 * sizeof(double);
  const int fin = (g_direct && ctx->fin_pref && ((size_t)C * B + 8 * C) * 8 <= room) ? 1 : 0;
  const int qf = (fin && ctx->qfuse_pref && ((size_t)C * B + 8 * C + QG_SHARED) * 8 <= room) ? 1 : 0;
  SweepArgs sa{ctx->d_tips,  ctx->d_w,     ctx->d_pmat,  d_model,      ctx->d_scratch, ctx->d_dstk,
               ctx->d_gslot, ctx->d_sslot, d_site,       d_out,        ctx->d_mat_branch, ctx->eig_cur,
               ctx->d_inner, ctx->S,       ctx->P,       ctx->Ppad,    C,              ctx->nsteps,
               ctx->nslots,  ctx->ndeep,   ctx->ndl,     ctx->nblk,    ctx->nmat,    ctx->R,         ctx->cap_m,
               B,            phy_output_len(ctx), g_direct, ctx->extra, fin, d_blens, grows, gstride,
               qf,           ctx->kind};
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (ctx->timing) {
    int rc = timing_begin(ctx, st, &e0, &e1);
    if (rc) return rc;
  }
  const int threads = C * WAVE;
  const void* kern = sweep_kernel_ptr(ctx->K, ctx->deep_lds, ctx->klat);
  {
    const int* prog = ctx->d_prog;
    void* kargs[] = {(void*)&sa, (void*)&prog};
    HIP_TRY(hipLaunchKernel(kern, dim3(gx, n), dim3(threads), kargs, lds, st));
  }
  HIP_TRY(hipGetLastError());
  if (ctx->timing) HIP_TRY(hipEventRecord(e1, st));
  // a draw over a few workgroups: the finalize sums their slots itself
  // (one epilogue launch: slot sums, finalize, chain rule); over many, the
  // wide gsum kernel first
  const int gsum_in = (!g_direct && gx <= 16) ? 1 : 0;
  FinArgs fa{ctx->d_gslot, ctx->d_sslot, ctx->d_pmat, ctx->eig_cur, d_blens, d_model, ctx->d_gpos, ctx->d_inner, d_out,
             C,            B,            ctx->nmat,   gx,          phy_output_len(ctx), g_direct, ctx->R, grows, gstride,
             ctx->kind,    gsum_in,      (!fin && ctx->qfuse_pref) ? 1 : 0};
  if (!g_direct && !gsum_in) {
    hipLaunchKernelGGL(gsum_kernel, dim3((C * B * 16 + 63) / 64, n), dim3(256), 0, st, fa);
    HIP_TRY(hipGetLastError());
  }
  bool fq = false;
  if (!fin) {
    fq = launch_finalize(fa, n, st);
    HIP_TRY(hipGetLastError());
  }
  if (qdone) *qdone = qf != 0 || fq;
  return PHY_OK;
}

// Per-workgroup regions of the pattern sweep for `cap` workgroup slots:
// moved-partial scratch, global deep entries, dL/dP and scalar slots.  The
// new regions are allocated first and swapped in only when all four
// succeed, so a failed grow leaves the context's current regions (and its
// wg_cap) valid.
int alloc_wg_buffers(phy_ctx* c, long cap) {
  const size_t ncolwg = (size_t)c->C * WAVE;
  double2 *scr = nullptr, *dsk = nullptr;
  double *gsl = nullptr, *ssl = nullptr;
  int rc = dalloc(&scr, (size_t)cap * std::max(c->nslots, 1) * 2 * 2 * ncolwg);
  if (!rc) rc = dalloc(&dsk, (size_t)cap * std::max(c->ndeep, 1) * 2 * 2 * ncolwg);
  if (!rc) rc = dalloc(&gsl, (size_t)cap * c->C * c->nmat * 16);
  if (!rc) rc = dalloc(&ssl, (size_t)cap * c->C * 8);
  if (rc) {
    const std::string msg = g_err;
    void* ps[] = {scr, dsk, gsl, ssl};
    for (void* p : ps)
      if (p) (void)hipFree(p);
    return fail(rc, msg);
  }
  void* old[] = {c->d_scratch, c->d_dstk, c->d_gslot, c->d_sslot};
  for (void* p : old)
    if (p) (void)hipFree(p);
  c->d_scratch = scr;
  c->d_dstk = dsk;
  c->d_gslot = gsl;
  c->d_sslot = ssl;
  return PHY_OK;
}

// The small host-buffer path's staging: blens, model vectors and the draws'
// eigensystems (eig_record on the host: the same operations in the same
// order as eig_kernel and the C oracle, with no FMA contraction, so the same
// bits; formed on the device by one lane per pmat wave they took 13 us of a
// 4-draw fluA call -- a serial chain of divisions and square roots) packed
// for one H2D copy.  Up to EIG_HOST_MAX draws (the host takes ~0.6 us per
// draw; measured per call: fluA 32 draws 175 us host-formed against 186-199
// device-formed, 100 draws 207-210 device-formed against 237-242): beyond
// that eig_kernel forms them, one thread per draw.
// Returns the doubles to copy; *host_eig says whether they include the
// eigensystems.
constexpr int EIG_HOST_MAX = 32;
size_t stage_small(phy_ctx* ctx, int n, const double* blens, const double* model, bool* host_eig) {
  const int ml = 10 + 2 * ctx->C;
  const size_t nb = (size_t)n * ctx->B, nm = (size_t)n * ml;
  std::memcpy(ctx->h_in, blens, sizeof(double) * nb);
  std::memcpy(ctx->h_in + nb, model, sizeof(double) * nm);
  *host_eig = n <= EIG_HOST_MAX;
  if (!*host_eig) return nb + nm;
  double* eg = ctx->h_in + nb + nm;
  for (int d = 0; d < n; ++d) eig_record(model + (size_t)d * ml, ctx->kind, eg + (size_t)d * EIG_LEN);
  return nb + nm + (size_t)n * EIG_LEN;
}

}  // namespace

// Work of `body(st)` on ctx's stream, fenced both ways with the legacy null
// stream (stream handle 0): ordered after everything queued on it before the
// call, and everything queued on it after the call waits for it.
template <typename F>
int null_fenced(phy_ctx* ctx, F&& body) {
  HIP_TRY(hipEventRecord(ctx->ev_nin, nullptr));
  HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_nin, 0));
  const int rc = body(ctx->stream);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(ctx->ev_nout, ctx->stream));
  HIP_TRY(hipStreamWaitEvent(nullptr, ctx->ev_nout, 0));
  return PHY_OK;
}

#include "multi_device.inc"

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
  int rc = build_program(S, peel, c->rooted, c->prog, mat_branch, c->nslots, c->ndeep);
  if (rc) {
    delete c;
    return rc;
  }
  c->nsteps = S - 1;
  c->nmat = (int)mat_branch.size();
  if (S > 16000 || c->ndeep > 127) {  // the packed device program's field widths
    delete c;
    return fail(PHY_EINVAL, "tree too large for the packed program (S <= 16000, deep stack <= 127)");
  }
  // matrix records: 4 columns + P t for every non-one-hot mask t in the data
  // (15 always: the padding patterns' mask)
  std::vector<int> vec_of(16, -1);
  {
    bool present[16] = {false};
    for (size_t k = 0; k < (size_t)S * P; ++k) present[tipcodes[k]] = true;
    present[15] = true;
    for (int j = 0; j < 4; ++j) vec_of[1 << j] = j;
    int R = 4;
    for (int t = 0; t < 16; ++t)
      if (present[t] && vec_of[t] < 0) {
        c->extra |= (unsigned long long)t << (4 * (R - 4));
        vec_of[t] = R++;
      }
    c->R = R;
  }
  c->cols_pref = 0;
  {
    const char* lb = getenv("PHY_LDS_BUDGET");
    c->lds_budget = lb ? std::max(16384, atoi(lb)) : 0;  // 0: automatic plan
    const char* env = getenv("PHY_WG_BUDGET");
    c->wg_budget = env ? std::max(1, atoi(env)) : 0;  // 0: resident workgroups of the plan
    const char* ck = getenv("PHY_COLS");
    c->cols_pref = ck ? std::max(0, std::min(2, atoi(ck))) : 0;
    const char* dk = getenv("PHY_DEEP");
    c->deep_pref = dk ? std::max(0, std::min(2, atoi(dk))) : 0;
    const char* rk = getenv("PHY_RECOMPUTE");
    c->recompute = rk ? atoi(rk) != 0 : true;
    const char* fk = getenv("PHY_FIN");
    c->fin_pref = fk ? atoi(fk) != 0 : true;
    const char* qk = getenv("PHY_QFUSE");
    c->qfuse_pref = qk ? atoi(qk) != 0 : true;
    const char* qk2 = getenv("PHY_QUAD");
    c->quad_pref = qk2 ? atoi(qk2) != 0 : true;
    const char* qm = getenv("PHY_QMW");
    c->qmw_pref = qm ? atoi(qm) != 0 : true;

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
    for (int k = 0; k < 8; ++k)
      (void)hipFuncSetAttribute(sweep_kernel_ptr(1 + (k & 1), (k >> 1) & 1, (k >> 2) & 1),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_CAP);
    (void)hipFuncSetAttribute((const void*)finalize_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_CAP);
    for (const void* kern : {(const void*)qsweep_kernel<256>, (const void*)qsweep_kernel<1024>, (const void*)qmw_kernel}) {
      hipFuncAttributes fa{};  // its static eigensystem copy counts against the cap too
      const size_t stat = hipFuncGetAttributes(&fa, kern) == hipSuccess ? fa.sharedSizeBytes : 1024;
      (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(LDS_CAP - stat));
    }
  }
  if (((size_t)C * c->B + 16 + 1024) * sizeof(double) > LDS_CAP) {
    delete c;
    return fail(PHY_EINVAL, "too many branches x categories for the finalize's LDS (C * B must be <= 19,440)");
  }
  if (lds_bytes(S, C, c->R, 3, 1, 0) > LDS_CAP) {
    delete c;
    return fail(PHY_EINVAL, "too many taxa for one block's tips in LDS");
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
  HIP_C(hipEventCreateWithFlags(&c->ev_nin, hipEventDisableTiming));
  HIP_C(hipEventCreateWithFlags(&c->ev_nout, hipEventDisableTiming));
  const size_t ncolwg = (size_t)C * WAVE;
  TRY_C(dalloc(&c->d_tips, (size_t)S * c->Ppad / 2));
  TRY_C(dalloc(&c->d_w, (size_t)c->Ppad));
  TRY_C(dalloc(&c->d_prog, c->prog.size()));
  TRY_C(dalloc(&c->d_mat_branch, (size_t)c->nmat));
  TRY_C(dalloc(&c->d_gpos, (size_t)c->B));
  TRY_C(dalloc(&c->d_pmat, (size_t)max_draws * C * c->nmat * c->R * 4));
  TRY_C(dalloc(&c->d_eig, (size_t)max_draws * EIG_LEN));
  TRY_C(dalloc(&c->d_inner, (size_t)max_draws * C * c->B));
  TRY_C(dalloc(&c->d_model, (size_t)max_draws * (10 + 2 * C)));
  TRY_C(dalloc(&c->d_blens, (size_t)max_draws * c->B));
  TRY_C(dalloc(&c->d_out, (size_t)max_draws * phy_output_len(c)));
  TRY_C(dalloc(&c->d_site, (size_t)max_draws * P));
  TRY_C(alloc_wg_buffers(c, c->wg_cap));
  {
    const size_t pin = (size_t)std::min(max_draws, PIN_DRAWS);
    const size_t outlen_full = (size_t)1 + c->B + 2 * C + 14 + (size_t)16 * C * c->B;
    TRY_C(dalloc(&c->d_in, pin * (c->B + 10 + 2 * C + EIG_LEN)));
    // portable: a multi-device context's shards all upload from shard 0's staging (multi_enqueue)
    HIP_C(hipHostMalloc((void**)&c->h_in, sizeof(double) * pin * (c->B + 10 + 2 * C + EIG_LEN), hipHostMallocPortable));
    HIP_C(hipHostMalloc((void**)&c->h_out, sizeof(double) * pin * outlen_full, hipHostMallocPortable));
  }
  {
    // tip nibbles: record vector of the pattern's mask (R <= 16); padding =
    // mask 15; pattern 2j in the low nibble of byte j, 2j+1 in the high one
    const int row = c->Ppad / 2;
    const uint8_t pad = (uint8_t)vec_of[15];
    std::vector<uint8_t> tips((size_t)S * row, (uint8_t)(pad | (pad << 4)));
    for (int t = 0; t < S; ++t)
      for (int i = 0; i < P; ++i) {
        const uint8_t v = (uint8_t)vec_of[tipcodes[(size_t)t * P + i]];
        uint8_t& b = tips[(size_t)t * row + i / 2];
        b = (i & 1) ? (uint8_t)((b & 0x0F) | (v << 4)) : (uint8_t)((b & 0xF0) | v);
      }
    std::vector<double> w(c->Ppad, 0.0);
    std::memcpy(w.data(), weights, sizeof(double) * P);
    std::vector<int> gpos(c->B, -1);
    if (c->nmat != c->B) {
      free_ctx(c);
      return fail(PHY_EINVAL, "internal: one matrix per branch expected");
    }
    for (int m = 0; m < c->nmat; ++m) gpos[mat_branch[m]] = m;
    c->gpos = gpos;
    for (int b = 0; b < c->B; ++b)
      if (gpos[b] < 0) {
        std::string m_ = "internal: branch " + std::to_string(b) + " not in the program";
        free_ctx(c);
        return fail(PHY_EINVAL, m_);
      }
    HIP_C(hipMemcpy(c->d_tips, tips.data(), tips.size(), hipMemcpyHostToDevice));
    HIP_C(hipMemcpy(c->d_w, w.data(), w.size() * sizeof(double), hipMemcpyHostToDevice));
    {
      const std::vector<int> packed = pack_program(c->prog);
      HIP_C(hipMemcpy(c->d_prog, packed.data(), packed.size() * sizeof(int), hipMemcpyHostToDevice));
    }
    HIP_C(hipMemcpy(c->d_mat_branch, mat_branch.data(), mat_branch.size() * sizeof(int), hipMemcpyHostToDevice));
    HIP_C(hipMemcpy(c->d_gpos, gpos.data(), gpos.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  TRY_C(plan_chunks(c));
  {  // the quad sweep's program: every moved partial stored (no rebuilt cherries)
    c->quad_lds = quad_lds_bytes(S, C, c->nmat, c->R, c->ndeep);
    c->quad_ok = c->quad_lds + EIG_LEN * sizeof(double) <= LDS_CAP;  // + qsweep_kernel's static eigensystem copy
    if (c->quad_ok) {
      const std::vector<int> qp = quad_program(c->prog, c->nsteps, C, c->R);
      TRY_C(dalloc(&c->d_qprog, qp.size()));
      HIP_C(hipMemcpy(c->d_qprog, qp.data(), qp.size() * sizeof(int), hipMemcpyHostToDevice));
      // the multi-wave variant: as many waves per category as a 1024-thread
      // workgroup holds (<= 4), fewer when that schedule's hand-off slots
      // overflow LDS (a balanced 64-taxon tree at C = 4: 3 waves)
      QmwPlan mp;
      for (int W = std::min(QMW_MAXW, 16 / C); W >= 2 && !c->qmw_ok; --W) {
        if (!quad_mw_plan(c->prog, qp, c->nsteps, W, mp)) continue;
        const size_t lds = qmw_lds_bytes(S, C, c->nmat, c->R, mp.nslot);
        if (lds + EIG_LEN * sizeof(double) <= LDS_CAP) {
          TRY_C(dalloc(&c->d_mprog, mp.prog.size()));
          HIP_C(hipMemcpy(c->d_mprog, mp.prog.data(), mp.prog.size() * sizeof(int), hipMemcpyHostToDevice));
          c->qmw_ok = true;
          c->qmw_W = mp.W;
          c->qmw_maxst = mp.maxst;
          c->qmw_nslot = mp.nslot;
          c->qmw_root = mp.root_wave;
          c->qmw_span = mp.span;
          for (int k = 0; k < 4; ++k) c->qmw_nst[k] = mp.nst[k];
          c->qmw_lds = lds;
        }
      }
    }
  }
  c->h_tips.assign(tipcodes, tipcodes + (size_t)S * P);
  c->h_w.assign(weights, weights + P);
  c->h_peel.assign(peel, peel + 3 * (S - 1));
  c->vec_of = vec_of;
  {
    const char* ek = getenv("PHY_ENGINE");
    c->engine_pref = ek ? std::max(0, std::min(3, atoi(ek))) : 0;
  }
  TRY_C(select_engine(c));
  *out = c;
  return PHY_OK;
}

int phy_create_multi(int S, int P, int C, int rooted, int model, const uint8_t* tipcodes, const double* weights,
                     const int32_t* peel, int max_draws, int n_shards, const int* devices, phy_ctx** out) {
  g_err.clear();
  if (!out) return fail(PHY_EINVAL, "out is NULL");
  *out = nullptr;
  if (n_shards < 1 || n_shards > MAX_SHARDS) return fail(PHY_EINVAL, "n_shards must be in 1..16");
  if (!devices || !tipcodes || !weights || !peel) return fail(PHY_EINVAL, "NULL input array");
  if (S < 3 || P < 1) return fail(PHY_EINVAL, "need S >= 3 taxa and P >= 1 patterns");
  bool same = true, distinct = true;
  for (int k = 0; k < n_shards; ++k)
    for (int j = 0; j < k; ++j) {
      same = same && devices[j] == devices[k];
      distinct = distinct && devices[j] != devices[k];
    }
  if (!same && !distinct)
    return fail(PHY_EINVAL, "phy_create_multi: devices must be all distinct (RCCL) or all the same");
  // contiguous ranges of whole 128-pattern blocks, counts differing by <= 1
  const int nb = (P + 127) / 128;
  if (n_shards > nb) return fail(PHY_EINVAL, "phy_create_multi: more shards than 128-pattern blocks");
  MultiState* m = new MultiState();
  m->P = P;
  m->same_device = same;
  {
    int b0 = 0;
    for (int k = 0; k < n_shards; ++k) {
      const int nbk = nb / n_shards + (k < nb % n_shards ? 1 : 0);
      m->p0.push_back(b0 * 128);
      m->p1.push_back(std::min(P, (b0 + nbk) * 128));
      b0 += nbk;
    }
  }
  auto bail = [&](int rc) {
    const std::string msg = g_err;
    free_multi(m);
    return fail(rc, msg);
  };
  for (int k = 0; k < n_shards; ++k) {
    const int pk = m->p1[k] - m->p0[k];
    std::vector<uint8_t> tk((size_t)S * pk);
    for (int t = 0; t < S; ++t)
      std::memcpy(&tk[(size_t)t * pk], tipcodes + (size_t)t * P + m->p0[k], pk);
    phy_ctx* sh = nullptr;
    int rc = phy_create(S, pk, C, rooted, model, tk.data(), weights + m->p0[k], peel, max_draws, devices[k], &sh);
    if (rc) return bail(rc);
    m->shard.push_back(sh);
    hipEvent_t ev = nullptr;
    if (hipSetDevice(devices[k]) != hipSuccess || hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
      return bail(fail(PHY_EHIP, "hipEventCreate failed"));
    m->ev.push_back(ev);
  }
  if (!same) {
    // peer access between shard 0's device and every other: phy_eval_device's input copies
    // (hipMemcpyPeerAsync) go device to device over xGMI instead of through the host
    for (int k = 1; k < n_shards; ++k) {
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, devices[k], devices[0]) == hipSuccess && can) {
        (void)hipSetDevice(devices[k]);
        (void)hipDeviceEnablePeerAccess(devices[0], 0);  // "already enabled" is fine
        (void)hipSetDevice(devices[0]);
        (void)hipDeviceEnablePeerAccess(devices[k], 0);
      }
    }
    (void)hipGetLastError();
    int rc = rccl_api(&m->rccl);
    if (rc) return bail(rc);
    m->comm.assign(n_shards, nullptr);
    ncclResult_t r = m->rccl->initAll(m->comm.data(), n_shards, devices);
    if (r != ncclSuccess) {
      m->comm.clear();
      return bail(fail(PHY_EHIP, std::string("ncclCommInitAll: ") + m->rccl->errStr(r)));
    }
  }
  phy_ctx* c = new phy_ctx();
  c->S = S;
  c->P = P;
  c->C = C;
  c->rooted = rooted ? 1 : 0;
  c->kind = model;
  c->max_draws = max_draws;
  c->device = devices[0];
  c->B = m->shard[0]->B;
  c->ms = m;
  *out = c;
  return PHY_OK;
}

#ifdef PHY_EPITIME
extern "C" int phy_debug_epitime(unsigned long long* out) {  // diagnostic build only (tools/epitime.py)
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_et), sizeof(g_et)));
  return PHY_OK;
}
#endif
#ifdef PHY_STEPTIME
extern "C" int phy_debug_steptime(unsigned long long* out) {  // diagnostic build only (tools/steptime.py)
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tt), sizeof(g_tt)));
  return PHY_OK;
}
#endif

int phy_destroy(phy_ctx* ctx) {
  free_ctx(ctx);
  return PHY_OK;
}

int phy_num_branches(const phy_ctx* ctx) { return ctx ? ctx->B : -1; }

int phy_output_len(const phy_ctx* ctx) {
  if (!ctx) return -1;
  if (ctx->ms) return phy_output_len(ctx->ms->shard[0]);
  return PHY_OUT_G(ctx->B, ctx->C) + (ctx->compact ? 0 : 16 * ctx->C * ctx->B);
}

int phy_set_output(phy_ctx* ctx, int compact) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->pending || (ctx->ms && ctx->ms->pending))  // phy_eval_wait copies rows of the submitted layout
    return fail(PHY_EINVAL, "phy_set_output: a phy_eval_submit is still in flight (phy_eval_wait first)");
  if (ctx->ms) {
    for (phy_ctx* s : ctx->ms->shard) {
      int rc = phy_set_output(s, compact);
      if (rc) return rc;
    }
    ctx->compact = compact ? 1 : 0;
    return PHY_OK;
  }
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  if (compact && !ctx->d_grows) {
    int rc = dalloc(&ctx->d_grows, (size_t)ctx->max_draws * 16 * ctx->C * ctx->B);
    if (rc) return rc;
  }
  ctx->compact = compact ? 1 : 0;
  return PHY_OK;
}

int phy_program_info(const phy_ctx* ctx, int* nsteps, int* nslots, int* depth, int* nblocks) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->ms) return phy_program_info(ctx->ms->shard[0], nsteps, nslots, depth, nblocks);
  if (nsteps) *nsteps = ctx->nsteps;
  if (nslots) *nslots = ctx->nslots;
  if (depth) *depth = ctx->ndeep;
  if (nblocks) *nblocks = ctx->nblk;
  return PHY_OK;
}

int phy_eval_device(phy_ctx* ctx, int n_draws, const double* d_blens, const double* d_model,
                    double* d_out, double* d_site_ll, void* stream) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->ms) return multi_eval_device(ctx, n_draws, d_blens, d_model, d_out, d_site_ll, stream);
  if (n_draws < 1 || n_draws > ctx->max_draws) return fail(PHY_ERANGE, "n_draws out of range");
  if (!d_blens || !d_model || !d_out) return fail(PHY_EINVAL, "NULL device buffer");
  if (ctx->pending)  // the submitted evaluation still uses the context's work buffers
    return fail(PHY_EINVAL, "phy_eval_device: a phy_eval_submit is still in flight (phy_eval_wait first)");
  HIP_TRY(hipSetDevice(ctx->device));
  if (stream) return launch(ctx, n_draws, d_blens, d_model, d_out, d_site_ll, reinterpret_cast<hipStream_t>(stream));
  // NULL: the caller's legacy null stream (a HIP / torch default-stream caller,
  // prune_stan.hpp:9-17's synchronous contract): the evaluation runs on the
  // context's stream, after the null stream's earlier work and before its later
  return null_fenced(ctx, [&](hipStream_t st) { return launch(ctx, n_draws, d_blens, d_model, d_out, d_site_ll, st); });
}

// The small-batch path's launches: inputs staged in h_in (stage_small), one
// blit in, the launches, the rows to h_out (one blit out).
int launch_small(phy_ctx* ctx, int n_draws, size_t nin, size_t nb, size_t nm, size_t no, bool heig, double* dsite,
                 hipStream_t st) {
  HIP_TRY(hipMemcpyAsync(ctx->d_in, ctx->h_in, sizeof(double) * nin, hipMemcpyHostToDevice, st));
  const double* in = ctx->d_in;
  int r = launch(ctx, n_draws, in, in + nb, ctx->d_out, dsite, st, heig ? in + nb + nm : nullptr);
  if (r) return r;
  HIP_TRY(hipMemcpyAsync(ctx->h_out, ctx->d_out, sizeof(double) * no, hipMemcpyDeviceToHost, st));
  return PHY_OK;
}

// phy_eval_submit / phy_eval_wait: the small-batch path split at the stream
// synchronisation, so a host can overlap its own work (or another context's
// GPU work) with this evaluation.
int phy_eval_submit(phy_ctx* ctx, int n_draws, const double* blens, const double* model) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->ms) {
    if (ctx->ms->pending) return fail(PHY_EINVAL, "phy_eval_submit: an evaluation is already in flight");
    if (n_draws < 1 || n_draws > ctx->max_draws || n_draws > PIN_DRAWS)
      return fail(PHY_ERANGE, "phy_eval_submit: n_draws must be in [1, min(max_draws, 128)]");
    if (!blens || !model) return fail(PHY_EINVAL, "NULL host buffer");
    int rc = multi_enqueue(ctx, n_draws, blens, model, false);
    if (rc) return rc;
    ctx->ms->pending = n_draws;
    return PHY_OK;
  }
  if (ctx->pending) return fail(PHY_EINVAL, "phy_eval_submit: an evaluation is already in flight");
  if (n_draws < 1 || n_draws > ctx->max_draws || n_draws > PIN_DRAWS || !ctx->h_in || !ctx->h_out || !ctx->d_in)
    return fail(PHY_ERANGE, "phy_eval_submit: n_draws must be in [1, min(max_draws, 128)]");
  if (!blens || !model) return fail(PHY_EINVAL, "NULL host buffer");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  const int ml = 10 + 2 * ctx->C;
  const size_t nb = (size_t)n_draws * ctx->B, nm = (size_t)n_draws * ml;
  const size_t no = (size_t)n_draws * phy_output_len(ctx);
  bool heig = false;
  const size_t nin = stage_small(ctx, n_draws, blens, model, &heig);
  int rc = launch_small(ctx, n_draws, nin, nb, nm, no, heig, nullptr, st);
  if (rc) return rc;
  ctx->pending = n_draws;
  return PHY_OK;
}

int phy_eval_wait(phy_ctx* ctx, double* out) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->ms) {
    if (!ctx->ms->pending) return fail(PHY_EINVAL, "phy_eval_wait: nothing submitted");
    if (!out) return fail(PHY_EINVAL, "NULL host buffer");
    const int n = ctx->ms->pending;
    ctx->ms->pending = 0;
    return multi_collect(ctx, n, out, nullptr);
  }
  if (!ctx->pending) return fail(PHY_EINVAL, "phy_eval_wait: nothing submitted");
  if (!out) return fail(PHY_EINVAL, "NULL host buffer");
  HIP_TRY(hipSetDevice(ctx->device));
  const int n = ctx->pending;
  ctx->pending = 0;
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  std::memcpy(out, ctx->h_out, sizeof(double) * (size_t)n * phy_output_len(ctx));
  return PHY_OK;
}

int phy_eval(phy_ctx* ctx, int n_draws, const double* blens, const double* model, double* out,
             double* site_ll) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->ms) return multi_eval(ctx, n_draws, blens, model, out, site_ll);
  if (ctx->pending) return fail(PHY_EINVAL, "phy_eval: a phy_eval_submit is still in flight (phy_eval_wait first)");
  if (n_draws < 1 || n_draws > ctx->max_draws) return fail(PHY_ERANGE, "n_draws out of range");
  if (!blens || !model || !out) return fail(PHY_EINVAL, "NULL host buffer");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  const int ml = 10 + 2 * ctx->C;
  if (n_draws <= PIN_DRAWS && ctx->h_in && ctx->h_out && ctx->d_in) {  // the small-batch (sampler) path
    const size_t nb = (size_t)n_draws * ctx->B, nm = (size_t)n_draws * ml;
    const size_t no = (size_t)n_draws * phy_output_len(ctx);
    bool heig = false;
    const size_t nin = stage_small(ctx, n_draws, blens, model, &heig);
    double* dsite = site_ll ? ctx->d_site : nullptr;
    int rc = launch_small(ctx, n_draws, nin, nb, nm, no, heig, dsite, st);
    if (rc) return rc;
    if (site_ll)
      HIP_TRY(hipMemcpyAsync(site_ll, ctx->d_site, sizeof(double) * n_draws * ctx->P, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    std::memcpy(out, ctx->h_out, sizeof(double) * no);
    return PHY_OK;
  }
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
  if (ctx->ms) {
    for (phy_ctx* s : ctx->ms->shard) {
      int rc = phy_sync(s);
      if (rc) return rc;
    }
    return PHY_OK;
  }
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return PHY_OK;
}

int phy_timing_start(phy_ctx* ctx) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->ms) return phy_timing_start(ctx->ms->shard[0]);
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
  if (ctx->ms) return phy_timing_read(ctx->ms->shard[0], total_ms, launches);
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
  if (ctx->ms) {  // every shard
    for (phy_ctx* s : ctx->ms->shard) {
      int rc = phy_set_tuning(s, wg_budget, cols, lds_budget);
      if (rc) return rc;
    }
    return PHY_OK;
  }
  if (wg_budget > 0) {
    const long need = std::min<long>((long)nblk_for(ctx->P, 1) * ctx->max_draws,
                                     (long)std::max(wg_budget, 4 * ctx->cu_count) + ctx->max_draws);
    if (need > ctx->wg_cap) {  // grow the per-workgroup regions (after the stream's work drains)
      HIP_TRY(hipSetDevice(ctx->device));
      HIP_TRY(hipStreamSynchronize(ctx->stream));
      int rc = alloc_wg_buffers(ctx, need);
      if (rc) return rc;
      ctx->wg_cap = (int)need;
    }
    ctx->wg_budget = wg_budget;
  }
  if (cols < 0 || cols > 2) return fail(PHY_EINVAL, "cols must be 0 (automatic), 1 or 2");
  ctx->cols_pref = cols;
  if (lds_budget > 0) ctx->lds_budget = std::max(16384, std::min(lds_budget, (int)LDS_CAP));
  HIP_TRY(hipSetDevice(ctx->device));
  return plan_chunks(ctx);
}

int phy_columns_per_lane(const phy_ctx* ctx) { return ctx ? (ctx->ms ? ctx->ms->shard[0]->K : ctx->K) : -1; }

int phy_set_deep_stack(phy_ctx* ctx, int mode) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->ms) {  // every shard
    for (phy_ctx* s : ctx->ms->shard) {
      int rc = phy_set_deep_stack(s, mode);
      if (rc) return rc;
    }
    return PHY_OK;
  }
  if (mode < 0 || mode > 2) return fail(PHY_EINVAL, "deep-stack mode must be 0 (automatic), 1 (LDS) or 2 (global)");
  ctx->deep_pref = mode;
  HIP_TRY(hipSetDevice(ctx->device));
  return plan_chunks(ctx);
}
int phy_deep_stack_in_lds(const phy_ctx* ctx) { return ctx ? (ctx->ms ? ctx->ms->shard[0]->ndl : ctx->ndl) : -1; }

int phy_set_recompute(phy_ctx* ctx, int on) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->ms) {  // every shard
    for (phy_ctx* s : ctx->ms->shard) {
      int rc = phy_set_recompute(s, on);
      if (rc) return rc;
    }
    return PHY_OK;
  }
  ctx->recompute = on != 0;
  HIP_TRY(hipSetDevice(ctx->device));
  return plan_chunks(ctx);
}
int phy_recomputed_partials(const phy_ctx* ctx) { return ctx ? (ctx->ms ? ctx->ms->shard[0]->nrec : ctx->nrec) : -1; }

int phy_set_engine(phy_ctx* ctx, int mode) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->ms) {  // every shard
    for (phy_ctx* s : ctx->ms->shard) {
      int rc = phy_set_engine(s, mode);
      if (rc) return rc;
    }
    return PHY_OK;
  }
  if (mode == 3)
    return fail(PHY_EINVAL, "engine 3 (the resident class sweep) was retired: the quad sweep is faster for a "
                            "sampler's calls on every workload (DESIGN.md 5d)");
  if (mode < 0 || mode > 2) return fail(PHY_EINVAL, "engine must be 0 (automatic), 1 (pattern) or 2 (class)");
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  ctx->engine_pref = mode;
  return select_engine(ctx);
}

int phy_engine(const phy_ctx* ctx) { return ctx ? (ctx->ms ? ctx->ms->shard[0]->engine : ctx->engine) : -1; }

int phy_class_info(const phy_ctx* ctx, long long* classes, int* levels, int* root_classes, long long* stage,
                   long long* staged, int* tiles, int* spans) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->ms) return phy_class_info(ctx->ms->shard[0], classes, levels, root_classes, stage, staged, tiles, spans);
  const ClassEngine* e = ctx->ce;
  long long ns = 0;
  int nspan = 0;
  if (e)
    for (const ClassLevel& L : e->lv) nspan += L.nspan;
  if (e) ns = e->stage_elems;
  if (classes) *classes = e ? e->classes : 0;
  if (levels) *levels = e ? e->levels : 0;
  if (root_classes) *root_classes = e ? e->nroot : 0;
  if (stage) *stage = ns;
  if (staged) *staged = e ? e->stage_sec : 0;
  if (tiles) *tiles = e ? e->ntiles : 0;
  if (spans) *spans = nspan;
  return PHY_OK;
}

int phy_quad_plan(const phy_ctx* ctx, int* waves, int* span, int* slots) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->ms) return phy_quad_plan(ctx->ms->shard[0], waves, span, slots);
  const bool on = ctx->qmw_ok && ctx->qmw_pref;
  if (waves) *waves = on ? ctx->qmw_W : (ctx->quad_ok ? 1 : 0);
  if (span) *span = on ? ctx->qmw_span : ctx->nsteps;
  if (slots) *slots = on ? ctx->qmw_nslot : 0;
  return PHY_OK;
}

int phy_class_chain(const phy_ctx* ctx, int* levels, int* lowest, int* top_classes) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->ms) return phy_class_chain(ctx->ms->shard[0], levels, lowest, top_classes);
  const ClassEngine* e = ctx->ce;
  if (levels) *levels = e ? e->chain_m : 0;
  if (lowest) *lowest = e && e->chain_m ? e->chain_lo : 0;
  if (top_classes) *top_classes = e ? e->chain_ntop : 0;
  return PHY_OK;
}

int phy_class_fused(const phy_ctx* ctx, int* level_pairs, int* chunk_spans, int* parent_order_levels) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->ms) return phy_class_fused(ctx->ms->shard[0], level_pairs, chunk_spans, parent_order_levels);
  if (level_pairs) *level_pairs = ctx->ce ? ctx->ce->npairs : 0;
  if (chunk_spans) *chunk_spans = ctx->ce ? ctx->ce->nclong : 0;
  if (parent_order_levels) *parent_order_levels = ctx->ce ? ctx->ce->nsord : 0;
  return PHY_OK;
}

int phy_class_clades(const phy_ctx* ctx, int* fused_levels, int* clades, long long* largest) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->ms) return phy_class_clades(ctx->ms->shard[0], fused_levels, clades, largest);
  const ClassEngine* e = ctx->ce;
  if (fused_levels) *fused_levels = e ? e->Lc : 0;
  if (clades) *clades = e ? e->nclade : 0;
  if (largest) *largest = e ? e->clade_max : 0;
  return PHY_OK;
}

int phy_lds_plan(const phy_ctx* ctx, int* n_chunks, int* matrices_per_chunk, int* lds_bytes_out) {
  if (!ctx) return fail(PHY_EINVAL, "NULL ctx");
  if (ctx->ms) return phy_lds_plan(ctx->ms->shard[0], n_chunks, matrices_per_chunk, lds_bytes_out);
  if (n_chunks) *n_chunks = ctx->nchunks;  // matrix-record chunks per pass
  if (matrices_per_chunk) *matrices_per_chunk = ctx->cap_m;
  if (lds_bytes_out)
    *lds_bytes_out = (int)lds_bytes(ctx->S, ctx->C, ctx->R, ctx->cap_m, ctx->K, ctx->ndl);
  return PHY_OK;
}

}  // extern "C"
