// mjw_dense.h -- register-resident factor / solve / integrate of one small dense world (nv <= 32
// dofs, <= 64 constraint rows) by one wavefront: the device code of the dense kernel
// (mjw_dense.hip) and of the fused step kernel (mjw_step.hip).
//
// One 64-lane wavefront owns one world.  Compared with the generic LDS path in
// mjw_step.hip this path
//   * keeps the mass matrix M and its inverse in the 32x32 MFMA accumulator layout
//     (16 VGPRs each: lane l holds column l&31, rows 8*(r>>2) + 4*(l>>5) + (r&3)),
//   * factors M = L L^T with rows in lanes and v_readlane broadcasts (no barriers),
//     forms X = L^-1 with columns in lanes, and M^-1 = X^T X with 16
//     v_mfma_f32_32x32x2_f32 (exact fp32 FMA chains),
//   * stages the constraint Jacobian once in LDS (odd row stride: conflict-free row
//     and column reads) and keeps one constraint row per lane in VGPRs,
//   * reduces over the wave with DPP (quad_perm / row_ror / row_bcast) + one readlane
//     instead of LDS-crossbar shuffles.
// The CG preconditioner M^-1 grad is therefore one 16-FMA matvec per iteration instead
// of two serial triangular solves (solver.py:2879-2895 restated with an explicit
// inverse; the minimiser and the termination tests are unchanged).


#pragma once
#include "mjw_common.h"
#include "mjw_tendon.h"

// pair independent wave reductions (two 32-lane sums in one reduction, mjw_common.h dsum_halves / dsum2);
// 0 builds the one-reduction-per-sum variant for A/B runs
#ifndef MJW_DENSE_PAIRED
#define MJW_DENSE_PAIRED 1
#endif

namespace mjw {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifndef MJW_SCHED_EARLY
#define MJW_SCHED_EARLY 1
#endif

constexpr int DJS = 33;             // LDS row stride of J (odd: conflict-free rows and columns)
constexpr int DSS = 36;             // LDS row stride of the 32x32 scratch (16-B aligned rows)
constexpr int DJ_WORDS = 64 * DJS;  // 2112
constexpr int DS_WORDS = 32 * DSS;  // 1152

// lanes l and l^32 both receive p(l) + p(l^32)
__device__ __forceinline__ float xhalf_add(float p) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(p), __float_as_uint(p), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// row of register r of a 32x32 MFMA accumulator in lane half h
__device__ __forceinline__ constexpr int acc_row(int r, int h) { return 8 * (r >> 2) + 4 * h + (r & 3); }

// (A v) for symmetric A in accumulator layout; v = vec[0..31] in LDS (16-B aligned).
// Result in lanes c and c+32.
__device__ __forceinline__ float symv(const f32x16& A, const float* vec, int h) {
  const f32x4* v4 = reinterpret_cast<const f32x4*>(vec);
  float p0 = 0.0f, p1 = 0.0f;
#pragma unroll
  for (int g = 0; g < 4; g++) {
    f32x4 q = v4[2 * g + h];
    p0 = fmaf(A[4 * g + 0], q.x, p0);
    p1 = fmaf(A[4 * g + 1], q.y, p1);
    p0 = fmaf(A[4 * g + 2], q.z, p0);
    p1 = fmaf(A[4 * g + 3], q.w, p1);
  }
  return xhalf_add(p0 + p1);
}

// SPD inverse.  a[k] = row (lane&31) of an SPD 32x32 matrix (identity-padded past n).
// On return a[] holds row (lane&31) of L (A = L L^T, upper part zero); the result is
// A^-1 in accumulator layout.  All broadcasts are v_readlane into SGPRs, so the only
// live VGPR arrays are a[32], x[32] and the accumulator.
// NB (>= n, compile time): the factor and substitution loops stop there -- rows and columns past n
// are the identity, which the skipped steps would leave unchanged (exact), so a model with nv <= 16
// does a quarter of the readlane / FMA work of the full 32 (the unrolled schedule is kept: no
// runtime early-outs, which measured slower)
template <bool STORE_L = false, int NB = 32>
__device__ __forceinline__ f32x16 spd_inverse(float (&a)[32], int lane, float* S = nullptr) {
  const int c = lane & 31;
  // right-looking Cholesky, rows in lanes (wp.tile_cholesky, smooth.py:2860-2928);
  // 1/L[j][j] by v_rsq_f32 keeps the per-column critical path short
#pragma unroll
  for (int j = 0; j < NB; j++) {
    float piv = rdlane(a[j], j);
    float inv = __builtin_amdgcn_rsqf(piv);
    a[j] = (c > j) ? a[j] * inv : (c == j ? piv * inv : 0.0f);
#pragma unroll
    for (int k = j + 1; k < NB; k++) a[k] = fmaf(-a[j], rdlane(a[j], k), a[k]);
  }
  if (STORE_L && lane < 32) {
    f32x4* rw = reinterpret_cast<f32x4*>(S + c * DSS);
#pragma unroll
    for (int q = 0; q < 8; q++) rw[q] = f32x4{a[4 * q], a[4 * q + 1], a[4 * q + 2], a[4 * q + 3]};
  }
  // X = L^-1, lane computes column c by right-looking forward substitution (critical path
  // 32 steps, the other updates are independent); L[j][k] = readlane(a[k], j)
  float x[32];
#pragma unroll
  for (int j = 0; j < 32; j++) x[j] = (c == j) ? 1.0f : 0.0f;
#pragma unroll
  for (int k = 0; k < NB; k++) {
    x[k] *= __builtin_amdgcn_rcpf(rdlane(a[k], k));
#pragma unroll
    for (int j = k + 1; j < NB; j++) x[j] = fmaf(-rdlane(a[k], j), x[k], x[j]);
  }
  // A^-1 = X^T X : 16 x (32x32x2) f32 MFMA in two independent chains, operand X[2t + h][c]
  const bool hi = lane >= 32;
  f32x16 r0 = {}, r1 = {};
#pragma unroll
  for (int t = 0; t < 16; t += 2) {
    float v0 = hi ? x[2 * t + 1] : x[2 * t];
    float v1 = hi ? x[2 * t + 3] : x[2 * t + 2];
    r0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v0, v0, r0, 0, 0, 0);
    r1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v1, v1, r1, 0, 0, 0);
  }
  return r0 + r1;
}

// Cholesky in place (rows in lanes) and L rows -> S; no inverse (NB as in spd_inverse)
template <int NB = 32>
__device__ __forceinline__ void chol_factor(float (&a)[32], int lane, float* S) {
  const int c = lane & 31;
#pragma unroll
  for (int j = 0; j < NB; j++) {
    float piv = rdlane(a[j], j);
    float inv = __builtin_amdgcn_rsqf(piv);
    a[j] = (c > j) ? a[j] * inv : (c == j ? piv * inv : 0.0f);
#pragma unroll
    for (int k = j + 1; k < NB; k++) a[k] = fmaf(-a[j], rdlane(a[j], k), a[k]);
  }
  __syncthreads();
  if (lane < 32) {
    f32x4* rw = reinterpret_cast<f32x4*>(S + c * DSS);
#pragma unroll
    for (int q = 0; q < 8; q++) rw[q] = f32x4{a[4 * q], a[4 * q + 1], a[4 * q + 2], a[4 * q + 3]};
  }
  __syncthreads();
}

// (L L^T) x = b for a dof vector b (lane c, both halves): forward sweep with L rows in
// registers, backward sweep with L columns read from S (wp.tile_cholesky_solve); b = 0 past NB
template <int NB = 32>
__device__ __forceinline__ float chol_solve(const float (&a)[32], const float* S, int lane, float b) {
  const int c = lane & 31;
#pragma unroll
  for (int k = 0; k < NB; k++) {
    float yk = rdlane(b, k) * __builtin_amdgcn_rcpf(rdlane(a[k], k));
    b = (c > k) ? fmaf(-a[k], yk, b) : (c == k ? yk : b);
  }
#pragma unroll
  for (int k = NB - 1; k >= 0; k--) {
    float xk = rdlane(b, k) * __builtin_amdgcn_rcpf(S[k * DSS + k]);
    b = (c < k) ? fmaf(-S[k * DSS + c], xk, b) : (c == k ? xk : b);
  }
  return b;
}

// LDL' in place (A = L1 D L1', L1 unit lower), rows in lanes: the factor + solve of the matrices that are
// factored for one solve and need no L (Newton's Hessian every iteration, the implicit-Euler matrix).
// Per column: one pivot readlane, one reciprocal, and the trailing update's readlane + FMA pairs, whose
// readlanes read the unscaled column (they do not wait on the reciprocal) -- no per-column lane selects.
// A lane's entries right of its own column pick up rounding-level residue during the loop; they only
// ever update entries of that same lane right of its column, and are cleared at the end.
// On return a[k] (lane c) = L1[c][k] for k < c and 0 otherwise (the unit diagonal is implicit), S holds
// the same rows and S[c * DSS + 32] (the scratch's padding column) = 1 / D[c] (1 past NB).
template <int NB = 32>
__device__ __forceinline__ void ldl_factor(float (&a)[32], int lane, float* S) {
  const int c = lane & 31;
#pragma unroll
  for (int j = 0; j < NB; j++) {
    const float col = a[j];
    const float r = __builtin_amdgcn_rcpf(rdlane(col, j));
    S[j * DSS + 32] = r;  // the same value from every lane
    a[j] = col * r;
#pragma unroll
    for (int k = j + 1; k < NB; k++) a[k] = fmaf(-a[j], rdlane(col, k), a[k]);
  }
#pragma unroll
  for (int j = NB; j < 32; j++) S[j * DSS + 32] = 1.0f;
#pragma unroll
  for (int k = 0; k < NB; k++) a[k] = k < c ? a[k] : 0.0f;
  __syncthreads();
  if (lane < 32) {
    f32x4* rw = reinterpret_cast<f32x4*>(S + c * DSS);
#pragma unroll
    for (int q = 0; q < 8; q++) rw[q] = f32x4{a[4 * q], a[4 * q + 1], a[4 * q + 2], a[4 * q + 3]};
  }
  __syncthreads();
}

// (L1 D L1') x = b for a dof vector b (lane c, both halves; b = 0 past NB) with ldl_factor's a / S:
// L1 z = b right-looking with the multipliers in registers (lanes at or above the column add an exact
// zero), x = D^-1 z, then L1' x right-looking backward with the rows of L1 from S -- one readlane and one
// FMA per column and sweep, no selects
template <int NB = 32>
__device__ __forceinline__ float ldl_solve(const float (&a)[32], const float* S, int lane, float b) {
  const int c = lane & 31;
  const float rd = S[c * DSS + 32];
#pragma unroll
  for (int k = 0; k < NB - 1; k++) b = fmaf(-a[k], rdlane(b, k), b);
  b *= rd;
#pragma unroll
  for (int k = NB - 1; k > 0; k--) b = fmaf(-S[k * DSS + c], rdlane(b, k), b);
  return b;
}

// stage an n x n block (global row stride gs) into S with identity padding to 32x32,
// plus an optional diagonal term
// (all 16 loads per lane are issued before the first LDS write: one global-latency wait per
// staging instead of one per element, which a load -> wait -> ds_write loop costs)
__device__ __forceinline__ void stage_fill(const float* g, int gs, int n, const float* diag_add, float diag_scale, float* S,
                                           int lane) {
  float v[16];
#pragma unroll
  for (int q = 0; q < 16; q++) {
    const int e = lane + 64 * q, r = e >> 5, k = e & 31;
    v[q] = g[(r < n && k < n) ? r * gs + k : 0];
  }
#pragma unroll
  for (int q = 0; q < 16; q++) {
    const int e = lane + 64 * q, r = e >> 5, k = e & 31;
    float x = (r < n && k < n) ? v[q] : ((r == k) ? 1.0f : 0.0f);
    if (diag_add && r == k && r < n) x += diag_scale * diag_add[r];
    S[r * DSS + k] = x;
  }
  __syncthreads();
}

// rows (lane&31) of the staged matrix into a[], and the n x n block in accumulator layout
__device__ __forceinline__ void stage_rows(int n, const float* S, int lane, float (&a)[32], f32x16& Macc) {
  const int c = lane & 31, h = lane >> 5;
  const f32x4* row = reinterpret_cast<const f32x4*>(S + c * DSS);
#pragma unroll
  for (int q = 0; q < 8; q++) {
    f32x4 v = row[q];
    a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int r = 0; r < 16; r++) {
    int i = acc_row(r, h);
    Macc[r] = (i < n && c < n) ? S[i * DSS + c] : 0.0f;
  }
  __syncthreads();
}

__device__ __forceinline__ void stage_spd(const float* g, int gs, int n, const float* diag_add, float diag_scale, float* S,
                                          int lane, float (&a)[32], f32x16& Macc) {
  stage_fill(g, gs, n, diag_add, diag_scale, S, lane);
  stage_rows(n, S, lane, a, Macc);
}

// lane r: sum_k J[r][k] v[k] over k < 4*nq (JS: the LDS row stride of J)
template <int JS = DJS>
__device__ __forceinline__ float gemv_rows(const float* Jl, const float* vec, int lane, int nq) {
  const f32x4* v4 = reinterpret_cast<const f32x4*>(vec);
  const float* jr = Jl + lane * JS;
  float p0 = 0.0f, p1 = 0.0f;
  for (int q = 0; q < nq; q++) {
    f32x4 v = v4[q];
    p0 = fmaf(jr[4 * q + 0], v.x, p0);
    p1 = fmaf(jr[4 * q + 1], v.y, p1);
    p0 = fmaf(jr[4 * q + 2], v.z, p0);
    p1 = fmaf(jr[4 * q + 3], v.w, p1);
  }
  return p0 + p1;
}

// lane c (both halves): sum_r J[r][c] f[r]; half h sums rows 32h + [0, 4*nq); J holds JS - 1 columns
// (lanes past them return 0)
template <int JS = DJS>
__device__ __forceinline__ float gemv_cols(const float* Jl, const float* fvec, int lane, int nq) {
  const int c = lane & 31, h = lane >> 5;
  const bool in = c < JS - 1;
  const f32x4* f4 = reinterpret_cast<const f32x4*>(fvec + 32 * h);
  const float* jc = Jl + 32 * h * JS + (in ? c : 0);
  float p0 = 0.0f, p1 = 0.0f;
  for (int q = 0; q < nq; q++) {
    f32x4 f = f4[q];
    p0 = fmaf(jc[(4 * q + 0) * JS], f.x, p0);
    p1 = fmaf(jc[(4 * q + 1) * JS], f.y, p1);
    p0 = fmaf(jc[(4 * q + 2) * JS], f.z, p0);
    p1 = fmaf(jc[(4 * q + 3) * JS], f.w, p1);
  }
  return xhalf_add(in ? p0 + p1 : 0.0f);
}

// The same two products with compile-time trip counts, fully unrolled, so that every LDS read is issued
// before the first FMA instead of one LDS round trip per loop iteration.  The terms past the runtime
// bound are exact zeros (J is staged zero-padded; the dof / row vectors are zero past nv / nefc), so the
// sums are the loops' sums.
template <int JS, int NQ>
__device__ __forceinline__ float gemv_rows_u(const float* Jl, const float* vec, int lane) {
  const f32x4* v4 = reinterpret_cast<const f32x4*>(vec);
  const float* jr = Jl + lane * JS;
  float p0 = 0.0f, p1 = 0.0f;
#pragma unroll
  for (int q = 0; q < NQ; q++) {
    f32x4 v = v4[q];
    p0 = fmaf(jr[4 * q + 0], v.x, p0);
    p1 = fmaf(jr[4 * q + 1], v.y, p1);
    p0 = fmaf(jr[4 * q + 2], v.z, p0);
    p1 = fmaf(jr[4 * q + 3], v.w, p1);
  }
  return p0 + p1;
}
template <int JS, int NQ>
__device__ __forceinline__ float gemv_cols_u(const float* Jl, const float* fvec, int lane) {
  const int c = lane & 31, h = lane >> 5;
  const bool in = c < JS - 1;
  const f32x4* f4 = reinterpret_cast<const f32x4*>(fvec + 32 * h);
  const float* jc = Jl + 32 * h * JS + (in ? c : 0);
  float p0 = 0.0f, p1 = 0.0f;
#pragma unroll
  for (int q = 0; q < NQ; q++) {
    f32x4 f = f4[q];
    p0 = fmaf(jc[(4 * q + 0) * JS], f.x, p0);
    p1 = fmaf(jc[(4 * q + 1) * JS], f.y, p1);
    p0 = fmaf(jc[(4 * q + 2) * JS], f.z, p0);
    p1 = fmaf(jc[(4 * q + 3) * JS], f.w, p1);
  }
  return xhalf_add(in ? p0 + p1 : 0.0f);
}
// J' f over the rows of each half up to 4 * nq (nq <= 8, wave-uniform): the smallest unrolled width
template <int JS>
__device__ __forceinline__ float gemv_cols_n(const float* Jl, const float* fvec, int lane, int nq) {
  if (nq <= 2) return gemv_cols_u<JS, 2>(Jl, fvec, lane);
  if (nq <= 4) return gemv_cols_u<JS, 4>(Jl, fvec, lane);
  return gemv_cols_u<JS, 8>(Jl, fvec, lane);
}

// ---- solver row math (solver.py:886-1341 linesearch, 2154-2219 update_constraint) -----------
// cls: 0 = equality (always quadratic), 1 = friction loss, 2 = one-sided (limit / contact)
struct Row {
  float D, jaref, jv, fl, rf;
  int cls;
};

// MJW_DENSE_FASTLS (default 1): the line search's row evaluation and row_force as selects instead of
// per-lane branches (same values; the branches cost exec-mask bookkeeping on every evaluation: the CG
// loop is 9 % shorter); 0 builds the branchy form for A/B runs
#ifndef MJW_DENSE_FASTLS
#define MJW_DENSE_FASTLS 1
#endif
__device__ __forceinline__ void row_eval(const Row& w, float alpha, float& c, float& g, float& hh) {
  float x = fmaf(alpha, w.jv, w.jaref);
  bool quad = (w.cls == 0) || (w.cls == 2 && x < 0.0f) || (w.cls == 1 && -w.rf < x && x < w.rf);
  float jvD = w.jv * w.D;
#if MJW_DENSE_FASTLS
  // non-short-circuit form (the && / || above become exec-mask branches)
  quad = (w.cls == 0) | ((w.cls == 2) & (x < 0.0f)) | ((w.cls == 1) & (-w.rf < x) & (x < w.rf));
  const bool lin = (w.cls == 1) & !quad;
  const bool neg = x <= -w.rf;
  const float cq = 0.5f * w.D * x * x, gq = jvD * x, hq = w.jv * jvD;
  const float cl = w.fl * (-0.5f * w.rf + (neg ? -x : x)), gl = neg ? -w.fl * w.jv : w.fl * w.jv;
  c = quad ? cq : (lin ? cl : 0.0f);
  g = quad ? gq : (lin ? gl : 0.0f);
  hh = quad ? hq : 0.0f;
#else
  if (quad) {
    c = 0.5f * w.D * x * x; g = jvD * x; hh = w.jv * jvD;
  } else if (w.cls == 1) {
    bool neg = x <= -w.rf;
    c = w.fl * (-0.5f * w.rf + (neg ? -x : x));
    g = neg ? -w.fl * w.jv : w.fl * w.jv;
    hh = 0.0f;
  } else {
    c = 0.0f; g = 0.0f; hh = 0.0f;
  }
#endif
}


struct Pt {
  float alpha, c, g, h;
};

__device__ __forceinline__ Pt ls_point(const Row& w, float alpha, float q1, float q2, float qg0) {
  float c, g, hh;
  row_eval(w, alpha, c, g, hh);
  Pt p;
  p.alpha = alpha;
#if MJW_DENSE_PAIRED
  float sc, sg;
  dsum2(c, g, sc, sg);
#else
  const float sc = dsum(c), sg = dsum(g);
#endif
  p.c = sc + alpha * alpha * q2 + alpha * q1 + qg0;
  p.g = sg + 2.0f * alpha * q2 + q1;
  p.h = dsum(hh) + 2.0f * q2;
  return p;
}

// ---- elliptic cones (solver.py:263-323 _eval_elliptic, 1550-1611 quad, 1886-1942 update) ----------
// quad / quad1 / quad2 of one contact, held by the lane of its first row for one line search
struct Ell {
  float q0, q1, q2, u0, v0, uu, uv, vv, dm, mu;
};

__device__ __forceinline__ void eval_elliptic(const Ell& e, float alpha, float& c, float& g, float& hh) {
  c = g = hh = 0.0f;
  const float N = e.u0 + alpha * e.v0;
  const float Tsqr = e.uu + alpha * (2.0f * e.uv + alpha * e.vv);
  bool bottom = false;
  if (Tsqr <= 0.0f) {
    bottom = N < 0.0f;
  } else {
    const float T = sqrtf(Tsqr);
    if (N >= e.mu * T) return;
    if (e.mu * N + T <= 0.0f) {
      bottom = true;
    } else {
      const float N1 = e.v0, T1 = (e.uv + alpha * e.vv) / T;
      const float T2 = e.vv / T - (e.uv + alpha * e.vv) * T1 / (T * T);
      const float nmt = N - e.mu * T, d1 = N1 - e.mu * T1;
      c = 0.5f * e.dm * nmt * nmt;
      g = e.dm * nmt * d1;
      hh = e.dm * (d1 * d1 + nmt * (-e.mu * T2));
      return;
    }
  }
  if (bottom) {
    const float aq2 = alpha * e.q2;
    c = alpha * aq2 + alpha * e.q1 + e.q0;
    g = 2.0f * aq2 + e.q1;
    hh = 2.0f * e.q2;
  }
}

// ls_point with elliptic rows (cls 3): the contact's first row evaluates the cone, the others add 0
__device__ __forceinline__ Pt ls_point_e(const Row& w, const Ell& e, bool first, float alpha, float q1, float q2, float qg0) {
  float c, g, hh;
  if (w.cls == 3) {
    if (first) eval_elliptic(e, alpha, c, g, hh);
    else c = g = hh = 0.0f;
  } else {
    row_eval(w, alpha, c, g, hh);
  }
  Pt p;
  p.alpha = alpha;
#if MJW_DENSE_PAIRED
  float sc, sg;
  dsum2(c, g, sc, sg);
#else
  const float sc = dsum(c), sg = dsum(g);
#endif
  p.c = sc + alpha * alpha * q2 + alpha * q1 + qg0;
  p.g = sg + 2.0f * alpha * q2 + q1;
  p.h = dsum(hh) + 2.0f * q2;
  return p;
}

__device__ __forceinline__ bool bracket(const Pt& x, const Pt& y) { return (x.g < y.g && y.g < 0.0f) || (x.g > y.g && y.g > 0.0f); }

// force / state / cost of one row at its current jaref
__device__ __forceinline__ float row_force(const Row& w, int& state, float& cost) {
#if MJW_DENSE_FASTLS
  // the same cases as selects (no per-lane branches)
  const bool fr = w.cls == 1;
  const bool lneg = fr & (w.jaref <= -w.rf), lpos = fr & !lneg & (w.jaref >= w.rf);
  const bool sat = (w.cls == 2) & (w.jaref >= 0.0f);
  const float fq = -w.D * w.jaref, cq = 0.5f * w.D * w.jaref * w.jaref;
  const float cneg = -w.fl * (0.5f * w.rf + w.jaref), cpos = -w.fl * (0.5f * w.rf - w.jaref);
  state = lneg ? STATE_LINEARNEG : (lpos ? STATE_LINEARPOS : (sat ? STATE_SATISFIED : STATE_QUADRATIC));
  cost = lneg ? cneg : (lpos ? cpos : (sat ? 0.0f : cq));
  return lneg ? w.fl : (lpos ? -w.fl : (sat ? 0.0f : fq));
#endif
  float f;
  cost = 0.0f;
  if (w.cls == 1) {
    if (w.jaref <= -w.rf) { f = w.fl; state = STATE_LINEARNEG; cost = -w.fl * (0.5f * w.rf + w.jaref); }
    else if (w.jaref >= w.rf) { f = -w.fl; state = STATE_LINEARPOS; cost = -w.fl * (0.5f * w.rf - w.jaref); }
    else { f = -w.D * w.jaref; state = STATE_QUADRATIC; cost = 0.5f * w.D * w.jaref * w.jaref; }
  } else if (w.cls == 2 && w.jaref >= 0.0f) {
    f = 0.0f; state = STATE_SATISFIED;
  } else {
    f = -w.D * w.jaref; state = STATE_QUADRATIC; cost = 0.5f * w.D * w.jaref * w.jaref;
  }
  return f;
}

// ---- the kernel ---------------------------------------------------------------------------
// LDS words of one world of the dense path
// elliptic-cone workspace (ELL): per row D, cone coefficient, two scratch rows, first row / dim of its
// contact, and the 6 cone-Hessian coefficients of the row (Newton)
constexpr int DE_WORDS = 6 * 64 + 6 * 64;
// LDS row stride of the staged J: 33 (32 columns), 17 for the NB = 16 kernels (16 columns)
template <int NB>
__host__ __device__ constexpr int dense_js() { return NB <= 16 ? 17 : DJS; }
template <int FLAGS, bool NEWTON, bool ELL = false, int NB = 32>
__host__ __device__ constexpr int dense_j_words() {
  // CG: the 32x32 scratch aliases J, so the region is the larger of the two
  return (NEWTON && (FLAGS & DF_SOLVE)) ? 64 * dense_js<NB>() : (64 * dense_js<NB>() > DS_WORDS ? 64 * dense_js<NB>() : DS_WORDS);
}
template <int FLAGS, bool NEWTON, bool ELL = false, int NB = 32>
__host__ __device__ constexpr int dense_lds_words() {
  // launches without the solve stage no J, only the 32x32 scratch (the Euler-only kernel: 5.9 KB)
  return ((NEWTON && (FLAGS & DF_SOLVE)) ? dense_j_words<FLAGS, NEWTON, ELL, NB>() + DS_WORDS
          : (FLAGS & DF_SOLVE)           ? dense_j_words<FLAGS, NEWTON, ELL, NB>()
                                         : DS_WORDS) +
         5 * 64 + (ELL && (FLAGS & DF_SOLVE) ? DE_WORDS : 0);
}


// factor / solve / integrate of world `wid` by the calling wavefront; sm: dense_lds_words() floats of
// LDS, 16-B aligned (the dense kernel's own, or the fused step kernel's dynamic LDS once the
// forward stages are done with it)
template <int FLAGS, bool NEWTON, bool ELL = false, int NB = 32>
__device__ __forceinline__ void dense_world(const mjw_model_t& m, const mjw_data_t& d, const int wid, float* sm) {
  constexpr bool NT = NEWTON && (FLAGS & DF_SOLVE);
  constexpr bool EL = ELL && (FLAGS & DF_SOLVE);
  constexpr int JS = dense_js<NB>(), JC = JS - 1;  // J row stride and staged columns
  constexpr int JW = dense_j_words<FLAGS, NEWTON, ELL, NB>();
  constexpr int S_OFF = NT ? JW : 0;  // CG: the 32x32 scratch aliases J (used before J is staged)
  constexpr int V_OFF = NT ? JW + DS_WORDS : (FLAGS & DF_SOLVE) ? JW : DS_WORDS;
  float* Jl = sm;
  float* S = sm + S_OFF;
  float* vd = sm + V_OFF;        // dof vector broadcast buffer (32)
  float* vd2 = vd + 64;          // second dof buffer
  float* vr = vd + 128;          // row vector buffer (64)
  float* vr2 = vd + 192;         // second row buffer (Newton weights)
  float* vq = vd + 256;          // qpos (Euler)
  // elliptic workspace (EL only): per row D, cone coefficient (mu for the first row of a contact, its
  // friction coefficient for the others), scratch A / B, first row and dim of the contact, cone Hessian
  float* eD = vd + 320;
  float* eF = eD + 64;
  float* eA = eD + 128;
  float* eB = eD + 192;
  int* eR0 = reinterpret_cast<int*>(eD + 256);
  int* eDim = reinterpret_cast<int*>(eD + 320);
  float* eC = eD + 384;  // 6 per row
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  const int nv = m.nv, np = m.nv_pad;
  const bool dof = c < nv;      // lane holds a dof value (both halves)
  const bool lo = lane < 32;
  const long gi = (long)wid * nv + c;

  // per-world inputs of the later phases, loaded up front so that their global latency overlaps
  // the qM staging and the factorisation instead of stalling each phase
  const int nq = m.nq;
  const bool qpos_lds = nq <= 64;
  float pf_qfrc_smooth = 0.0f, pf_warm = 0.0f, pf_qvel = 0.0f, pf_qpos = 0.0f, pf_D = 0.0f, pf_aref = 0.0f, pf_fl = 0.0f, pf_time = 0.0f;
  int pf_nefc = 0, pf_ne = 0, pf_nf = 0;
  if ((FLAGS & (DF_FACTOR | DF_SOLVE)) && dof) pf_qfrc_smooth = d.qfrc_smooth[gi];
  if (FLAGS & DF_SOLVE) {
    if (dof) pf_warm = d.qacc_warmstart[gi];
    pf_nefc = d.nefc[wid];
    pf_ne = d.ne[wid];
    pf_nf = d.nf[wid];
    if (lane < d.njmax) {
      pf_D = d.efc_D[(long)wid * d.njmax_pad + lane];
      pf_aref = d.efc_aref[(long)wid * d.njmax + lane];
      pf_fl = d.efc_frictionloss[(long)wid * d.njmax + lane];
    }
  }
  if (FLAGS & DF_EULER) {
    if (dof) pf_qvel = d.qvel[gi];
    if (qpos_lds && lane < nq) pf_qpos = d.qpos[(long)wid * nq + lane];
    // the time too: read at the end, after the solve's stores, its load would wait for all of them (vmcnt
    // counts loads and stores in issue order)
    if (lane == 0) pf_time = d.time[wid];
  }

  PROF_T0();
  float qacc = 0.0f, ma = 0.0f;
  f32x16 Mm = {}, Mi = {};
  float qfrc_smooth = 0.0f, qacc_smooth = 0.0f;
  if (FLAGS & (DF_FACTOR | DF_SOLVE)) {
    // ---- factor M, form M^-1, qacc_smooth (smooth.py:2860-2928 factor_solve_i)
    float a[32];
    stage_spd(d.qM + (long)wid * np * np, np, nv, nullptr, 0.0f, S, lane, a, Mm);
    // CG preconditions with M^-1 every iteration, so it forms the inverse; Newton (its own Hessian
    // factor) and the factor-only launch need L and one solve only
    constexpr bool NEED_INV = (FLAGS & DF_SOLVE) && !NEWTON;
    if (NEED_INV) Mi = spd_inverse<(FLAGS & DF_FACTOR) != 0, NB>(a, lane, S);
    else chol_factor<NB>(a, lane, S);  // L rows -> S
    if (FLAGS & DF_FACTOR) {
      // L rows -> qLD (nv x nv) through S for coalesced stores
      __syncthreads();
      float* gL = d.qLD + (long)wid * nv * nv;
      for (int e = lane; e < nv * nv; e += 64) {
        int r = e / nv, k = e - r * nv;
        gL[e] = S[r * DSS + k];
      }
    }
    qfrc_smooth = pf_qfrc_smooth;
    if (NEED_INV) {
      if (lo) vd[c] = qfrc_smooth;
      __syncthreads();
      qacc_smooth = symv(Mi, vd, h);
    } else {
      qacc_smooth = chol_solve<NB>(a, S, lane, dof ? qfrc_smooth : 0.0f);
    }
    if (!dof) qacc_smooth = 0.0f;
    if ((FLAGS & DF_FACTOR) && lo && dof) d.qacc_smooth[gi] = qacc_smooth;
  }

  PROF_MARK(PH_DFACTOR);
  int niter_out = 0;  // CG / Newton iterations of this world (0 without rows)
  if (FLAGS & DF_SOLVE) {
    const int njmax = d.njmax;
    const int nefc = min(pf_nefc, njmax);
    const int ne = pf_ne, nf = pf_nf;
    __syncthreads();  // S (aliasing J for CG) is free again
    if (njmax == 0 || nv == 0) {
      qacc = qacc_smooth;
      if (lo) vd[c] = qacc;
      __syncthreads();
      ma = symv(Mm, vd, h);
      if (lo && dof) {
        d.qacc[gi] = qacc;
        d.efc_Ma[gi] = ma;
      }
      if (lane == 0) d.solver_niter[wid] = 0;
    } else {
      // stage J (zero padded to 64 x JC), 16 loads in flight per lane and batch
      const float* gJ = d.efc_J + (long)wid * d.njmax_pad * np;
#pragma unroll
      for (int half = 0; half < JC / 16; half++) {
        float v[16];
#pragma unroll
        for (int q = 0; q < 16; q++) {
          const int e = lane + 64 * (16 * half + q), r = e / JC, k = e % JC;
          v[q] = gJ[(r < nefc && k < nv) ? r * np + k : 0];
        }
#pragma unroll
        for (int q = 0; q < 16; q++) {
          const int e = lane + 64 * (16 * half + q), r = e / JC, k = e % JC;
          Jl[r * JS + k] = (r < nefc && k < nv) ? v[q] : 0.0f;
        }
      }
      Row w;
      const bool row = lane < nefc;
      w.D = row ? pf_D : 0.0f;
      float aref = row ? pf_aref : 0.0f;
      w.fl = row ? pf_fl : 0.0f;
      w.rf = safe_div(w.fl, w.D);
      w.cls = lane < ne ? 0 : (lane < ne + nf ? 1 : 2);
      w.jv = 0.0f;
      // elliptic contacts (cls 3): the rows of one contact are consecutive (constraint rows are emitted
      // per contact); e_r0 = its first row (segment start of equal efc_id), e_dim its rows, e_fr this
      // row's cone coefficient; a contact cut by njmax (e_r0 + e_dim > nefc) contributes nothing
      int e_r0 = lane, e_dim = 1;
      float e_fr = 0.0f, e_mu = 0.0f;
      bool e_cut = false;
      if (EL) {
        const int typ = row ? d.efc_type[(long)wid * njmax + lane] : -1;
        const bool ell = typ == CNSTR_CONTACT_ELLIPTIC;
        const int cid = ell ? d.efc_id[(long)wid * njmax + lane] : -1;
        const int prev = __shfl_up(cid, 1, 64);
        const unsigned long long starts = __ballot(ell && (lane == 0 || prev != cid));
        if (ell) {
          e_r0 = 63 - __clzll(starts & ((2ull << lane) - 1ull));
          e_dim = d.contact_dim[cid];
          const float* fr = d.contact_friction + 5L * cid;
          e_mu = fr[0] * MR(opt_impratio_invsqrt)[0];
          const int k = lane - e_r0;
          e_fr = k == 0 ? e_mu : fr[k - 1];
          e_cut = e_r0 + e_dim > nefc;
          w.cls = 3;
        }
        eD[lane] = w.D;
        eF[lane] = e_fr;
        eR0[lane] = e_r0;
        eDim[lane] = (ell && !e_cut) ? e_dim : 1;
      }
      Ell ecoef = {};
      const float tolerance = MR(opt_tolerance)[0];
      const float ls_tolerance = MR(opt_ls_tolerance)[0];
      const float meaninertia = MR(stat_meaninertia)[0];
      // qacc init (solver.py:3308-3311)
      qacc = dof ? ((m.opt_disableflags & DSBL_WARMSTART) ? qacc_smooth : pf_warm) : 0.0f;
      if (lo) vd[c] = qacc;
      __syncthreads();
      ma = symv(Mm, vd, h);
      w.jaref = gemv_rows_u<JS, NB / 4>(Jl, vd, lane) - aref;
      const int nrq = (min(nefc, 32) + 3) >> 2;

      float cost, gauss, qfrc_c, grad, Mgrad, grad_dot;
      int state = STATE_SATISFIED;
      float force = 0.0f;
      auto update_constraint = [&]() {
        float rc;
        force = row_force(w, state, rc);
        if (EL) {
          // elliptic cone zones (solver.py:1886-1942): N from the first row, T from the friction rows
          eA[lane] = w.jaref * e_fr;
          __syncthreads();
          if (w.cls == 3) {
            float TT = 0.0f;
            for (int j = 1; j < e_dim && !e_cut; j++) {
              const float u = eA[e_r0 + j];
              TT += u * u;
            }
            const float N = eA[e_r0], mu = e_mu;
            const float T = TT <= 0.0f ? 0.0f : sqrtf(TT);
            rc = 0.0f;
            if (e_cut || N >= mu * T || (T <= 0.0f && N >= 0.0f)) {
              force = 0.0f; state = STATE_SATISFIED;
            } else if (mu * N + T <= 0.0f || (T <= 0.0f && N < 0.0f)) {
              force = -w.D * w.jaref; state = STATE_QUADRATIC; rc = 0.5f * w.D * w.jaref * w.jaref;
            } else {
              const float dm = safe_div(eD[e_r0], mu * mu * (1.0f + mu * mu));
              const float nmt = N - mu * T;
              const float f0 = -dm * nmt * mu;
              if (lane == e_r0) { force = f0; rc = 0.5f * dm * nmt * nmt; }
              else force = -safe_div(f0, T) * (eA[lane] * e_fr);
              state = STATE_CONE;
            }
          }
        }
        if (!row) { force = 0.0f; rc = 0.0f; }
        vr[lane] = force;
        __syncthreads();
        qfrc_c = gemv_cols_n<JS>(Jl, vr, lane, nrq);
        // update_gradient's grad (solver.py:2879-2890) here, so that the Gauss term and |grad|^2 -- both
        // sums over the dofs -- share one reduction (dofs in lanes 0-31, replicated in 32-63)
        grad = dof ? ma - qfrc_smooth - qfrc_c : 0.0f;
#if MJW_DENSE_PAIRED
        float g2;
        dsum_halves(lo ? (ma - qfrc_smooth) * (qacc - qacc_smooth) : grad * grad, g2, grad_dot);
        gauss = 0.5f * g2;
#else
        gauss = 0.5f * dsum(lo ? (ma - qfrc_smooth) * (qacc - qacc_smooth) : 0.0f);
        grad_dot = dsum(lo ? grad * grad : 0.0f);
#endif
        cost = dsum(rc) + gauss;
      };
      auto update_gradient = [&]() {
        if (lo) vd2[c] = grad;
        if (NEWTON) {
          // H = M + J' diag(D * quadratic) J (solver.py:2896-3008): 32x32x2 MFMA over row pairs
          vr2[lane] = (row && state == STATE_QUADRATIC) ? w.D : 0.0f;
          if (EL) {
            // + J_c' C J_c for elliptic contacts in the cone state (solver.py:2430-2585): row a's MFMA
            // operand becomes sum_k C[a][k] J[r0 + k] (C = D on the diagonal for quadratic rows)
            const int ea = lane - e_r0;
            const bool quad = row && state == STATE_QUADRATIC;
            const bool cone = w.cls == 3 && state == STATE_CONE;
            float dm = 0.0f, mu = e_mu, mu_over_t = 0.0f, mu_n_over_ttt = 0.0f, diag = 0.0f, ua = 0.0f;
            if (cone) {
              const float mu2 = mu * mu;
              dm = safe_div(eD[e_r0], mu2 * (1.0f + mu2));
              const float n = eA[e_r0];
              float tt = 0.0f;
              for (int j = 1; j < e_dim; j++) tt += eA[e_r0 + j] * eA[e_r0 + j];
              float t = tt <= 0.0f ? 0.0f : sqrtf(tt);
              t = fmaxf(t, MJW_MINVAL);
              const float ttt = fmaxf(t * t * t, MJW_MINVAL);
              mu_over_t = safe_div(mu, t);
              mu_n_over_ttt = mu * safe_div(n, ttt);
              diag = mu2 - mu * safe_div(n, t);
              ua = eA[lane];
            }
#pragma unroll
            for (int k = 0; k < 6; k++) {
              float ck = (quad && k == ea) ? w.D : 0.0f;
              if (cone && k < e_dim) {
                const float ub = eA[e_r0 + k];
                float hc;
                if (ea == 0 && k == 0) hc = 1.0f;
                else if (ea == 0) hc = -mu_over_t * ub;
                else if (k == 0) hc = -mu_over_t * ua;
                else hc = mu_n_over_ttt * ua * ub + (ea == k ? diag : 0.0f);
                ck = hc * dm * e_fr * eF[e_r0 + k];
              }
              eC[6 * lane + k] = ck;
            }
          }
          __syncthreads();
          PROF_T0_SUB();
          f32x16 H = Mm;
          const int npair = (nefc + 1) >> 1;
          for (int t = 0; t < npair; t++) {
            int r = 2 * t + h;
            float jrc = c < JC ? Jl[r * JS + c] : 0.0f;
            float wrc = vr2[r] * jrc;
            if (EL) {
              wrc = 0.0f;
              const int r0 = eR0[r], dm_ = eDim[r];
              for (int k = 0; k < dm_; k++) wrc = fmaf(eC[6 * r + k], c < JC ? Jl[(r0 + k) * JS + c] : 0.0f, wrc);
            }
            H = __builtin_amdgcn_mfma_f32_32x32x2f32(jrc, wrc, H, 0, 0, 0);
          }
          // identity-pad rows/cols >= nv, then rows into lanes through S
#pragma unroll
          for (int q = 0; q < 16; q++) {
            int i = acc_row(q, h);
            S[i * DSS + c] = (i < nv && c < nv) ? H[q] : (i == c ? 1.0f : 0.0f);
          }
          __syncthreads();
          float a[32];
          const f32x4* rw = reinterpret_cast<const f32x4*>(S + c * DSS);
#pragma unroll
          for (int q = 0; q < 8; q++) {
            f32x4 v = rw[q];
            a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
          }
          PROF_MARK_SUB(PH_NT_H);
          ldl_factor<NB>(a, lane, S);
          Mgrad = ldl_solve<NB>(a, S, lane, grad);
          PROF_MARK_SUB(PH_NT_CHOL);
        } else {
          __syncthreads();
          Mgrad = symv(Mi, vd2, h);
        }
        if (!dof) Mgrad = 0.0f;
      };

      float prev_cost;
      update_constraint();
      update_gradient();
      float search = -Mgrad;
      float search_dot = dsum(lo ? search * search : 0.0f);
      int niter = 0;
      const float scale = 1.0f / (meaninertia * (float)nv);
      bool done = m.opt_iterations == 0;
      while (!done) {
        // ---- linesearch (solver.py:886-1341, 1662-1703)
        if (lo) vd[c] = search;
        __syncthreads();
        float mv = symv(Mm, vd, h);
        w.jv = gemv_rows_u<JS, NB / 4>(Jl, vd, lane);
        const float snorm = sqrtf(search_dot);
        const float gtol = fmaxf(tolerance * ls_tolerance * snorm * meaninertia * (float)nv, 1e-6f);
#if MJW_DENSE_PAIRED
        float q1, q2;
        dsum_halves(lo ? search * (ma - qfrc_smooth) : 0.5f * search * mv, q1, q2);
#else
        const float q1 = dsum(lo ? search * (ma - qfrc_smooth) : 0.0f);
        const float q2 = dsum(lo ? 0.5f * search * mv : 0.0f);
#endif
        const float qg0 = gauss;
        const bool e_first = EL && w.cls == 3 && lane == e_r0 && !e_cut;
        if (EL) {
          // per-contact quad / quad1 / quad2 at the first row (solver.py:1550-1611)
          eA[lane] = w.jaref;
          eB[lane] = w.jv;
          __syncthreads();
          ecoef = Ell{};
          if (e_first) {
            const float D0 = w.D, ja = w.jaref, jv = w.jv, mu = e_mu;
            ecoef.q0 = 0.5f * ja * ja * D0; ecoef.q1 = jv * ja * D0; ecoef.q2 = 0.5f * jv * jv * D0;
            ecoef.u0 = ja * mu; ecoef.v0 = jv * mu; ecoef.mu = mu;
            for (int j = 1; j < e_dim; j++) {
              const int rj = lane + j;
              const float jaj = eA[rj], jvj = eB[rj], dj = eD[rj], fj = eF[rj], DJj = dj * jaj;
              ecoef.q0 += 0.5f * jaj * DJj; ecoef.q1 += jvj * DJj; ecoef.q2 += 0.5f * jvj * dj * jvj;
              const float uj = jaj * fj, vj = jvj * fj;
              ecoef.uu += uj * uj; ecoef.uv += uj * vj; ecoef.vv += vj * vj;
            }
            ecoef.dm = D0 / (mu * mu * (1.0f + mu * mu));
          }
        }
        auto lsp = [&](float al) -> Pt { return EL ? ls_point_e(w, ecoef, e_first, al, q1, q2, qg0) : ls_point(w, al, q1, q2, qg0); };
        float alpha;
        if (m.opt_ls_parallel) {
          // solver.py:325-478 parallel linesearch: the cheapest of ls_iterations log-spaced step sizes
          // in [ls_parallel_min_step, 1] (the first one on ties)
          alpha = 0.0f;
          float best = MJW_MAXVAL;
          for (int i = 0; i < m.opt_ls_iterations; i++) {
            const float al = ls_parallel_alpha(MR(opt_ls_parallel_min_step)[0], m.opt_ls_iterations, i);
            const float cst = lsp(al).c;
            if (cst < best) { best = cst; alpha = al; }
          }
        } else {
        Pt p0 = lsp(0.0f);
        float lo_alpha_in = -safe_div(p0.g, p0.h);
        Pt lo_in = lsp(lo_alpha_in);
        if (fabsf(lo_in.g) < gtol && lo_in.c < p0.c) {
          alpha = lo_alpha_in;
        } else {
          alpha = 0.0f;
          bool lo_less = lo_in.g < p0.g;
          Pt plo = lo_less ? lo_in : p0;
          Pt phi = lo_less ? p0 : lo_in;
          for (int it = 0; it < m.opt_ls_iterations; it++) {
            Pt ln = lsp(plo.alpha - safe_div(plo.g, plo.h));
            Pt hn = lsp(phi.alpha - safe_div(phi.g, phi.h));
            Pt md = lsp(0.5f * (plo.alpha + phi.alpha));
            bool s1 = bracket(plo, ln);
            if (s1) plo = ln;
            bool s2 = bracket(plo, md);
            if (s2) plo = md;
            bool s3 = bracket(plo, hn);
            if (s3) plo = hn;
            bool h1 = bracket(phi, hn);
            if (h1) phi = hn;
            bool h2 = bracket(phi, md);
            if (h2) phi = md;
            bool h3 = bracket(phi, ln);
            if (h3) phi = ln;
            bool ls_done = (!(s1 || s2 || s3) && !(h1 || h2 || h3)) || (plo.g < 0.0f && plo.g > -gtol) ||
                           (phi.g > 0.0f && phi.g < gtol);
            bool improved = plo.c < p0.c || phi.c < p0.c;
            if (improved) alpha = plo.c < phi.c ? plo.alpha : phi.alpha;
            if (ls_done) break;
          }
        }
        }
        qacc = fmaf(alpha, search, qacc);
        ma = fmaf(alpha, mv, ma);
        w.jaref = fmaf(alpha, w.jv, w.jaref);
        // ---- update constraint + gradient, CG direction (solver.py:3187-3254)
        float prev_grad = grad, prev_Mgrad = Mgrad;
        prev_cost = cost;
        update_constraint();
        update_gradient();
        float beta = 0.0f;
        if (!NEWTON) {
#if MJW_DENSE_PAIRED
          float num, den;
          dsum_halves(lo ? grad * (Mgrad - prev_Mgrad) : prev_grad * prev_Mgrad, num, den);
#else
          float num = dsum(lo ? grad * (Mgrad - prev_Mgrad) : 0.0f);
          float den = dsum(lo ? prev_grad * prev_Mgrad : 0.0f);
#endif
          beta = fmaxf(0.0f, num / fmaxf(MJW_MINVAL, den));
        }
        search = dof ? (-Mgrad + beta * search) : 0.0f;
        search_dot = dsum(lo ? search * search : 0.0f);
        niter++;
        float improvement = (prev_cost - cost) * scale;
        float gradient = sqrtf(grad_dot) * scale;
        done = (improvement < tolerance) || (gradient < tolerance) || niter == m.opt_iterations;
      }
      if (lo && dof) {
        d.qacc[gi] = qacc;
        d.efc_Ma[gi] = ma;
        d.qfrc_constraint[gi] = qfrc_c;
      }
      if (row) {
        d.efc_force[(long)wid * njmax + lane] = force;
        d.efc_state[(long)wid * d.njmax_pad + lane] = state;
      }
      if (lane == 0) d.solver_niter[wid] = niter;
      niter_out = niter;
    }
  }

  PROF_MARK(PH_DSOLVE);
#if MJW_SCHED_EARLY
  // the next step's longest-first order (see dense_kernel): this world's iteration bucket, stored here,
  // before the integration; the counter-reset kernel of the next step histograms the buckets itself (no
  // atomics here: same-address bucket atomics held the wave slots while they drained)
  if ((FLAGS & DF_SOLVE) && d.sched && lane == 0)
    d.world_key[wid] = MJW_SCHED_BUCKETS - 1 - min(niter_out >> 1, MJW_SCHED_BUCKETS - 1);
#endif
  if (FLAGS & DF_EULER) {
    // ---- forward.py:51-354 (_advance + euler)
    const float dt = MR(opt_timestep)[0];
    if (!(FLAGS & DF_SOLVE)) {
      qacc = dof ? d.qacc[gi] : 0.0f;
      ma = dof ? d.efc_Ma[gi] : 0.0f;
    }
    float qacc_adv = qacc;
    __syncthreads();
    // implicit integration only in the Euler-only kernel (dense_launch splits the step when needed)
    const int fl = m.opt_disableflags;
    const bool implicitfast = m.opt_integrator == INT_IMPLICITFAST;
    const bool need_implicit = implicitfast ? (fl & (DSBL_ACTUATION | DSBL_SPRING | DSBL_DAMPER)) != (DSBL_ACTUATION | DSBL_SPRING | DSBL_DAMPER)
                                            : !(fl & (DSBL_EULERDAMP | DSBL_DAMPER));
    if (FLAGS == DF_EULER && need_implicit) {
      // euler damping: (M + dt diag(damping)) qacc_adv = M qacc (forward.py:322-340); implicitfast:
      // (M - dt qDeriv) qacc_adv = M qacc, qDeriv = sum_a vel_a m_a m_a' - diag(damping) on the
      // ancestor pattern of qM (forward.py:494-510, derivative.py:320-416)
      float a[32];
      f32x16 Md;
      stage_fill(d.qM + (long)wid * np * np, np, nv, (fl & DSBL_DAMPER) ? nullptr : MR(dof_damping), dt, S, lane);
      if (implicitfast && m.nu > 0 && !(fl & DSBL_ACTUATION)) {
        for (int u = 0; u < m.nu; u++) {
          float vel = actuator_vel_deriv(m, d, wid, u);
          if (vel == 0.0f) continue;
          const long gu = (long)wid * m.nu + u;
          const int nnz = d.moment_rownnz[gu], adr = d.moment_rowadr[gu];
          if (lane < nnz * nnz) {
            const int k1 = lane / nnz, k2 = lane - k1 * nnz;
            const long base = (long)wid * m.nJmom + adr;
            const int i = d.moment_colind[base + k1], j = d.moment_colind[base + k2];
            int p = i;
            while (p > j) p = m.dof_parentid[p];
            if (p == j && i < 32 && j < 32) {
              float v = dt * vel * d.actuator_moment[base + k1] * d.actuator_moment[base + k2];
              S[i * DSS + j] -= v;
              if (i != j) S[j * DSS + i] -= v;
            }
          }
          __syncthreads();
        }
      }
      if (implicitfast && m.ntendon && !(fl & DSBL_DAMPER)) {
        // derivative.py:267-320: tendon damping enters qDeriv as -damping J_i J_j on the qM pattern
        const float* tdamp = MR(tendon_damping);
        for (int t = 0; t < m.ntendon; t++) {
          if (tdamp[t] == 0.0f) continue;
          const int rn = m.ten_J_rownnz[t], ra = m.ten_J_rowadr[t];
          for (int p = lane; p < rn * rn; p += 64) {
            const int k1 = p / rn, k2 = p - k1 * rn;
            if (k2 > k1) continue;
            const int i = m.ten_J_colind[ra + k1], j = m.ten_J_colind[ra + k2];
            int q = i;
            while (q > j) q = m.dof_parentid[q];
            if (q != j || i >= 32) continue;
            const float v = dt * tdamp[t] * ten_coef(m, d, wid, t, i) * ten_coef(m, d, wid, t, j);
            S[i * DSS + j] += v;
            if (i != j) S[j * DSS + i] += v;
          }
          __syncthreads();
        }
      }
      stage_rows(nv, S, lane, a, Md);
      __syncthreads();
      // one solve with the factor (forward + backward sweep), no explicit inverse
      ldl_factor<NB>(a, lane, S);
      qacc_adv = ldl_solve<NB>(a, S, lane, dof ? ma : 0.0f);
      if (!dof) qacc_adv = 0.0f;
    }
    // activations (forward.py:132-168)
    const float* actrange = MR(actuator_actrange);
    for (int u = lane; u < m.nu; u += 64) {
      int adr = m.actuator_actadr[u];
      for (int j = adr; adr >= 0 && j < adr + m.actuator_actnum[u]; j++) {
        long ga = (long)wid * m.na + j;
        d.act[ga] = next_act(dt, m.actuator_dyntype[u], MR(actuator_dynprm)[10 * u], actrange + 2 * u, d.act[ga], d.act_dot[ga], 1.0f,
                             m.actuator_actlimited[u] != 0);
      }
    }
    float qvel = dof ? pf_qvel + qacc_adv * dt : 0.0f;
    if (lo) {
      vd2[c] = qvel;
      if (dof) {
        d.qvel[gi] = qvel;
        d.qacc_warmstart[gi] = qacc;
      }
    }
    if (qpos_lds) vq[lane] = pf_qpos;
    __syncthreads();
    // positions are integrated in LDS and written back coalesced (global when nq > 64)
    float* gq = qpos_lds ? vq : d.qpos + (long)wid * nq;
    for (int j = lane; j < m.njnt; j += 64) {
      int qa = m.jnt_qposadr[j], da = m.jnt_dofadr[j], jt = m.jnt_type[j];
      if (jt == JNT_FREE) {
        float q[4], qn[4];
        for (int i = 0; i < 3; i++) gq[qa + i] = gq[qa + i] + dt * vd2[da + i];
        for (int i = 0; i < 4; i++) q[i] = gq[qa + 3 + i];
        quat_integrate(qn, q, vd2 + da + 3, dt);
        for (int i = 0; i < 4; i++) gq[qa + 3 + i] = qn[i];
      } else if (jt == JNT_BALL) {
        float q[4], qn[4];
        for (int i = 0; i < 4; i++) q[i] = gq[qa + i];
        quat_integrate(qn, q, vd2 + da, dt);
        for (int i = 0; i < 4; i++) gq[qa + i] = qn[i];
      } else {
        gq[qa] = gq[qa] + dt * vd2[da];
      }
    }
    if (qpos_lds) {
      __syncthreads();
      if (lane < nq) d.qpos[(long)wid * nq + lane] = vq[lane];
    }
    if (lane == 0) d.time[wid] = pf_time + dt;
  }
  PROF_MARK(PH_DEULER);
}

}  // namespace mjw
