// mjw_ccd.h -- convex collision for one geom pair: GJK distance, EPA penetration and box
// multi-contact (mujoco_warp/_src/collision_gjk.py; pair driver collision_convex.py:701-890).
//
// Execution model: the whole wavefront runs one pair at a time in lockstep (every lane
// computes the same values), so there is no divergence, and every array of the algorithm
// (GJK simplex, EPA polytope, clipping buffers) lives in a per-world LDS workspace instead of
// dynamically indexed registers (which would spill to scratch).  Pairs needing CCD are rare
// (box-box in the benchmark models) and run only when the broadphase keeps them.
#pragma once

#include "mjw_common.h"

namespace mjw {

constexpr float CCD_FLOAT_MAX = 1e30f;
constexpr float CCD_MINVAL = 1e-15f;
constexpr float CCD_MIN_DIST = 1e-10f;
constexpr int CCD_MAX_EPAFACES = 5;
constexpr int CCD_MAX_EPAHORIZON = 24;
constexpr float CCD_INTERSECT_TOL = 0.0000003f;
constexpr unsigned CCD_FACE_DELETED = 0x80000000u;
constexpr unsigned CCD_FACE_INVALID = 0x40000000u;

// one geom in the workspace: pos[3] rot[9] size[3] margin type mesh_vertadr mesh_vertnum mesh id
constexpr int CGEOM_WORDS = 20;
// per-pair result record in HBM (d.ccd_out): count, normal[3], then per point (dist, pos[3]) x 4, then per
// point normal[3] x 4 (words 20-31).  The convex pairs (GJK / EPA / box multi-contact) give every point the
// pair's distance and normal; the multi-point primitives the pre-passes also run (plane-cylinder,
// plane-mesh) give each point its own distance, and heightfield pairs each point its own distance and normal.
constexpr int CCD_OUT = 32;
// heightfield pairs (collision_convex.py:158-697): at most mjMAXCONPAIR prism contacts per pair
constexpr int HF_MAXCON = 50;
// heightfield scratch: the prism (6 x 3), then per prism contact dist, pos[3], normal[3]
constexpr int HF_WORDS = 18 + 7 * HF_MAXCON;

// LDS workspace layout (offsets in words) for epa_iterations = it
struct CcdLay {
  int vert, vidx, face, pr, norm2, horizon, simplex, sidx, coords, nrm, idx, endvert, f1, f2, pn, pd, poly, clip, w1, w2;
  int geoms, out, hf;
  int cap_vert, cap_face, npoly, ndeg, total;
};

// hf: reserve the heightfield scratch (models with heightfield geoms).  npoly / ndeg: the multi-contact
// buffers' bounds (collision_convex.py:1120-1140: a box face has 4 corners and a corner 3 faces; with
// MULTICCD on mesh pairs the model's largest polygon and vertex degree, m.nmaxpolygon / m.nmaxmeshdeg).
// The multi-contact buffers follow the fixed part, and the heightfield scratch comes last, so every
// offset but hf is the same with or without it.
__host__ __device__ inline CcdLay ccd_layout(int it, bool hf = false, int npoly = 4, int ndeg = 3) {
  CcdLay L;
  int o = 0;
  auto take = [&](int n) { int r = o; o += n; return r; };
  L.cap_vert = 10 + 2 * it;  // vec3 slots, two per polytope vertex (collision_convex.py:1146)
  L.cap_face = 6 + CCD_MAX_EPAFACES * it;
  L.npoly = npoly < 4 ? 4 : npoly;
  L.ndeg = ndeg < 3 ? 3 : ndeg;
  L.vert = take(L.cap_vert * 3); L.vidx = take(L.cap_vert);
  L.face = take(L.cap_face); L.pr = take(L.cap_face * 3); L.norm2 = take(L.cap_face);
  L.horizon = take(CCD_MAX_EPAHORIZON);
  L.simplex = take(3 * 4 * 3); L.sidx = take(2 * 4); L.coords = take(4);
  L.geoms = take(2 * CGEOM_WORDS); L.out = take(CCD_OUT);
  L.w1 = take(4 * 3); L.w2 = take(4 * 3);
  const int nclip = 2 * L.npoly > 16 ? 2 * L.npoly : 16;
  L.nrm = take(2 * L.ndeg * 3); L.idx = take(2 * L.ndeg); L.endvert = take(L.ndeg * 3);
  L.f1 = take(L.npoly * 3); L.f2 = take(L.npoly * 3); L.pn = take(L.npoly * 3); L.pd = take(L.npoly);
  L.poly = take(nclip * 3); L.clip = take(nclip * 3);
  L.hf = take(hf ? HF_WORDS : 0);
  L.total = o;
  return L;
}

// a mesh's polygon data (mesh_poly*: the model's arrays; collision_gjk.py:1403-1790 reads them)
struct MeshPoly {
  const float* polynormal;
  const int *polyadr, *polynum, *polyvertadr, *polyvertnum, *polyvert, *polymapadr, *polymapnum, *polymap, *vertadr;
};

struct CGeom {
  float pos[3], rot[9], size[3], margin;
  int type;
  const float* mv;  // mesh vertices (geom frame), GEOM_MESH only
  int nvert;
  const float* prism;  // GEOM_HFIELD: the 6 prism vertices (heightfield frame, LDS); pos = the prism center
  // GEOM_MESH polygon data, offset to this mesh (pnormal / pvadr / pvnum by its polygon address, pmapadr /
  // pmapnum by its vertex address; pvert / pmap hold mesh-local vertex / polygon ids); null: none
  const float* pnormal;
  const int *pvadr, *pvnum, *pvert, *pmapadr, *pmapnum, *pmap;
};

__device__ __forceinline__ float ccd_sign(float x) { return x < 0.0f ? -1.0f : 1.0f; }  // wp.sign

__device__ __forceinline__ void rot_apply(float* r, const float* R, float x, float y, float z) {
  for (int i = 0; i < 3; i++) r[i] = R[3 * i] * x + R[3 * i + 1] * y + R[3 * i + 2] * z;
}

// collision_gjk.py:97-190 (primitive geoms)
__device__ __forceinline__ void ccd_support(const CGeom& g, const float* dir, float* pt, int* vidx) {
  if (g.type == GEOM_HFIELD) {
    // collision_gjk.py:178-187: first strict maximum over the prism's vertices, already in the
    // heightfield frame (no pose); the index only tells the top (-3) from the bottom (-2) direction
    *vidx = dir[2] < 0.0f ? -2 : -3;
    float best = -CCD_FLOAT_MAX;
    pt[0] = pt[1] = pt[2] = 0.0f;
    for (int i = 0; i < 6; i++) {
      const float* v = g.prism + 3 * i;
      const float dd = v[0] * dir[0] + v[1] * dir[1] + v[2] * dir[2];
      if (dd > best) { best = dd; pt[0] = v[0]; pt[1] = v[1]; pt[2] = v[2]; }
    }
    if (g.margin > 0.0f)
      for (int i = 0; i < 3; i++) pt[i] += dir[i] * (0.5f * g.margin);
    return;
  }
  *vidx = -1;
  float ld[3], res[3] = {0.0f, 0.0f, 0.0f};
  for (int i = 0; i < 3; i++) ld[i] = g.rot[i] * dir[0] + g.rot[3 + i] * dir[1] + g.rot[6 + i] * dir[2];
  if (g.type == GEOM_SPHERE) {
    for (int i = 0; i < 3; i++) pt[i] = g.pos[i] + (g.size[0] + 0.5f * g.margin) * dir[i];
    return;
  }
  if (g.type == GEOM_BOX) {
    float t0 = ccd_sign(ld[0]), t1 = ccd_sign(ld[1]), t2 = ccd_sign(ld[2]);
    res[0] = t0 * g.size[0]; res[1] = t1 * g.size[1]; res[2] = t2 * g.size[2];
    *vidx = (t0 > 0.0f) + 2 * (t1 > 0.0f) + 4 * (t2 > 0.0f);
  } else if (g.type == GEOM_CAPSULE) {
    for (int i = 0; i < 3; i++) res[i] = ld[i] * g.size[0];
    res[2] += ccd_sign(ld[2]) * g.size[1];
  } else if (g.type == GEOM_ELLIPSOID) {
    for (int i = 0; i < 3; i++) res[i] = ld[i] * g.size[i];
    normalize3(res);
    for (int i = 0; i < 3; i++) res[i] *= g.size[i];
  } else if (g.type == GEOM_CYLINDER) {
    float dd = sqrtf(ld[0] * ld[0] + ld[1] * ld[1]);
    if (dd > CCD_MINVAL) { res[0] = ld[0] * g.size[0] / dd; res[1] = ld[1] * g.size[0] / dd; }
    res[2] = ccd_sign(ld[2]) * g.size[1];
  } else if (g.type == GEOM_MESH) {
    // collision_gjk.py:136-151 exhaustive search over the vertices, spread over the wave: each lane
    // keeps its strided subset's first maximum, a butterfly then keeps the largest (lowest index on
    // ties), i.e. the sequential loop's first strict maximum.  Every lane calls this in lockstep.
    float best = -CCD_FLOAT_MAX;
    int bi = 0x7fffffff;
    for (int i = (int)(threadIdx.x & 63); i < g.nvert; i += 64) {
      const float* v = g.mv + 3 * i;
      const float dd = v[0] * ld[0] + v[1] * ld[1] + v[2] * ld[2];
      if (dd > best) { best = dd; bi = i; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (bi < g.nvert) {
      const float* v = g.mv + 3 * bi;
      res[0] = v[0]; res[1] = v[1]; res[2] = v[2];
      *vidx = bi;
    }
  }
  rot_apply(pt, g.rot, res[0], res[1], res[2]);
  for (int i = 0; i < 3; i++) pt[i] += g.pos[i];
  if (g.margin > 0.0f)
    for (int i = 0; i < 3; i++) pt[i] += dir[i] * (0.5f * g.margin);
}

__device__ __forceinline__ float det3v(const float* a, const float* b, const float* c) {
  float t[3];
  cross3(t, b, c);
  return dot3(a, t);
}

__device__ __forceinline__ int same_sign(float a, float b) {
  if (a > 0.0f && b > 0.0f) return 1;
  if (a < 0.0f && b < 0.0f) return -1;
  return 0;
}

// collision_gjk.py:286-315 (returns 1 on degenerate input)
__device__ __forceinline__ int project_origin_plane(float* r, const float* v1, const float* v2, const float* v3) {
  float d21[3], d31[3], d32[3], n[3];
  for (int i = 0; i < 3; i++) { d21[i] = v2[i] - v1[i]; d31[i] = v3[i] - v1[i]; d32[i] = v3[i] - v2[i]; r[i] = 0.0f; }
  cross3(n, d32, d21);
  float nv = dot3(n, v2), nn = dot3(n, n);
  if (nn == 0.0f) return 1;
  if (nv != 0.0f && nn > CCD_MINVAL) { for (int i = 0; i < 3; i++) r[i] = (nv / nn) * n[i]; return 0; }
  cross3(n, d21, d31);
  nv = dot3(n, v1); nn = dot3(n, n);
  if (nn == 0.0f) return 1;
  if (nv != 0.0f && nn > CCD_MINVAL) { for (int i = 0; i < 3; i++) r[i] = (nv / nn) * n[i]; return 0; }
  cross3(n, d31, d32);
  nv = dot3(n, v3); nn = dot3(n, n);
  for (int i = 0; i < 3; i++) r[i] = (nv / nn) * n[i];
  return 0;
}

// collision_gjk.py:539-559
__device__ __forceinline__ void S1D(float* out, const float* s1, const float* s2) {
  float diff[3] = {s2[0] - s1[0], s2[1] - s1[1], s2[2] - s1[2]};
  float scl = -(dot3(s2, diff) / dot3(diff, diff));
  float p[3] = {s2[0] + scl * diff[0], s2[1] + scl * diff[1], s2[2] + scl * diff[2]};
  float mu_max = 0.0f, ps = 0.0f, s1s = 0.0f, s2s = 0.0f;
  for (int i = 0; i < 3; i++) {
    float mu = s1[i] - s2[i];
    if (fabsf(mu) >= fabsf(mu_max)) { mu_max = mu; ps = p[i]; s1s = s1[i]; s2s = s2[i]; }
  }
  float C1 = ps - s2s, C2 = s1s - ps;
  if (same_sign(mu_max, C1) && same_sign(mu_max, C2)) { out[0] = C1 / mu_max; out[1] = C2 / mu_max; }
  else { out[0] = 0.0f; out[1] = 1.0f; }
}

// pick the two coordinates that drop the axis with the largest projection (S2D / _tri_affine_coord)
__device__ __forceinline__ float proj2(const float* s1, const float* s2, const float* s3, int* xo, int* yo) {
  float M14 = s2[1] * s3[2] - s2[2] * s3[1] - s1[1] * s3[2] + s1[2] * s3[1] + s1[1] * s2[2] - s1[2] * s2[1];
  float M24 = s2[0] * s3[2] - s2[2] * s3[0] - s1[0] * s3[2] + s1[2] * s3[0] + s1[0] * s2[2] - s1[2] * s2[0];
  float M34 = s2[0] * s3[1] - s2[1] * s3[0] - s1[0] * s3[1] + s1[1] * s3[0] + s1[0] * s2[1] - s1[1] * s2[0];
  float mu1 = fabsf(M14), mu2 = fabsf(M24), mu3 = fabsf(M34);
  if (mu1 >= mu2 && mu1 >= mu3) { *xo = 1; *yo = 2; return M14; }
  if (mu2 >= mu3) { *xo = 0; *yo = 2; return M24; }
  *xo = 0; *yo = 1;
  return M34;
}

__device__ __forceinline__ float pick(const float* v, int i) { return i == 0 ? v[0] : (i == 1 ? v[1] : v[2]); }

// collision_gjk.py:394-536
__device__ __forceinline__ void S2D(float* out, const float* s1, const float* s2, const float* s3) {
  float p[3];
  if (project_origin_plane(p, s1, s2, s3)) {
    float v[2];
    S1D(v, s1, s2);
    out[0] = v[0]; out[1] = v[1]; out[2] = 0.0f;
    return;
  }
  int x, y;
  float Mmax = proj2(s1, s2, s3, &x, &y);
  float a0 = pick(s1, x), a1 = pick(s1, y), b0 = pick(s2, x), b1 = pick(s2, y), c0 = pick(s3, x), c1 = pick(s3, y);
  float o0 = pick(p, x), o1 = pick(p, y);
  float C31 = o0 * b1 + o1 * c0 + b0 * c1 - o0 * c1 - o1 * b0 - c0 * b1;
  float C32 = o0 * c1 + o1 * a0 + c0 * a1 - o0 * a1 - o1 * c0 - a0 * c1;
  float C33 = o0 * a1 + o1 * b0 + a0 * b1 - o0 * b1 - o1 * a0 - b0 * a1;
  int comp1 = same_sign(Mmax, C31), comp2 = same_sign(Mmax, C32), comp3 = same_sign(Mmax, C33);
  if (comp1 && comp2 && comp3) { out[0] = C31 / Mmax; out[1] = C32 / Mmax; out[2] = C33 / Mmax; return; }
  float dmin = CCD_FLOAT_MAX, sc[2], xx[3];
  out[0] = out[1] = out[2] = 0.0f;
  if (!comp1) {
    S1D(sc, s2, s3);
    for (int i = 0; i < 3; i++) xx[i] = sc[0] * s2[i] + sc[1] * s3[i];
    out[0] = 0.0f; out[1] = sc[0]; out[2] = sc[1];
    dmin = dot3(xx, xx);
  }
  if (!comp2) {
    S1D(sc, s1, s3);
    for (int i = 0; i < 3; i++) xx[i] = sc[0] * s1[i] + sc[1] * s3[i];
    float dd = dot3(xx, xx);
    if (dd < dmin) { out[0] = sc[0]; out[1] = 0.0f; out[2] = sc[1]; dmin = dd; }
  }
  if (!comp3) {
    S1D(sc, s1, s2);
    for (int i = 0; i < 3; i++) xx[i] = sc[0] * s1[i] + sc[1] * s2[i];
    float dd = dot3(xx, xx);
    if (dd < dmin) { out[0] = sc[0]; out[1] = sc[1]; out[2] = 0.0f; }
  }
}

// collision_gjk.py:318-391
__device__ __forceinline__ void S3D(float* out, const float* s1, const float* s2, const float* s3, const float* s4) {
  float C41 = -det3v(s2, s3, s4), C42 = det3v(s1, s3, s4), C43 = -det3v(s1, s2, s4), C44 = det3v(s1, s2, s3);
  float mdet = C41 + C42 + C43 + C44;
  int c1 = same_sign(mdet, C41), c2 = same_sign(mdet, C42), c3 = same_sign(mdet, C43), c4 = same_sign(mdet, C44);
  if (c1 && c2 && c3 && c4) { out[0] = C41 / mdet; out[1] = C42 / mdet; out[2] = C43 / mdet; out[3] = C44 / mdet; return; }
  float dmin = CCD_FLOAT_MAX, sc[3], xx[3];
  out[0] = out[1] = out[2] = out[3] = 0.0f;
  if (!c1) {
    S2D(sc, s2, s3, s4);
    for (int i = 0; i < 3; i++) xx[i] = sc[0] * s2[i] + sc[1] * s3[i] + sc[2] * s4[i];
    out[0] = 0.0f; out[1] = sc[0]; out[2] = sc[1]; out[3] = sc[2];
    dmin = dot3(xx, xx);
  }
  if (!c2) {
    S2D(sc, s1, s3, s4);
    for (int i = 0; i < 3; i++) xx[i] = sc[0] * s1[i] + sc[1] * s3[i] + sc[2] * s4[i];
    float dd = dot3(xx, xx);
    if (dd < dmin) { out[0] = sc[0]; out[1] = 0.0f; out[2] = sc[1]; out[3] = sc[2]; dmin = dd; }
  }
  if (!c3) {
    S2D(sc, s1, s2, s4);
    for (int i = 0; i < 3; i++) xx[i] = sc[0] * s1[i] + sc[1] * s2[i] + sc[2] * s4[i];
    float dd = dot3(xx, xx);
    if (dd < dmin) { out[0] = sc[0]; out[1] = sc[1]; out[2] = 0.0f; out[3] = sc[2]; dmin = dd; }
  }
  if (!c4) {
    S2D(sc, s1, s2, s3);
    for (int i = 0; i < 3; i++) xx[i] = sc[0] * s1[i] + sc[1] * s2[i] + sc[2] * s3[i];
    float dd = dot3(xx, xx);
    if (dd < dmin) { out[0] = sc[0]; out[1] = sc[1]; out[2] = sc[2]; out[3] = 0.0f; }
  }
}

// workspace accessors (W = LDS base of the world's CCD workspace)
struct CcdWS {
  float* W;
  CcdLay L;
  __device__ float* vert(int k) const { return W + L.vert + 3 * k; }  // k = 2 * v + (0: geom1, 1: geom2)
  __device__ int* vidx() const { return reinterpret_cast<int*>(W + L.vidx); }
  __device__ unsigned* face() const { return reinterpret_cast<unsigned*>(W + L.face); }
  __device__ float* pr(int f) const { return W + L.pr + 3 * f; }
  __device__ float* norm2() const { return W + L.norm2; }
  __device__ unsigned* horizon() const { return reinterpret_cast<unsigned*>(W + L.horizon); }
  __device__ float* simplex(int which, int k) const { return W + L.simplex + 12 * which + 3 * k; }  // 0: minkowski, 1: geom1, 2: geom2
  __device__ int* sidx(int which) const { return reinterpret_cast<int*>(W + L.sidx) + 4 * which; }
  __device__ float* coords() const { return W + L.coords; }
};

__device__ __forceinline__ void ld3(float* r, const float* p) { r[0] = p[0]; r[1] = p[1]; r[2] = p[2]; }
__device__ __forceinline__ void st3(float* p, const float* r) { p[0] = r[0]; p[1] = r[1]; p[2] = r[2]; }

struct GjkOut {
  float dist, x1[3], x2[3];
  int dim;
};

// collision_gjk.py:562-685 (simplex kept in the workspace)
__device__ __forceinline__ GjkOut gjk(const CcdWS& w, float tolerance, int iterations, const CGeom& g1, const CGeom& g2, float cutoff, int discrete) {
  GjkOut r;
  // a zero-initialised result (warp structs are): an early exit past the cutoff reports x1 = x2 = 0, which the
  // heightfield path caches as a (never active) prism contact at the heightfield's origin
  for (int i = 0; i < 3; i++) r.x1[i] = r.x2[i] = 0.0f;
  const float cutoff2 = cutoff * cutoff, tol2 = tolerance * tolerance;
  const float epsilon = discrete ? 0.0f : 0.5f * tol2;
  float* coords = w.coords();
  int n = 0;
  float xk[3] = {g1.pos[0] - g2.pos[0], g1.pos[1] - g2.pos[1], g1.pos[2] - g2.pos[2]};
  float xnorm_old = CCD_FLOAT_MAX;
  for (int it = 0; it < iterations; it++) {
    float xnorm = dot3(xk, xk);
    if (xnorm < tol2 || fabsf(xnorm_old - xnorm) < tol2) break;
    xnorm_old = xnorm;
    float sq = sqrtf(xnorm);
    float dneg[3] = {xk[0] / sq, xk[1] / sq, xk[2] / sq}, dpos[3] = {-dneg[0], -dneg[1], -dneg[2]};
    float p1[3], p2[3], sm[3];
    int i1, i2;
    ccd_support(g1, dpos, p1, &i1);
    ccd_support(g2, dneg, p2, &i2);
    for (int i = 0; i < 3; i++) sm[i] = p1[i] - p2[i];
    st3(w.simplex(1, n), p1); st3(w.simplex(2, n), p2); st3(w.simplex(0, n), sm);
    w.sidx(0)[n] = i1; w.sidx(1)[n] = i2;
    float vs = dot3(xk, sm);
    if (cutoff == 0.0f) {
      if (vs > 0.0f) { r.dim = 0; r.dist = CCD_FLOAT_MAX; return r; }
    } else if (cutoff < CCD_FLOAT_MAX) {
      if (vs > 0.0f && (vs * vs / xnorm) >= cutoff2) { r.dim = 0; r.dist = CCD_FLOAT_MAX; return r; }
    }
    float dk[3] = {xk[0] - sm[0], xk[1] - sm[1], xk[2] - sm[2]};
    if (dot3(xk, dk) < epsilon) break;
    float c4[4] = {1.0f, 0.0f, 0.0f, 0.0f};
    float s0[3], s1[3], s2[3], s3[3];
    ld3(s0, w.simplex(0, 0));
    if (n + 1 >= 2) ld3(s1, w.simplex(0, 1));
    if (n + 1 >= 3) ld3(s2, w.simplex(0, 2));
    if (n + 1 == 4) { ld3(s3, w.simplex(0, 3)); S3D(c4, s0, s1, s2, s3); }
    else if (n + 1 == 3) { S2D(c4, s0, s1, s2); c4[3] = 0.0f; }
    else if (n + 1 == 2) { S1D(c4, s0, s1); c4[2] = c4[3] = 0.0f; }
    n = 0;
    for (int i = 0; i < 4; i++) {
      if (c4[i] == 0.0f) continue;
      for (int s = 0; s < 3; s++) st3(w.simplex(s, n), w.simplex(s, i));
      w.sidx(0)[n] = w.sidx(0)[i];
      w.sidx(1)[n] = w.sidx(1)[i];
      coords[n] = c4[i];
      n++;
    }
    if (n < 1) break;
    float xn[3] = {0.0f, 0.0f, 0.0f};
    for (int k = 0; k < n; k++)
      for (int i = 0; i < 3; i++) xn[i] += coords[k] * w.simplex(0, k)[i];
    if (fabsf(xn[0] - xk[0]) < CCD_MINVAL && fabsf(xn[1] - xk[1]) < CCD_MINVAL && fabsf(xn[2] - xk[2]) < CCD_MINVAL) break;
    xk[0] = xn[0]; xk[1] = xn[1]; xk[2] = xn[2];
    if (n == 4) break;
  }
  if (n == 0) {
    st3(r.x1, g1.pos);
    st3(r.x2, g2.pos);
  } else {
    for (int i = 0; i < 3; i++) {
      float a = 0.0f, b = 0.0f;
      for (int k = 0; k < n; k++) { a += coords[k] * w.simplex(1, k)[i]; b += coords[k] * w.simplex(2, k)[i]; }
      r.x1[i] = a; r.x2[i] = b;
    }
  }
  r.dist = sqrtf(dot3(xk, xk));
  r.dim = n;
  return r;
}

__device__ __forceinline__ void pvert(const CcdWS& w, int v, float* out) {
  const float* a = w.vert(2 * v);
  const float* b = w.vert(2 * v + 1);
  for (int i = 0; i < 3; i++) out[i] = a[i] - b[i];
}

// collision_gjk.py:194-213
__device__ __forceinline__ float attach_face(const CcdWS& w, int nface, int idx, int v1, int v2, int v3) {
  if (nface == w.L.cap_face) return 0.0f;
  float p1[3], p2[3], p3[3], r[3];
  pvert(w, v1, p1); pvert(w, v2, p2); pvert(w, v3, p3);
  if (project_origin_plane(r, p3, p2, p1)) return 0.0f;
  w.face()[idx] = (unsigned)(v1 + (v2 << 10) + (v3 << 20));
  st3(w.pr(idx), r);
  float n2 = dot3(r, r);
  w.norm2()[idx] = n2;
  return n2;
}

// collision_gjk.py:216-230
__device__ __forceinline__ void epa_support(const CcdWS& w, int idx, const CGeom& g1, const CGeom& g2, const float* dir) {
  float nd[3] = {-dir[0], -dir[1], -dir[2]}, p[3];
  int vi;
  ccd_support(g1, dir, p, &vi);
  st3(w.vert(2 * idx), p);
  w.vidx()[2 * idx] = vi;
  ccd_support(g2, nd, p, &vi);
  st3(w.vert(2 * idx + 1), p);
  w.vidx()[2 * idx + 1] = vi;
}

// collision_gjk.py:701-741
__device__ __forceinline__ void tri_affine_coord(float* out, const float* v1, const float* v2, const float* v3, const float* p) {
  int x, y;
  float Mmax = proj2(v1, v2, v3, &x, &y);
  float px = pick(p, x), py = pick(p, y), v1x = pick(v1, x), v1y = pick(v1, y), v2x = pick(v2, x), v2y = pick(v2, y);
  float v3x = pick(v3, x), v3y = pick(v3, y);
  float C31 = px * v2y + py * v3x + v2x * v3y - px * v3y - py * v2x - v3x * v2y;
  float C32 = px * v3y + py * v1x + v3x * v1y - px * v1y - py * v3x - v1x * v3y;
  float C33 = px * v1y + py * v2x + v1x * v2y - px * v2y - py * v1x - v2x * v1y;
  out[0] = C31 / Mmax; out[1] = C32 / Mmax; out[2] = C33 / Mmax;
}

// collision_gjk.py:744-758
__device__ __forceinline__ bool tri_point_intersect(const float* v1, const float* v2, const float* v3, const float* p) {
  float c[3];
  tri_affine_coord(c, v1, v2, v3, p);
  if (c[0] < 0.0f || c[1] < 0.0f || c[2] < 0.0f) return false;
  float d[3];
  for (int i = 0; i < 3; i++) d[i] = v1[i] * c[0] + v2[i] * c[1] + v3[i] * c[2] - p[i];
  return sqrtf(dot3(d, d)) < CCD_MINVAL;
}

// collision_gjk.py:688-698
__device__ __forceinline__ bool same_side(const float* p0, const float* p1, const float* p2, const float* p3) {
  float a[3], b[3], n[3], c[3], m0[3] = {-p0[0], -p0[1], -p0[2]};
  for (int i = 0; i < 3; i++) { a[i] = p1[i] - p0[i]; b[i] = p2[i] - p0[i]; c[i] = p3[i] - p0[i]; }
  cross3(n, a, b);
  float d1 = dot3(n, c), d2 = dot3(n, m0);
  return (d1 > 0.0f && d2 > 0.0f) || (d1 < 0.0f && d2 < 0.0f);
}
__device__ __forceinline__ bool test_tetra(const float* p0, const float* p1, const float* p2, const float* p3) {
  return same_side(p0, p1, p2, p3) && same_side(p1, p2, p3, p0) && same_side(p2, p3, p0, p1) && same_side(p3, p0, p1, p2);
}

// collision_gjk.py:761-797: GJK simplex := polytope vertices v1 v2 v3
__device__ __forceinline__ void replace_simplex3(const CcdWS& w, int v1, int v2, int v3) {
  const int vs[3] = {v1, v2, v3};
  for (int k = 0; k < 3; k++) {
    float a[3], b[3];
    ld3(a, w.vert(2 * vs[k]));
    ld3(b, w.vert(2 * vs[k] + 1));
    st3(w.simplex(1, k), a);
    st3(w.simplex(2, k), b);
    float d[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
    st3(w.simplex(0, k), d);
    w.sidx(0)[k] = w.vidx()[2 * vs[k]];
    w.sidx(1)[k] = w.vidx()[2 * vs[k] + 1];
  }
}

// copy the GJK simplex (first n vertices) into the polytope
__device__ __forceinline__ void simplex_to_polytope(const CcdWS& w, int n) {
  for (int k = 0; k < n; k++) {
    st3(w.vert(2 * k), w.simplex(1, k));
    st3(w.vert(2 * k + 1), w.simplex(2, k));
    w.vidx()[2 * k] = w.sidx(0)[k];
    w.vidx()[2 * k + 1] = w.sidx(1)[k];
  }
}

// collision_gjk.py:936-1023; returns status (-1: fall back to polytope3 with the replaced simplex)
__device__ __forceinline__ int polytope2(const CcdWS& w, int* nvert, int* nface, const CGeom& g1, const CGeom& g2) {
  float s0[3], s1[3], diff[3];
  ld3(s0, w.simplex(0, 0));
  ld3(s1, w.simplex(0, 1));
  for (int i = 0; i < 3; i++) diff[i] = s1[i] - s0[i];
  float value = CCD_FLOAT_MAX;
  int index = 0;
  for (int i = 0; i < 3; i++)
    if (fabsf(diff[i]) < value) { value = fabsf(diff[i]); index = i; }
  float e[3] = {index == 0 ? 1.0f : 0.0f, index == 1 ? 1.0f : 0.0f, index == 2 ? 1.0f : 0.0f}, d1[3], d2[3], d3[3], R[9];
  cross3(d1, e, diff);
  {  // collision_gjk.py:800-819 (120 degree rotation about diff)
    float nn = sqrtf(dot3(diff, diff));
    float u1 = diff[0] / nn, u2 = diff[1] / nn, u3 = diff[2] / nn;
    const float s = 0.86602540378f, c = -0.5f;
    R[0] = c + u1 * u1 * (1.0f - c); R[1] = u1 * u2 * (1.0f - c) - u3 * s; R[2] = u1 * u3 * (1.0f - c) + u2 * s;
    R[3] = u2 * u1 * (1.0f - c) + u3 * s; R[4] = c + u2 * u2 * (1.0f - c); R[5] = u2 * u3 * (1.0f - c) - u1 * s;
    R[6] = u1 * u3 * (1.0f - c) - u2 * s; R[7] = u2 * u3 * (1.0f - c) + u1 * s; R[8] = c + u3 * u3 * (1.0f - c);
  }
  matvec3(d2, R, d1);
  matvec3(d3, R, d2);
  simplex_to_polytope(w, 2);
  float n1 = sqrtf(dot3(d1, d1)), n2 = sqrtf(dot3(d2, d2)), n3 = sqrtf(dot3(d3, d3));
  float u1[3] = {d1[0] / n1, d1[1] / n1, d1[2] / n1}, u2[3] = {d2[0] / n2, d2[1] / n2, d2[2] / n2};
  float u3[3] = {d3[0] / n3, d3[1] / n3, d3[2] / n3};
  epa_support(w, 2, g1, g2, u1);
  epa_support(w, 3, g1, g2, u2);
  epa_support(w, 4, g1, g2, u3);
  const int F[6][3] = {{0, 2, 3}, {0, 4, 2}, {0, 3, 4}, {1, 3, 2}, {1, 2, 4}, {1, 4, 3}};
  for (int k = 0; k < 6; k++) {
    if (attach_face(w, 0, k, F[k][0], F[k][1], F[k][2]) < CCD_MIN_DIST) {
      replace_simplex3(w, F[k][0], F[k][1], F[k][2]);
      return -1;
    }
  }
  float v2[3], v3[3], v4[3];
  pvert(w, 2, v2); pvert(w, 3, v3); pvert(w, 4, v4);
  {  // collision_gjk.py:822-832 _ray_triangle
    float a[3], b[3], c[3], dd[3];
    for (int i = 0; i < 3; i++) { a[i] = v2[i] - s0[i]; b[i] = v3[i] - s0[i]; c[i] = s1[i] - s0[i]; dd[i] = v4[i] - s0[i]; }
    float vol1 = det3v(a, b, c), vol2 = det3v(b, dd, c), vol3 = det3v(dd, a, c);
    bool hit = (vol1 >= 0.0f && vol2 >= 0.0f && vol3 >= 0.0f) || (vol1 <= 0.0f && vol2 <= 0.0f && vol3 <= 0.0f);
    if (!hit) return 1;
  }
  *nvert = 5;
  *nface = 6;
  return 0;
}

// collision_gjk.py:1026-1111
__device__ __forceinline__ int polytope3(const CcdWS& w, int* nvert, int* nface, float dist, const CGeom& g1, const CGeom& g2) {
  float v1[3], v2[3], v3[3], a[3], b[3], n[3];
  ld3(v1, w.simplex(0, 0)); ld3(v2, w.simplex(0, 1)); ld3(v3, w.simplex(0, 2));
  for (int i = 0; i < 3; i++) { a[i] = v2[i] - v1[i]; b[i] = v3[i] - v1[i]; }
  cross3(n, a, b);
  if (sqrtf(dot3(n, n)) < CCD_MINVAL) return 2;
  simplex_to_polytope(w, 3);
  float nn[3] = {-n[0], -n[1], -n[2]};
  epa_support(w, 3, g1, g2, nn);
  epa_support(w, 4, g1, g2, n);
  float v4[3], v5[3];
  pvert(w, 3, v4); pvert(w, 4, v5);
  if (tri_point_intersect(v1, v2, v3, v4)) return 3;
  if (tri_point_intersect(v1, v2, v3, v5)) return 4;
  if (dist > 1e-5f && !test_tetra(v1, v2, v3, v4) && !test_tetra(v1, v2, v3, v5)) return 5;
  const int F[6][3] = {{4, 0, 1}, {4, 2, 0}, {4, 1, 2}, {3, 1, 0}, {3, 0, 2}, {3, 2, 1}};
  for (int k = 0; k < 6; k++)
    if (attach_face(w, 0, k, F[k][0], F[k][1], F[k][2]) < CCD_MIN_DIST) return 6 + k;
  *nvert = 5;
  *nface = 6;
  return 0;
}

// collision_gjk.py:1114-1168
__device__ __forceinline__ int polytope4(const CcdWS& w, int* nvert, int* nface) {
  simplex_to_polytope(w, 4);
  const int F[4][3] = {{0, 1, 2}, {0, 3, 1}, {0, 2, 3}, {3, 2, 1}};
  for (int k = 0; k < 4; k++) {
    if (attach_face(w, 0, k, F[k][0], F[k][1], F[k][2]) < CCD_MIN_DIST) {
      replace_simplex3(w, F[k][0], F[k][1], F[k][2]);
      return -1;
    }
  }
  float s0[3], s1[3], s2[3], s3[3];
  ld3(s0, w.simplex(0, 0)); ld3(s1, w.simplex(0, 1)); ld3(s2, w.simplex(0, 2)); ld3(s3, w.simplex(0, 3));
  if (!test_tetra(s0, s1, s2, s3)) return 12;
  *nvert = 4;
  *nface = 4;
  return 0;
}

__device__ __forceinline__ void face_verts(unsigned f, int* v) { v[0] = f & 0x3FF; v[1] = (f >> 10) & 0x3FF; v[2] = (f >> 20) & 0x3FF; }

// collision_gjk.py:840-858
__device__ __forceinline__ int add_edge(const CcdWS& w, int n, int e1, int e2) {
  if (n < 0) return -1;
  unsigned edge = (unsigned)(((e1 < e2 ? e1 : e2) << 10) | (e1 > e2 ? e1 : e2));
  unsigned* hz = w.horizon();
  for (int i = 0; i < n; i++)
    if (edge == hz[i]) { hz[i] = hz[n - 1]; return n - 1; }
  if (n == CCD_MAX_EPAHORIZON) return -1;
  hz[n] = edge;
  return n + 1;
}

// collision_gjk.py:2173-2186 / 914-921: the heightfield-side witness below x2 on the prism's top triangle
// (its vertical projection when inside, else onto the plane through the nearest corner); returns -|x1 - x2|
__device__ __forceinline__ float hfield_top_witness(const CGeom& g1, const float* x2, float* x1) {
  const float *a = g1.prism + 9, *b = g1.prism + 12, *c = g1.prism + 15;
  float co[3];
  tri_affine_coord(co, a, b, c, x2);
  if (co[0] > 0.0f && co[1] > 0.0f && co[2] > 0.0f) {
    for (int i = 0; i < 3; i++) x1[i] = co[0] * a[i] + co[1] * b[i] + co[2] * c[i];
  } else {
    const float* p = co[0] > 0.0f ? a : (co[1] > 0.0f ? b : c);
    const float dz = x2[2] - p[2];  // dot(x2 - p, n), n = +z
    x1[0] = x2[0]; x1[1] = x2[1]; x1[2] = x2[2] - dz;
  }
  float dd[3] = {x1[0] - x2[0], x1[1] - x2[1], x1[2] - x2[2]};
  return -sqrtf(dot3(dd, dd));
}

// collision_gjk.py:1201-1328 + witness :861-933; returns the face index or -1
__device__ __forceinline__ int epa(const CcdWS& w, int nvert, int nface, float tolerance, int iterations, const CGeom& g1, const CGeom& g2, int discrete,
                   float* dist, float* x1, float* x2) {
  float upper = CCD_FLOAT_MAX, upper2 = CCD_FLOAT_MAX;
  int idx = -1, pidx = -1;
  const float epsilon = discrete ? 1e-15f : tolerance;
  int nvalid = nface;
  unsigned* face = w.face();
  float* norm2 = w.norm2();
  if (iterations > 1000) iterations = 1000;
  for (int it = 0; it < iterations; it++) {
    pidx = idx;
    idx = -1;
    float lower2 = CCD_FLOAT_MAX;
    for (int i = 0; i < nface; i++)
      if (!(face[i] & (CCD_FACE_DELETED | CCD_FACE_INVALID)) && norm2[i] < lower2) { idx = i; lower2 = norm2[i]; }
    if (lower2 > upper2 || idx < 0) { idx = pidx; break; }
    if (lower2 <= 0.0f) break;
    const float lower = sqrtf(lower2);
    const int wi = nvert;
    float dir[3], wv[3];
    ld3(dir, w.pr(idx));
    for (int i = 0; i < 3; i++) dir[i] /= lower;
    epa_support(w, wi, g1, g2, dir);
    pvert(w, wi, wv);
    nvert++;
    float upper_k = dot3(dir, wv);
    if (upper_k < upper) { upper = upper_k; upper2 = upper * upper; }
    if (upper - lower < epsilon) break;
    if (discrete) {
      bool rep = false;
      const int* vi = w.vidx();
      for (int i = 0; i < nvert - 1; i++)
        if (vi[2 * i] == vi[2 * wi] && vi[2 * i + 1] == vi[2 * wi + 1]) { rep = true; break; }
      if (rep) break;
    }
    nvalid--;
    face[idx] |= CCD_FACE_DELETED;
    int f[3];
    face_verts(face[idx], f);
    int nh = add_edge(w, 0, f[0], f[1]);
    nh = add_edge(w, nh, f[1], f[2]);
    nh = add_edge(w, nh, f[2], f[0]);
    if (nh == -1) { idx = -1; break; }
    for (int i = 0; i < nface; i++) {
      if (face[i] & CCD_FACE_DELETED) continue;
      if (dot3(w.pr(i), wv) - norm2[i] > 1e-10f) {
        if (!(face[i] & CCD_FACE_INVALID)) nvalid--;
        face[i] |= CCD_FACE_DELETED;
        face_verts(face[i], f);
        nh = add_edge(w, nh, f[0], f[1]);
        nh = add_edge(w, nh, f[1], f[2]);
        nh = add_edge(w, nh, f[2], f[0]);
        if (nh == -1) { idx = -1; break; }
      }
    }
    for (int i = 0; i < nh; i++) {
      unsigned e = w.horizon()[i];
      float d2 = attach_face(w, nface, nface, wi, e & 0x3FF, (e >> 10) & 0x3FF);
      if (d2 == 0.0f) { idx = -1; break; }
      nface++;
      if (d2 >= lower2 && d2 <= upper2) nvalid++;
      else face[nface - 1] |= CCD_FACE_INVALID;
    }
    if (nvalid == 0 || idx == -1) break;
  }
  if (idx < 0) { *dist = 0.0f; return -1; }
  int f[3];
  face_verts(face[idx], f);
  float v1[3], v2[3], v3[3], c[3], p[3];
  pvert(w, f[0], v1); pvert(w, f[1], v2); pvert(w, f[2], v3);
  ld3(p, w.pr(idx));
  tri_affine_coord(c, v1, v2, v3, p);
  for (int i = 0; i < 3; i++) {
    x2[i] = w.vert(2 * f[0] + 1)[i] * c[0] + w.vert(2 * f[1] + 1)[i] * c[1] + w.vert(2 * f[2] + 1)[i] * c[2];
    x1[i] = w.vert(2 * f[0])[i] * c[0] + w.vert(2 * f[1])[i] * c[1] + w.vert(2 * f[2])[i] * c[2];
  }
  const int* vi = w.vidx();
  if (g1.type == GEOM_HFIELD && (vi[2 * f[0]] != vi[2 * f[1]] || vi[2 * f[0]] != vi[2 * f[2]])) {
    // collision_gjk.py:886-922: a face spanning the prism's top and bottom -- geom2's support point
    // against the top triangle instead
    float sp[3];
    int si;
    if (g2.type == GEOM_CAPSULE || g2.type == GEOM_SPHERE) {
      CGeom g = g2;
      g.margin = 0.0f;
      g.size[0] = 0.0f;
      ccd_support(g, x2, sp, &si);
      for (int i = 0; i < 3; i++) x2[i] = sp[i];
      x2[2] -= 0.5f * g2.margin + g2.size[0];
    } else {
      normalize3(x2);
      ccd_support(g2, x2, sp, &si);
      for (int i = 0; i < 3; i++) x2[i] = sp[i];
    }
    *dist = hfield_top_witness(g1, x2, x1);
    return idx;
  }
  *dist = -sqrtf(norm2[idx]);
  return idx;
}

// ---- box multi-contact (collision_gjk.py:1331-2150, box branches) -----------------------
__device__ __forceinline__ float area4(const float* a, const float* b, const float* c, const float* d) {
  float t1[3], t2[3], c1[3], c2[3];
  for (int i = 0; i < 3; i++) { t1[i] = a[i] - d[i]; t2[i] = d[i] - b[i]; }
  cross3(c1, t1, t2);
  for (int i = 0; i < 3; i++) { t1[i] = b[i] - c[i]; t2[i] = c[i] - a[i]; }
  cross3(c2, t1, t2);
  for (int i = 0; i < 3; i++) c1[i] += c2[i];
  return 0.5f * sqrtf(dot3(c1, c1));
}

// collision_gjk.py:1337-1374 (poly: LDS, stride 3)
__device__ __forceinline__ void polygon_quad(int* res, const float* poly, int np) {
  int b = 1, c = 2, d = 3;
  res[0] = 0; res[1] = b; res[2] = c; res[3] = d;
  float m = area4(poly, poly + 3 * b, poly + 3 * c, poly + 3 * d);
  for (int a = 0; a < np; a++) {
    while (true) {
      float mn = area4(poly + 3 * a, poly + 3 * b, poly + 3 * c, poly + 3 * ((d + 1) % np));
      if (mn <= m) break;
      m = mn; d = (d + 1) % np;
      res[0] = a; res[1] = b; res[2] = c; res[3] = d;
      while (true) {
        mn = area4(poly + 3 * a, poly + 3 * b, poly + 3 * ((c + 1) % np), poly + 3 * d);
        if (mn <= m) break;
        m = mn; c = (c + 1) % np;
        res[0] = a; res[1] = b; res[2] = c; res[3] = d;
      }
      while (true) {
        mn = area4(poly + 3 * a, poly + 3 * ((b + 1) % np), poly + 3 * c, poly + 3 * d);
        if (mn <= m) break;
        m = mn; b = (b + 1) % np;
        res[0] = a; res[1] = b; res[2] = c; res[3] = d;
      }
    }
    if (b == a) {
      b = (b + 1) % np;
      if (c == b) {
        c = (c + 1) % np;
        if (d == c) d = (d + 1) % np;
      }
    }
  }
}

// collision_gjk.py:1377-1400 (feature vertices stay in the polytope: returns their vert slots)
__device__ __forceinline__ int feature_dim(const CcdWS& w, const int* face, int offset, int* fi, int* fslot) {
  const int* vi = w.vidx();
  int v1i = vi[2 * face[0] + offset], v2i = vi[2 * face[1] + offset], v3i = vi[2 * face[2] + offset];
  fi[0] = v1i; fi[1] = v2i; fi[2] = v3i;
  fslot[0] = 2 * face[0] + offset; fslot[1] = 2 * face[1] + offset; fslot[2] = 2 * face[2] + offset;
  if (v1i != v2i) return (v3i == v1i || v3i == v2i) ? 2 : 3;
  fi[1] = v3i;
  fslot[1] = 2 * face[2] + offset;
  return v1i != v3i ? 2 : 1;
}

// collision_gjk.py:1577-1607
__device__ __forceinline__ int box_normals2(const float* mat, const float* n, float* nout, int* iout) {
  float ln[3];
  for (int i = 0; i < 3; i++) ln[i] = mat[i] * n[0] + mat[3 + i] * n[1] + mat[6 + i] * n[2];
  normalize3(ln);
  const float tol = cosf(0.0016f);
  for (int i = 0; i < 6; i++) {
    const float s = (i & 1) ? -1.0f : 1.0f;
    const int ax = i >> 1;
    if (s * pick(ln, ax) > tol) {
      rot_apply(nout, mat, ax == 0 ? s : 0.0f, ax == 1 ? s : 0.0f, ax == 2 ? s : 0.0f);
      iout[0] = i;
      return 1;
    }
  }
  return 0;
}

// collision_gjk.py:1610-1681 (nout: 3 normals, stride 3; iout: 3 ints)
__device__ __forceinline__ int box_normals(int dim, const int* fi, const float* mat, const float* dir, float* nout, int* iout) {
  const int v1 = fi[0], v2 = fi[1], v3 = fi[2];
  if (dim == 3) {
    int c = 0;
    float x = (float)((v1 & 1) && (v2 & 1) && (v3 & 1)) - (float)(!(v1 & 1) && !(v2 & 1) && !(v3 & 1));
    float y = (float)((v1 & 2) && (v2 & 2) && (v3 & 2)) - (float)(!(v1 & 2) && !(v2 & 2) && !(v3 & 2));
    float z = (float)((v1 & 4) && (v2 & 4) && (v3 & 4)) - (float)(!(v1 & 4) && !(v2 & 4) && !(v3 & 4));
    rot_apply(nout, mat, x, y, z);
    float sgn = x + y + z;
    if (x != 0.0f) iout[c++] = 0;
    if (y != 0.0f) iout[c++] = 2;
    if (z != 0.0f) iout[c++] = 4;
    if (sgn == -1.0f) iout[0] = iout[0] + 1;
    if (c == 1) return 1;
    return box_normals2(mat, dir, nout, iout);
  }
  if (dim == 2) {
    int c = 0;
    float x = (float)((v1 & 1) && (v2 & 1)) - (float)(!(v1 & 1) && !(v2 & 1));
    float y = (float)((v1 & 2) && (v2 & 2)) - (float)(!(v1 & 2) && !(v2 & 2));
    float z = (float)((v1 & 4) && (v2 & 4)) - (float)(!(v1 & 4) && !(v2 & 4));
    if (x != 0.0f) { rot_apply(nout + 3 * c, mat, x, 0.0f, 0.0f); iout[c] = x > 0.0f ? 0 : 1; c++; }
    if (y != 0.0f) { rot_apply(nout + 3 * c, mat, 0.0f, y, 0.0f); iout[c] = y > 0.0f ? 2 : 3; c++; }
    if (z != 0.0f) { rot_apply(nout + 3 * c, mat, 0.0f, 0.0f, z); iout[c] = z > 0.0f ? 4 : 5; c++; }
    if (c == 1 || c == 2) return c;
    return box_normals2(mat, dir, nout, iout);
  }
  if (dim == 1) {
    float x = (v1 & 1) ? 1.0f : -1.0f, y = (v1 & 2) ? 1.0f : -1.0f, z = (v1 & 4) ? 1.0f : -1.0f;
    rot_apply(nout, mat, x, 0.0f, 0.0f);
    rot_apply(nout + 3, mat, 0.0f, y, 0.0f);
    rot_apply(nout + 6, mat, 0.0f, 0.0f, z);
    iout[0] = x > 0.0f ? 0 : 1; iout[1] = y > 0.0f ? 2 : 3; iout[2] = z > 0.0f ? 4 : 5;
    return 3;
  }
  return 0;
}

// collision_gjk.py:1684-1719
__device__ __forceinline__ int box_edge_normals(int dim, const CGeom& g, const float* v1, const float* v2, int v1i, float* nout, float* endvert) {
  if (dim == 2) {
    st3(endvert, v2);
    float t[3] = {v2[0] - v1[0], v2[1] - v1[1], v2[2] - v1[2]};
    normalize3(t);
    st3(nout, t);
    return 1;
  }
  if (dim == 1) {
    const float x = (v1i & 1) ? g.size[0] : -g.size[0], y = (v1i & 2) ? g.size[1] : -g.size[1], z = (v1i & 4) ? g.size[2] : -g.size[2];
    for (int k = 0; k < 3; k++) {
      float e[3];
      rot_apply(e, g.rot, k == 0 ? -x : x, k == 1 ? -y : y, k == 2 ? -z : z);
      for (int i = 0; i < 3; i++) e[i] += g.pos[i];
      st3(endvert + 3 * k, e);
      float t[3] = {e[0] - v1[0], e[1] - v1[1], e[2] - v1[2]};
      normalize3(t);
      st3(nout + 3 * k, t);
    }
    return 3;
  }
  return 0;
}

// collision_gjk.py:1722-1762
__device__ __forceinline__ int box_face(const CGeom& g, int idx, float* fo) {
  // corner sign patterns per face (x, y, z bits: 1 = +size)
  const unsigned char SG[6][4] = {{7, 3, 1, 5}, {2, 6, 4, 0}, {2, 3, 7, 6}, {4, 5, 1, 0}, {6, 7, 5, 4}, {3, 2, 0, 1}};
  if (idx < 0 || idx > 5) return 0;
  for (int k = 0; k < 4; k++) {
    const int c = SG[idx][k];
    float e[3];
    rot_apply(e, g.rot, (c & 1) ? g.size[0] : -g.size[0], (c & 2) ? g.size[1] : -g.size[1], (c & 4) ? g.size[2] : -g.size[2]);
    for (int i = 0; i < 3; i++) fo[3 * k + i] = e[i] + g.pos[i];
  }
  return 4;
}

// collision_gjk.py:1815-1909; w1 / w2: witness outputs (stride 3)
__device__ __forceinline__ int polygon_clip(const CcdWS& w, const float* face1, int nface1, const float* face2, int nface2, const float* n, const float* dir,
                            float* w1, float* w2) {
  if (nface1 < 3) return 0;
  float* pn = w.W + w.L.pn;
  float* pd = w.W + w.L.pd;
  for (int i = 0; i < nface1; i++) {
    const float* v1 = face1 + 3 * i;
    const float* v2 = face1 + 3 * ((i + 1) % nface1);
    float a[3], b[3], r[3];
    for (int k = 0; k < 3; k++) { a[k] = v2[k] - v1[k]; b[k] = n[k]; }
    cross3(r, a, b);
    st3(pn + 3 * i, r);
    pd[i] = dot3(r, v1);
  }
  float* poly = w.W + w.L.poly;
  float* clip = w.W + w.L.clip;
  const int ncap = 2 * w.L.npoly > 16 ? 2 * w.L.npoly : 16;
  int np = nface2, nc = 0;
  for (int i = 0; i < 3 * nface2; i++) poly[i] = face2[i];
  for (int e = 0; e < nface1; e++) {
    const float* fe = face1 + 3 * e;
    float pne[3];
    ld3(pne, pn + 3 * e);
    for (int i = 0; i < np; i++) {
      float P[3], Q[3];
      ld3(P, poly + 3 * i);
      ld3(Q, poly + 3 * ((i + 1) % np));
      float dP[3] = {P[0] - fe[0], P[1] - fe[1], P[2] - fe[2]}, dQ[3] = {Q[0] - fe[0], Q[1] - fe[1], Q[2] - fe[2]};
      const bool in1 = dot3(dP, pne) > -1e-10f, in2 = dot3(dQ, pne) > -1e-10f;
      if (!in1 && !in2) continue;
      if (nc >= ncap - 2) break;  // buffer guard (a convex n-gon clipped by an m-gon has <= n + m vertices)
      if (in1 && in2) { st3(clip + 3 * nc, Q); nc++; continue; }
      float PQ[3] = {Q[0] - P[0], Q[1] - P[1], Q[2] - P[2]};
      float dt = dot3(pne, PQ);
      float t = fabsf(dt) < 1e-10f ? CCD_FLOAT_MAX : (pd[e] - dot3(pne, P)) / dt;
      if (t > -CCD_INTERSECT_TOL && t < 1.0f + CCD_INTERSECT_TOL) {
        t = clampf(t, 0.0f, 1.0f);
        float X[3] = {P[0] + t * PQ[0], P[1] + t * PQ[1], P[2] + t * PQ[2]};
        st3(clip + 3 * nc, X);
        nc++;
      }
      if (in2) { st3(clip + 3 * nc, Q); nc++; }
    }
    float* tmp = poly;
    poly = clip;
    clip = tmp;
    np = nc;
    nc = 0;
  }
  if (np < 1) return 0;
  if (np > 4) {
    int q[4];
    polygon_quad(q, poly, np);
    for (int i = 0; i < 4; i++)
      for (int k = 0; k < 3; k++) { w2[3 * i + k] = poly[3 * q[i] + k]; w1[3 * i + k] = w2[3 * i + k] - dir[k]; }
    return 4;
  }
  for (int i = 0; i < np; i++)
    for (int k = 0; k < 3; k++) { w2[3 * i + k] = poly[3 * i + k]; w1[3 * i + k] = w2[3 * i + k] - dir[k]; }
  return np;
}

// collision_gjk.py:1427-1456 _intersect1 / _intersect2: up to two common entries, in a1's order
__device__ __forceinline__ int mesh_intersect(const int* a1, int n1, const int* a2, int n2, int* res) {
  int count = 0;
  for (int i = 0; i < n1; i++)
    for (int j = 0; j < n2; j++)
      if (a1[i] == a2[j]) {
        res[count++] = a1[i];
        if (count == 2) return 2;
      }
  return count;
}

// collision_gjk.py:1460-1527 _mesh_normals (nout: LDS, stride 3; iout: LDS)
__device__ __forceinline__ int mesh_normals(int dim, const int* fi, const CGeom& g, float* nout, int* iout, int ndeg) {
  const int v1 = fi[0], v2 = fi[1], v3 = fi[2];
  int edge[2], face[2], n;
  if (dim == 3) {
    n = mesh_intersect(g.pmap + g.pmapadr[v1], g.pmapnum[v1], g.pmap + g.pmapadr[v2], g.pmapnum[v2], edge);
    if (n == 0) return 0;
    n = mesh_intersect(edge, n, g.pmap + g.pmapadr[v3], g.pmapnum[v3], face);
    if (n == 0) return 0;
    const float* pn = g.pnormal + 3 * face[0];
    rot_apply(nout, g.rot, pn[0], pn[1], pn[2]);
    iout[0] = face[0];
    return 1;
  }
  if (dim == 2) {
    n = mesh_intersect(g.pmap + g.pmapadr[v1], g.pmapnum[v1], g.pmap + g.pmapadr[v2], g.pmapnum[v2], edge);
    for (int i = 0; i < n; i++) {
      const float* pn = g.pnormal + 3 * edge[i];
      rot_apply(nout + 3 * i, g.rot, pn[0], pn[1], pn[2]);
      iout[i] = edge[i];
    }
    return n;
  }
  if (dim == 1) {
    const int num = min(g.pmapnum[v1], ndeg);
    for (int i = 0; i < num; i++) {
      const int idx = g.pmap[g.pmapadr[v1] + i];
      const float* pn = g.pnormal + 3 * idx;
      rot_apply(nout + 3 * i, g.rot, pn[0], pn[1], pn[2]);
      iout[i] = idx;
    }
    return num;
  }
  return 0;
}

// collision_gjk.py:1530-1574 _mesh_edge_normals
__device__ __forceinline__ int mesh_edge_normals(int dim, const CGeom& g, const float* v1, const float* v2, int v1i, float* nout, float* endvert,
                                                 int ndeg) {
  if (dim == 2) {
    st3(endvert, v2);
    float t[3] = {v2[0] - v1[0], v2[1] - v1[1], v2[2] - v1[2]};
    normalize3(t);
    st3(nout, t);
    return 1;
  }
  if (dim == 1) {
    const int num = min(g.pmapnum[v1i], ndeg);
    for (int i = 0; i < num; i++) {
      const int idx = g.pmap[g.pmapadr[v1i] + i];
      const int adr = g.pvadr[idx], nv = g.pvnum[idx];
      for (int j = 0; j < nv; j++) {
        if (g.pvert[adr + j] != v1i) continue;
        const int k = j == 0 ? nv - 1 : j - 1;
        const float* vk = g.mv + 3 * g.pvert[adr + k];
        float e[3];
        rot_apply(e, g.rot, vk[0], vk[1], vk[2]);
        for (int c = 0; c < 3; c++) e[c] += g.pos[c];
        st3(endvert + 3 * i, e);
        float t[3] = {e[0] - v1[0], e[1] - v1[1], e[2] - v1[2]};
        normalize3(t);
        st3(nout + 3 * i, t);
      }
    }
    return num;
  }
  return 0;
}

// collision_gjk.py:1765-1787 _mesh_face: polygon idx in world coordinates, its loop reversed
__device__ __forceinline__ int mesh_face(const CGeom& g, int idx, float* fo, int npoly) {
  const int adr = g.pvadr[idx], nv = min(g.pvnum[idx], npoly);
  int j = 0;
  for (int i = nv - 1; i >= 0; i--, j++) {
    const float* v = g.mv + 3 * g.pvert[adr + i];
    float e[3];
    rot_apply(e, g.rot, v[0], v[1], v[2]);
    for (int c = 0; c < 3; c++) fo[3 * j + c] = e[c] + g.pos[c];
  }
  return nv;
}

// collision_gjk.py:1929-2150 multicontact (boxes, and meshes with polygon data); witnesses in the
// workspace (w1 / w2)
__device__ __forceinline__ int multicontact(const CcdWS& w, int fidx, const float* x1, const float* x2, const CGeom& g1, const CGeom& g2) {
  float* W1 = w.W + w.L.w1;
  float* W2 = w.W + w.L.w2;
  st3(W1, x1);
  st3(W2, x2);
  int face[3];
  face_verts(w.face()[fidx], face);
  int fi1[3], fi2[3], fs1[3], fs2[3];
  const int nface1 = feature_dim(w, face, 0, fi1, fs1);
  const int nface2 = feature_dim(w, face, 1, fi2, fs2);
  float dir[3] = {x2[0] - x1[0], x2[1] - x1[1], x2[2] - x1[2]}, dneg[3] = {-dir[0], -dir[1], -dir[2]};
  const int ndeg = w.L.ndeg, npoly = w.L.npoly;
  float* n1 = w.W + w.L.nrm;
  float* n2 = n1 + 3 * ndeg;
  int* idx1 = reinterpret_cast<int*>(w.W + w.L.idx);
  int* idx2 = idx1 + ndeg;
  float* endvert = w.W + w.L.endvert;
  int nn1 = g1.type == GEOM_BOX ? box_normals(nface1, fi1, g1.rot, dneg, n1, idx1) : mesh_normals(nface1, fi1, g1, n1, idx1, ndeg);
  int nn2 = g2.type == GEOM_BOX ? box_normals(nface2, fi2, g2.rot, dir, n2, idx2) : mesh_normals(nface2, fi2, g2, n2, idx2, ndeg);
  const float face_tol = cosf(0.0016f), edge_tol = sinf(0.0016f);
  int edge1 = 0, edge2 = 0, ri = 0, rj = 0;
  bool found = false;
  for (int i = 0; i < nn1 && !found; i++)
    for (int j = 0; j < nn2; j++)
      if (dot3(n1 + 3 * i, n2 + 3 * j) < -face_tol) { ri = i; rj = j; found = true; break; }
  if (!found) {
    if (nface1 < 3 && nface1 <= nface2) {
      nn1 = g1.type == GEOM_BOX ? box_edge_normals(nface1, g1, w.vert(fs1[0]), w.vert(fs1[1]), fi1[0], n1, endvert)
                                : mesh_edge_normals(nface1, g1, w.vert(fs1[0]), w.vert(fs1[1]), fi1[0], n1, endvert, ndeg);
      for (int i = 0; i < nn2 && !found; i++)
        for (int j = 0; j < nn1; j++)
          if (fabsf(dot3(n1 + 3 * j, n2 + 3 * i)) < edge_tol) { ri = j; rj = i; found = true; break; }
      if (!found) return 1;
      edge1 = 1;
    } else if (nface2 < 3) {
      nn2 = g2.type == GEOM_BOX ? box_edge_normals(nface2, g2, w.vert(fs2[0]), w.vert(fs2[1]), fi2[0], n2, endvert)
                                : mesh_edge_normals(nface2, g2, w.vert(fs2[0]), w.vert(fs2[1]), fi2[0], n2, endvert, ndeg);
      for (int i = 0; i < nn1 && !found; i++)
        for (int j = 0; j < nn2; j++)
          if (fabsf(dot3(n2 + 3 * j, n1 + 3 * i)) < edge_tol) { ri = j; rj = i; found = true; break; }
      if (!found) return 1;
      edge2 = 1;
    } else {
      return 1;
    }
  }
  float* f1 = w.W + w.L.f1;
  float* f2 = w.W + w.L.f2;
  int nf1, nf2;
  if (edge1) {
    st3(f1, w.vert(2 * face[0]));
    st3(f1 + 3, endvert + 3 * ri);
    nf1 = 2;
  } else {
    const int ind = edge2 ? idx1[rj] : idx1[ri];
    nf1 = g1.type == GEOM_BOX ? box_face(g1, ind, f1) : mesh_face(g1, ind, f1, npoly);
  }
  if (edge2) {
    st3(f2, w.vert(2 * face[0] + 1));
    st3(f2 + 3, endvert + 3 * ri);
    nf2 = 2;
  } else {
    nf2 = g2.type == GEOM_BOX ? box_face(g2, idx2[rj], f2) : mesh_face(g2, idx2[rj], f2, npoly);
  }
  const float dl = sqrtf(dot3(dir, dir));
  float ad[3], nrm[3];
  if (edge1) {
    ld3(nrm, n2 + 3 * rj);
    for (int i = 0; i < 3; i++) ad[i] = dl * nrm[i];
    return polygon_clip(w, f2, nf2, f1, nf1, nrm, ad, W1, W2);
  }
  if (edge2) {
    ld3(nrm, n1 + 3 * rj);
    for (int i = 0; i < 3; i++) ad[i] = -dl * nrm[i];
    return polygon_clip(w, f1, nf1, f2, nf2, nrm, ad, W1, W2);
  }
  for (int i = 0; i < 3; i++) ad[i] = dl * n2[3 * rj + i];
  ld3(nrm, n1 + 3 * ri);
  return polygon_clip(w, f1, nf1, f2, nf2, nrm, ad, W1, W2);
}

// box-box (the KAT kernel's name for it)
__device__ __forceinline__ int multicontact_box(const CcdWS& w, int fidx, const float* x1, const float* x2, const CGeom& g1, const CGeom& g2) {
  return multicontact(w, fidx, x1, x2, g1, g2);
}

// collision_gjk.py:2200-2345 ccd + collision_convex.py:763-852: contacts of one convex pair.
// Returns the contact count (0: not penetrating); *dist is corrected by +margin, `normal` is
// unnormalized (frame = make_frame(normal)), points in pts (stride 3, up to 4).
__device__ __forceinline__ void put_cgeom(float* dst, const float* pos, const float* rot, const float* size, int type, int vertadr = 0,
                                          int nvert = 0, int meshid = -1) {
  for (int i = 0; i < 3; i++) { dst[i] = pos[i]; dst[12 + i] = size[i]; }
  for (int i = 0; i < 9; i++) dst[3 + i] = rot[i];
  dst[15] = 0.0f;
  dst[16] = __int_as_float(type);
  dst[17] = __int_as_float(vertadr);
  dst[18] = __int_as_float(nvert);
  dst[19] = __int_as_float(meshid);
}

// lane `lane` (< CCD_OUT) of the record of a convex pair from the lockstep workspace's result
// (Wout: dist, normal[3], points[4][3]) and its contact count nc
__device__ __forceinline__ float ccd_record_word(int lane, int nc, const float* Wout) {
  if (lane == 0) return (float)nc;
  if (nc <= 0) return 0.0f;
  if (lane < 4) return Wout[lane];
  if (lane >= 20) return Wout[1 + (lane - 20) % 3];  // every point's normal = the pair's
  const int q = (lane - 4) >> 2, j = (lane - 4) & 3;
  return j == 0 ? Wout[0] : Wout[4 + 3 * q + j - 1];
}

__device__ __forceinline__ CGeom get_cgeom(const float* src, const float* mesh_vert, const MeshPoly* P = nullptr) {
  CGeom g;
  for (int i = 0; i < 3; i++) { g.pos[i] = src[i]; g.size[i] = src[12 + i]; }
  for (int i = 0; i < 9; i++) g.rot[i] = src[3 + i];
  g.margin = src[15];
  g.type = __float_as_int(src[16]);
  g.mv = mesh_vert ? mesh_vert + 3 * (long)__float_as_int(src[17]) : nullptr;
  g.nvert = mesh_vert ? __float_as_int(src[18]) : 0;
  g.prism = nullptr;
  g.pnormal = nullptr;
  g.pvadr = g.pvnum = g.pvert = g.pmapadr = g.pmapnum = g.pmap = nullptr;
  const int mid = __float_as_int(src[19]);
  if (P && g.type == GEOM_MESH && mid >= 0 && P->polynum[mid] > 0) {
    const int pa = P->polyadr[mid], va = P->vertadr[mid];
    g.pnormal = P->polynormal + 3 * pa;
    g.pvadr = P->polyvertadr + pa;
    g.pvnum = P->polyvertnum + pa;
    g.pvert = P->polyvert;
    g.pmapadr = P->polymapadr + va;
    g.pmapnum = P->polymapnum + va;
    g.pmap = P->polymap;
  }
  return g;
}

// the model's mesh polygon arrays
__device__ __forceinline__ MeshPoly mesh_poly(const mjw_model_t& m) {
  MeshPoly P;
  P.polynormal = m.mesh_polynormal;
  P.polyadr = m.mesh_polyadr; P.polynum = m.mesh_polynum; P.polyvertadr = m.mesh_polyvertadr; P.polyvertnum = m.mesh_polyvertnum;
  P.polyvert = m.mesh_polyvert; P.polymapadr = m.mesh_polymapadr; P.polymapnum = m.mesh_polymapnum; P.polymap = m.mesh_polymap;
  P.vertadr = m.mesh_vertadr;
  return P;
}

// collision_gjk.py:2200-2345 ccd: distance (or depth) of one convex pair and its first witness points.
// Returns the reference's ncon (1, or 0 when EPA fails); *idx = EPA face for box multi-contact or -1.
// g1 / g2 carry their margins on entry and leave with the sizes / margins the final GJK / EPA used
// (what multicontact_box needs); the polytope stays in the workspace.
__device__ __forceinline__ int ccd_raw(const CcdWS& w, int epa_it, float tolerance, int gjk_it, float cutoff, CGeom& g1, CGeom& g2, float* dist,
                                       float* x1, float* x2, int* idx) {
  *idx = -1;
  // collision_gjk.py:91-94 _discrete_geoms: boxes and meshes (polytopes)
  const int discrete = (g1.type == GEOM_BOX || g1.type == GEOM_MESH || g1.type == GEOM_HFIELD) &&
                       (g2.type == GEOM_BOX || g2.type == GEOM_MESH || g2.type == GEOM_HFIELD) && g1.margin == 0.0f && g2.margin == 0.0f;
  float full1 = 0.0f, full2 = 0.0f, size1 = 0.0f, size2 = 0.0f;
  if (g1.type == GEOM_SPHERE || g1.type == GEOM_CAPSULE) { size1 = g1.size[0]; full1 = size1 + 0.5f * g1.margin; g1.margin = 0.0f; g1.size[0] = 0.0f; }
  if (g2.type == GEOM_SPHERE || g2.type == GEOM_CAPSULE) { size2 = g2.size[0]; full2 = size2 + 0.5f * g2.margin; g2.margin = 0.0f; g2.size[0] = 0.0f; }
  GjkOut r;
  if (size1 + size2 > 0.0f) {
    cutoff += full1 + full2;
    r = gjk(w, tolerance, gjk_it, g1, g2, cutoff, discrete);
    if (r.dist > tolerance) {  // shallow: inflate (collision_gjk.py:194-213)
      if (r.dist == CCD_FLOAT_MAX) { *dist = r.dist; st3(x1, r.x1); st3(x2, r.x2); return 1; }
      if (g1.type == GEOM_HFIELD) {
        // collision_gjk.py:2160-2187: a simplex touching both the prism's top and bottom
        bool side = false;
        for (int i = 1; i < r.dim; i++) side |= w.sidx(0)[i] != w.sidx(0)[0];
        if (side) {
          float sp[3];
          int si;
          ccd_support(g2, r.x2, sp, &si);  // geom2 still shrunk to its point / segment
          st3(x2, sp);
          x2[2] -= full2;
          *dist = hfield_top_witness(g1, x2, x1);
          return 1;
        }
      }
      float n[3] = {r.x2[0] - r.x1[0], r.x2[1] - r.x1[1], r.x2[2] - r.x1[2]};
      normalize3(n);
      for (int i = 0; i < 3; i++) { x1[i] = r.x1[i] + (full1 > 0.0f ? full1 * n[i] : 0.0f); x2[i] = r.x2[i] - (full2 > 0.0f ? full2 * n[i] : 0.0f); }
      *dist = r.dist - (full1 + full2);
      return 1;
    }
    g1.margin = full1 - size1; g1.size[0] = size1;
    g2.margin = full2 - size2; g2.size[0] = size2;
    cutoff -= full1 + full2;
  }
  r = gjk(w, tolerance, gjk_it, g1, g2, cutoff, discrete);
  *dist = r.dist;
  st3(x1, r.x1);
  st3(x2, r.x2);
  if (r.dist > tolerance || r.dim < 2) return 1;
  int nvert = 0, nface = 0, status;
  if (r.dim == 2) {
    status = polytope2(w, &nvert, &nface, g1, g2);
    if (status == -1) status = polytope3(w, &nvert, &nface, r.dist, g1, g2);
  } else if (r.dim == 4) {
    status = polytope4(w, &nvert, &nface);
    if (status == -1) status = polytope3(w, &nvert, &nface, r.dist, g1, g2);
  } else {
    status = polytope3(w, &nvert, &nface, r.dist, g1, g2);
  }
  if (status) return 1;  // origin on the boundary: not penetrating
  const int f = epa(w, nvert, nface, tolerance, epa_it, g1, g2, discrete, dist, x1, x2);
  if (f == -1) {
    *dist = CCD_FLOAT_MAX;
    for (int i = 0; i < 3; i++) x1[i] = x2[i] = 0.0f;
    return 0;
  }
  // collision_gjk.py:2336-2345: multi-contact needs no margin and boxes or meshes (with polygon data,
  // collision_convex.py:810-818); the caller applies MULTICCD (box-box always, collision_convex.py:809)
  const bool bm1 = g1.type == GEOM_BOX || (g1.type == GEOM_MESH && g1.pnormal), bm2 = g2.type == GEOM_BOX || (g2.type == GEOM_MESH && g2.pnormal);
  *idx = (g1.margin != 0.0f || g2.margin != 0.0f || !bm1 || !bm2) ? -1 : f;
  return 1;
}

// collision_convex.py:763-852 (eval_ccd_write_contact): contacts of one convex pair.  The pair's geoms
// are read from the workspace (put_cgeom at L.geoms); the outputs are written to L.out: [0] dist
// (corrected by +margin), [1..3] normal (unnormalized; frame = make_frame(normal)), [4..15] up to 4
// points.  Returns the contact count (0: not penetrating).  Only scalars and the LDS base cross the
// call, so the CCD code does not touch the caller's register budget.
// cutoff > 0 (collision sensors, collision_convex.py:772-776): separated pairs are reported too
// P / multiccd / npoly / ndeg: the mesh polygon data, opt MULTICCD and the layout's multi-contact bounds
__device__ __forceinline__ int ccd_pair(float* W, int epa_it, float tolerance, int gjk_it, float margin, const float* mesh_vert = nullptr,
                                       float cutoff = 0.0f, const MeshPoly* P = nullptr, bool multiccd = false, int npoly = 4,
                                       int ndeg = 3) {
  CcdWS w;
  w.W = W;
  w.L = ccd_layout(epa_it, false, npoly, ndeg);
  CGeom g1 = get_cgeom(W + w.L.geoms, mesh_vert, P), g2 = get_cgeom(W + w.L.geoms + CGEOM_WORDS, mesh_vert, P);
  float* dist_out = W + w.L.out;
  float* normal = W + w.L.out + 1;
  float* pts = W + w.L.out + 4;
  g1.margin = margin;
  g2.margin = margin;
  float d, x1[3], x2[3];
  int idx;
  if (!ccd_raw(w, epa_it, tolerance, gjk_it, cutoff, g1, g2, &d, x1, x2, &idx)) return 0;
  if (d >= 0.0f && cutoff == 0.0f) return 0;
  *dist_out = d + margin;
  int n = 1;
  float* W1 = w.W + w.L.w1;
  float* W2 = w.W + w.L.w2;
  st3(W1, x1);
  st3(W2, x2);
  // collision_convex.py:809: box-box always, box-mesh / mesh-mesh under MULTICCD
  if (idx > -1 && (multiccd || (g1.type == GEOM_BOX && g2.type == GEOM_BOX))) n = multicontact(w, idx, x1, x2, g1, g2);
  for (int i = 0; i < n; i++)
    for (int k = 0; k < 3; k++) pts[3 * i + k] = 0.5f * (W1[3 * i + k] + W2[3 * i + k]);
  for (int k = 0; k < 3; k++) normal[k] = W1[k] - W2[k];
  return n;
}


// ---- heightfields (collision_convex.py:55-154 _hfield_filter, 158-697 ccd_hfield_kernel) ------------
// One heightfield-convex pair, the whole wave in lockstep: the filter, then GJK / EPA of geom2 against
// each triangular prism of the grid cells under geom2's bounding box (the heightfield frame; the prism
// holds the cell triangle raised by the margin and the base at -size[3]), every result cached, then up
// to four of them kept -- the deepest, the farthest from it, the farthest from their line, and the
// farthest from the triangle's other edges.  `rec` (LDS, CCD_OUT words) receives the record: every
// point with its own distance and normal.  Returns the number of points.
//   hpos / hmat: the heightfield geom's frame; hsize: hfield_size (x, y half-extents, top, base);
//   fmargin: geom_margin sum (the filter's); margin: the contact margin (contact_params).
__device__ __forceinline__ int hfield_pair(const CcdWS& w, int epa_it, float tolerance, int gjk_it, float fmargin, float margin,
                                           const float* hpos, const float* hmat, const float* hsize, int nrow, int ncol,
                                           const float* hdata, const float* gpos, const float* gmat, const float* gsize,
                                           float grbound, int t2, const float* mv, int nvert, float* rec) {
  rec[0] = 0.0f;
  float dp[3] = {gpos[0] - hpos[0], gpos[1] - hpos[1], gpos[2] - hpos[2]}, pos[3], rot[9];
  for (int i = 0; i < 3; i++) pos[i] = hmat[i] * dp[0] + hmat[3 + i] * dp[1] + hmat[6 + i] * dp[2];
  // box-sphere tests: horizontal, up, down
  for (int i = 0; i < 2; i++)
    if (hsize[i] < pos[i] - grbound - fmargin || -hsize[i] > pos[i] + grbound + fmargin) return 0;
  if (hsize[2] < pos[2] - grbound - fmargin) return 0;
  if (-hsize[3] > pos[2] + grbound + fmargin) return 0;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) rot[3 * i + j] = hmat[i] * gmat[j] + hmat[3 + i] * gmat[3 + j] + hmat[6 + i] * gmat[6 + j];
  CGeom g2;
  for (int i = 0; i < 3; i++) { g2.pos[i] = pos[i]; g2.size[i] = gsize[i]; }
  for (int i = 0; i < 9; i++) g2.rot[i] = rot[i];
  g2.margin = 0.0f;
  g2.type = t2;
  g2.mv = mv;
  g2.nvert = nvert;
  g2.prism = nullptr;
  // tight bounds from the support function (box-box test)
  float ext[6], sp[3];
  int si;
  for (int k = 0; k < 6; k++) {
    float dir[3] = {0.0f, 0.0f, 0.0f};
    dir[k >> 1] = (k & 1) ? -1.0f : 1.0f;
    ccd_support(g2, dir, sp, &si);
    ext[k] = sp[k >> 1];
  }
  const float xmax = ext[0], xmin = ext[1], ymax = ext[2], ymin = ext[3], zmax = ext[4], zmin = ext[5];
  if (xmin - fmargin > hsize[0] || xmax + fmargin < -hsize[0] || ymin - fmargin > hsize[1] || ymax + fmargin < -hsize[1] ||
      zmin - fmargin > hsize[2] || zmax + fmargin < -hsize[3])
    return 0;
  // the subgrid under geom2
  const float x_scale = 0.5f * (float)(ncol - 1) / hsize[0], y_scale = 0.5f * (float)(nrow - 1) / hsize[1];
  const int cmin = max(0, (int)floorf((xmin + hsize[0]) * x_scale));
  const int cmax = min(ncol - 1, (int)ceilf((xmax + hsize[0]) * x_scale));
  const int rmin = max(0, (int)floorf((ymin + hsize[1]) * y_scale));
  const int rmax = min(nrow - 1, (int)ceilf((ymax + hsize[1]) * y_scale));
  const float dx = (2.0f * hsize[0]) / (float)(ncol - 1), dy = (2.0f * hsize[1]) / (float)(nrow - 1);
  float* prism = w.W + w.L.hf;
  float* cd = prism + 18;               // per cached contact: dist
  float* cp = cd + HF_MAXCON;           // pos[3]
  float* cn = cp + 3 * HF_MAXCON;       // normal[3]
  for (int i = 0; i < 3; i++) prism[3 * i + 2] = -hsize[3];
  g2.margin = margin;
  CGeom g1;
  for (int i = 0; i < 9; i++) g1.rot[i] = (i % 4 == 0) ? 1.0f : 0.0f;
  g1.size[0] = g1.size[1] = g1.size[2] = 0.0f;
  g1.margin = 0.0f;
  g1.type = GEOM_HFIELD;
  g1.mv = nullptr;
  g1.nvert = 0;
  g1.prism = prism;
  auto push = [&](float x, float y, float z) {  // prism[0] = prism[1], prism[1] = prism[2], ...; new vertex 2 / 5
    for (int i = 0; i < 3; i++) {
      prism[i] = prism[3 + i]; prism[3 + i] = prism[6 + i];
      prism[9 + i] = prism[12 + i]; prism[12 + i] = prism[15 + i];
    }
    prism[6] = x; prism[15] = x;
    prism[7] = y; prism[16] = y;
    prism[17] = z;
  };
  int count = 0, min_id = -1;
  float min_dist = MJW_MAXVAL;
  for (int r = rmin; r < rmax; r++) {
    for (int i = 0; i < 2; i++)
      push(dx * (float)cmin - hsize[0], dy * (float)(r + i) - hsize[1], hdata[(r + i) * ncol + cmin] * hsize[2] + margin);
    for (int c = cmin + 1; c <= cmax; c++) {
      for (int i = 0; i < 2; i++) {
        if (count >= HF_MAXCON) continue;  // the reference reports the overflow and drops the prism
        push(dx * (float)c - hsize[0], dy * (float)(r + i) - hsize[1], hdata[(r + i) * ncol + c] * hsize[2] + margin);
        if (prism[11] < zmin && prism[14] < zmin && prism[17] < zmin) continue;  // prism height test
        for (int k = 0; k < 3; k++)
          g1.pos[k] = (prism[k] + prism[3 + k] + prism[6 + k] + prism[9 + k] + prism[12 + k] + prism[15 + k]) * (1.0f / 6.0f);
        CGeom a = g1, b = g2;
        float d, x1[3], x2[3];
        int idx;
        if (!ccd_raw(w, epa_it, tolerance, gjk_it, 0.0f, a, b, &d, x1, x2, &idx)) continue;
        float pl[3] = {0.5f * (x1[0] + x2[0]), 0.5f * (x1[1] + x2[1]), 0.5f * (x1[2] + x2[2])};
        float nl[3] = {x1[0] - x2[0], x1[1] - x2[1], x1[2] - x2[2]}, pg[3], ng[3];
        normalize3(nl);  // make_frame(w1 - w2)'s first row
        matvec3(pg, hmat, pl);
        matvec3(ng, hmat, nl);
        cd[count] = d;
        for (int k = 0; k < 3; k++) { cp[3 * count + k] = pg[k] + hpos[k]; cn[3 * count + k] = ng[k]; }
        if (d < min_dist) { min_dist = d; min_id = count; }
        count++;
      }
    }
  }
  // contact 0: the minimum distance
  float min_pos[3] = {MJW_MAXVAL, MJW_MAXVAL, MJW_MAXVAL}, min_nrm[3] = {MJW_MAXVAL, MJW_MAXVAL, MJW_MAXVAL};
  if (min_id >= 0)
    for (int k = 0; k < 3; k++) { min_pos[k] = cp[3 * min_id + k]; min_nrm[k] = cn[3 * min_id + k]; }
  auto put = [&](int q, float d, const float* p, const float* n) {
    rec[4 + 4 * q] = d;
    for (int k = 0; k < 3; k++) { rec[5 + 4 * q + k] = p[k]; rec[20 + 3 * q + k] = n[k]; }
  };
  put(0, min_dist, min_pos, min_nrm);
  for (int k = 0; k < 3; k++) rec[1 + k] = min_nrm[k];
  int n = 1;
  constexpr float MIN_DIST_TO_NEXT = 1.0e-3f;
  // contact 1: the farthest from contact 0
  int id1 = -1;
  float dist1 = -MJW_MAXVAL;
  for (int i = 0; i < count; i++) {
    if (i == min_id) continue;
    float t[3] = {cp[3 * i] - min_pos[0], cp[3 * i + 1] - min_pos[1], cp[3 * i + 2] - min_pos[2]};
    const float dd = sqrtf(dot3(t, t));
    if (dd > dist1) { id1 = i; dist1 = dd; }
  }
  if (!(id1 == -1 || (0.0f < dist1 && dist1 < MIN_DIST_TO_NEXT))) {
    const float* pos1 = cp + 3 * id1;
    put(n++, cd[id1], pos1, cn + 3 * id1);
    // contact 2: the farthest from the line through contacts 0 and 1
    float t[3] = {min_pos[0] - pos1[0], min_pos[1] - pos1[1], min_pos[2] - pos1[2]}, dmin1[3];
    cross3(dmin1, min_nrm, t);
    int id2 = -1;
    float dist12 = -MJW_MAXVAL;
    for (int i = 0; i < count; i++) {
      if (i == min_id || i == id1) continue;
      float u[3] = {cp[3 * i] - min_pos[0], cp[3 * i + 1] - min_pos[1], cp[3 * i + 2] - min_pos[2]};
      const float dd = fabsf(dot3(u, dmin1));
      if (dd > dist12) { id2 = i; dist12 = dd; }
    }
    if (!(id2 == -1 || (0.0f < dist12 && dist12 < MIN_DIST_TO_NEXT))) {
      const float* pos2 = cp + 3 * id2;
      put(n++, cd[id2], pos2, cn + 3 * id2);
      // contact 3: the farthest from the triangle's other two edges
      float a0[3] = {min_pos[0] - pos2[0], min_pos[1] - pos2[1], min_pos[2] - pos2[2]};
      float a1[3] = {pos1[0] - pos2[0], pos1[1] - pos2[1], pos1[2] - pos2[2]}, vmin2[3], v12[3];
      cross3(vmin2, min_nrm, a0);
      cross3(v12, min_nrm, a1);
      int id3 = -1;
      float dist3 = -MJW_MAXVAL;
      for (int i = 0; i < count; i++) {
        if (i == min_id || i == id1 || i == id2) continue;
        const float* pi = cp + 3 * i;
        float u[3] = {pi[0] - min_pos[0], pi[1] - min_pos[1], pi[2] - min_pos[2]};
        float v[3] = {pos1[0] - pi[0], pos1[1] - pi[1], pos1[2] - pi[2]};
        const float dd = fabsf(dot3(u, vmin2)) + fabsf(dot3(v, v12));
        if (dd > dist3) { id3 = i; dist3 = dd; }
      }
      if (!(id3 == -1 || (0.0f < dist3 && dist3 < MIN_DIST_TO_NEXT))) put(n++, cd[id3], cp + 3 * id3, cn + 3 * id3);
    }
  }
  rec[0] = (float)n;
  for (int q = n; q < 4; q++) put(q, 0.0f, min_pos, min_nrm);
  return n;
}

}  // namespace mjw
