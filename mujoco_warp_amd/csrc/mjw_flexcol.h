// mjw_flexcol.h -- triangle narrowphase of flex collision (collision_primitive_core.py:1495-1990):
// sphere / capsule / box / cylinder against one flex triangle, up to 2 candidate contacts each.
// Used by the sparse path's collision pass (mjw_sparse.hip) and by the known-answer kernel
// (mjw_kat.hip) that replays the reference's collision_primitive_core_test.py cases.
#pragma once

#include "mjw_common.h"

namespace mjw {
namespace sp {

struct Cand {
  float dist;
  float pos[3];
  float nrm[3];
};

// collision_primitive_core.py:1495-1597
__device__ __forceinline__ float tri_sign(const float* p1, const float* p2, const float* p3) {
  const float a = (p1[0] - p3[0]) * (p2[1] - p3[1]) - (p2[0] - p3[0]) * (p1[1] - p3[1]);
  return (float)((a > 0.0f) - (a < 0.0f));
}

__device__ __forceinline__ void tri_seg(float* r, const float* p, const float* u, const float* v) {
  const float uv[2] = {v[0] - u[0], v[1] - u[1]}, up[2] = {p[0] - u[0], p[1] - u[1]};
  const float a = (uv[0] * up[0] + uv[1] * up[1]) / fmaxf(MJW_MINVAL, uv[0] * uv[0] + uv[1] * uv[1]);
  if (a <= 0.0f) { r[0] = u[0]; r[1] = u[1]; }
  else if (a >= 1.0f) { r[0] = v[0]; r[1] = v[1]; }
  else { r[0] = u[0] + a * uv[0]; r[1] = u[1] + a * uv[1]; }
}

__device__ __forceinline__ float sphere_triangle(float* pos, float* nrm, const float* sp, float sr, const float* t1, const float* t2, const float* t3,
                                 float tr) {
  float S[3], A[3], B[3], N[3], P[3], V1[3], V2[3], X[3];
  for (int i = 0; i < 3; i++) { S[i] = sp[i] - t1[i]; A[i] = t2[i] - t1[i]; B[i] = t3[i] - t1[i]; }
  cross3(N, A, B);
  normalize3(N);
  const float dstS = dot3(N, S);
  for (int i = 0; i < 3; i++) P[i] = S[i] - dstS * N[i];
  const float lenA = sqrtf(dot3(A, A));
  for (int i = 0; i < 3; i++) V1[i] = A[i];
  normalize3(V1);
  cross3(V2, N, A);
  normalize3(V2);
  const float o[2] = {0.0f, 0.0f}, a[2] = {lenA, 0.0f}, b[2] = {dot3(V1, B), dot3(V2, B)}, p[2] = {dot3(V1, P), dot3(V2, P)};
  const float s1 = tri_sign(p, o, a), s2 = tri_sign(p, a, b), s3 = tri_sign(p, b, o);
  if (s1 == s2 && s2 == s3) {
    for (int i = 0; i < 3; i++) X[i] = P[i];
  } else {
    float x0[2], x1[2], x2[2];
    tri_seg(x0, p, o, a);
    tri_seg(x1, p, a, b);
    tri_seg(x2, p, b, o);
    const float d0 = hypotf(p[0] - x0[0], p[1] - x0[1]), d1 = hypotf(p[0] - x1[0], p[1] - x1[1]), d2 = hypotf(p[0] - x2[0], p[1] - x2[1]);
    const float* xs = (d0 < d1 && d0 < d2) ? x0 : (d1 < d2 ? x1 : x2);
    for (int i = 0; i < 3; i++) X[i] = xs[0] * V1[i] + xs[1] * V2[i];
  }
  for (int i = 0; i < 3; i++) nrm[i] = X[i] - S[i];
  const float dst = sqrtf(dot3(nrm, nrm));
  if (dst > MJW_MINVAL) for (int i = 0; i < 3; i++) nrm[i] /= dst;
  else for (int i = 0; i < 3; i++) nrm[i] = N[i];
  const float dist = dst - sr - tr;
  for (int i = 0; i < 3; i++) pos[i] = sp[i] + nrm[i] * (sr + 0.5f * dist);
  return dist;
}

// triangle vs sphere/capsule/box/cylinder: up to 2 candidates (collision_primitive_core.py:1600-1990)
__device__ __forceinline__ int geom_triangle(Cand* c, int gt, const float* gp, const float* gr, const float* gs, const float* const* t, float tr) {
  int n = 0;
  const float ax[3] = {gr[2], gr[5], gr[8]};
  if (gt == GEOM_SPHERE) {
    c[0].dist = sphere_triangle(c[0].pos, c[0].nrm, gp, gs[0], t[0], t[1], t[2], tr);
    return 1;
  }
  if (gt == GEOM_CAPSULE) {
    float p1[3], p2[3], ab[3];
    for (int i = 0; i < 3; i++) { p1[i] = gp[i] - ax[i] * gs[1]; p2[i] = gp[i] + ax[i] * gs[1]; ab[i] = p2[i] - p1[i]; }
    c[n].dist = sphere_triangle(c[n].pos, c[n].nrm, p1, gs[0], t[0], t[1], t[2], tr);
    if (c[n].dist < MJW_MAXVAL) n++;
    c[n].dist = sphere_triangle(c[n].pos, c[n].nrm, p2, gs[0], t[0], t[1], t[2], tr);
    if (c[n].dist < MJW_MAXVAL) n++;
    const float ab2 = 4.0f * gs[1] * gs[1];
    for (int vi = 0; vi < 3 && n < 2; vi++) {
      float vec[3], cl[3], df[3];
      for (int i = 0; i < 3; i++) vec[i] = t[vi][i] - p1[i];
      const float tp = dot3(vec, ab) / fmaxf(MJW_MINVAL, ab2);
      if (tp > MJW_MINVAL && tp < 1.0f - MJW_MINVAL) {
        for (int i = 0; i < 3; i++) { cl[i] = p1[i] + ab[i] * tp; df[i] = t[vi][i] - cl[i]; }
        const float draw = sqrtf(dot3(df, df));
        if (draw > MJW_MINVAL) {
          for (int i = 0; i < 3; i++) {
            c[n].nrm[i] = df[i] / draw;
            c[n].pos[i] = (cl[i] + t[vi][i] + c[n].nrm[i] * (gs[0] - tr)) * 0.5f;
          }
          c[n].dist = draw - gs[0] - tr;
          n++;
        }
      }
    }
    return n;
  }
  if (gt == GEOM_BOX) {
    for (int vi = 0; vi < 3; vi++) {
      float df[3], loc[3];
      for (int i = 0; i < 3; i++) df[i] = t[vi][i] - gp[i];
      for (int i = 0; i < 3; i++) loc[i] = gr[i] * df[0] + gr[3 + i] * df[1] + gr[6 + i] * df[2];
      int maxaxis = 0;
      float maxval = fabsf(loc[0]) - gs[0];
      for (int j = 1; j < 3; j++) {
        const float v = fabsf(loc[j]) - gs[j];
        if (v > maxval) { maxval = v; maxaxis = j; }
      }
      bool inside = true;
      for (int j = 0; j < 3; j++) if (fabsf(loc[j]) > gs[j] + tr) inside = false;
      if (inside && n < 2) {
        float nl[3] = {0.0f, 0.0f, 0.0f};
        nl[maxaxis] = (float)((loc[maxaxis] > 0.0f) - (loc[maxaxis] < 0.0f));
        matvec3(c[n].nrm, gr, nl);
        const float dd = maxval - tr, off = tr + dd * 0.5f;
        for (int i = 0; i < 3; i++) c[n].pos[i] = t[vi][i] - c[n].nrm[i] * off;
        c[n].dist = dd;
        n++;
      }
    }
    for (int i = 0; i < 8 && n < 2; i++) {
      float vec[3] = {(i & 1) ? gs[0] : -gs[0], (i & 2) ? gs[1] : -gs[1], (i & 4) ? gs[2] : -gs[2]}, corner[3];
      matvec3(corner, gr, vec);
      for (int k = 0; k < 3; k++) corner[k] += gp[k];
      c[n].dist = sphere_triangle(c[n].pos, c[n].nrm, corner, 0.0f, t[0], t[1], t[2], tr);
      if (c[n].dist < MJW_MAXVAL) n++;
    }
    return n;
  }
  // cylinder
  const float cr = gs[0], hh = gs[1];
  float p1[3], p2[3], ab[3];
  for (int i = 0; i < 3; i++) { p1[i] = gp[i] - ax[i] * hh; p2[i] = gp[i] + ax[i] * hh; ab[i] = p2[i] - p1[i]; }
  const float ab2 = 4.0f * hh * hh;
  for (int vi = 0; vi < 3 && n < 2; vi++) {
    const float* vert = t[vi];
    float vec[3];
    for (int i = 0; i < 3; i++) vec[i] = vert[i] - p1[i];
    const float tp = dot3(vec, ab) / fmaxf(MJW_MINVAL, ab2);
    if (tp > MJW_MINVAL && tp < 1.0f - MJW_MINVAL) {
      float cl[3], df[3];
      for (int i = 0; i < 3; i++) { cl[i] = p1[i] + ab[i] * tp; df[i] = vert[i] - cl[i]; }
      const float draw = sqrtf(dot3(df, df));
      if (draw < cr + tr) {
        if (draw > MJW_MINVAL) {
          for (int i = 0; i < 3; i++) { c[n].nrm[i] = df[i] / draw; c[n].pos[i] = (cl[i] + vert[i] + c[n].nrm[i] * (cr - tr)) * 0.5f; }
          c[n].dist = draw - cr - tr;
        } else {
          const float L = sqrtf(ab2), d2 = (1.0f - tp) * L, d1 = tp * L;
          if (d2 < cr && d2 < d1) {
            for (int i = 0; i < 3; i++) { c[n].nrm[i] = ax[i]; c[n].pos[i] = vert[i]; }
            c[n].dist = -d2 - tr;
          } else if (d1 < cr) {
            for (int i = 0; i < 3; i++) { c[n].nrm[i] = -ax[i]; c[n].pos[i] = vert[i]; }
            c[n].dist = -d1 - tr;
          } else {
            float e1[3], e2[3];
            for (int i = 0; i < 3; i++) { e1[i] = t[1][i] - t[0][i]; e2[i] = t[2][i] - t[0][i]; }
            cross3(c[n].nrm, e1, e2);
            normalize3(c[n].nrm);
            for (int i = 0; i < 3; i++) c[n].pos[i] = cl[i];
            c[n].dist = -cr - tr;
          }
        }
        n++;
      }
    } else {
      const float* pe = tp <= MJW_MINVAL ? p1 : p2;
      const float sg = tp <= MJW_MINVAL ? -1.0f : 1.0f;
      float df[3], perp[3];
      for (int i = 0; i < 3; i++) df[i] = vert[i] - pe[i];
      const float sd = dot3(df, ax);
      for (int i = 0; i < 3; i++) perp[i] = df[i] - ax[i] * sd;
      const float pl = sqrtf(dot3(perp, perp));
      if (pl < cr) {
        const float dd = sg * sd - tr;
        for (int i = 0; i < 3; i++) { c[n].nrm[i] = sg * ax[i]; c[n].pos[i] = vert[i] - c[n].nrm[i] * (tr + dd * 0.5f); }
        c[n].dist = dd;
        n++;
      } else if (pl < cr + tr) {
        float ep[3], de[3];
        for (int i = 0; i < 3; i++) { ep[i] = pe[i] + perp[i] / pl * cr; de[i] = vert[i] - ep[i]; }
        const float draw = sqrtf(dot3(de, de));
        if (draw > MJW_MINVAL) {
          const float dd = draw - tr;
          for (int i = 0; i < 3; i++) { c[n].nrm[i] = de[i] / draw; c[n].pos[i] = vert[i] - c[n].nrm[i] * (tr + dd * 0.5f); }
          c[n].dist = dd;
          n++;
        }
      }
    }
  }
  return n;
}

}  // namespace sp
}  // namespace mjw
