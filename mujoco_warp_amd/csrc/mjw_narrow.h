// mjw_narrow.h -- pure contact geometry shared by the world-per-wave kernel (mjw_step.hip) and the
// workgroup-per-world sparse/flex kernels (mjw_sparse.hip): primitive narrowphase functions
// (collision_primitive_core.py), the AABB / OBB broadphase filters (collision_driver.py) and the
// geom contact-parameter mixing (collision_core.py).
#pragma once

#include "mjw_common.h"

namespace mjw {


// -------------------------------------------------------------------------------------------
// collision (collision_driver.py / collision_core.py / collision_primitive_core.py)
// -------------------------------------------------------------------------------------------
struct Con2 {
  float dist[2];
  float pos[2][3];
  float frame[2][9];
  int n;
};

// collision_primitive_core.py:106-111
__device__ __forceinline__ float plane_sphere(float* pos, const float* n, const float* ppos, const float* spos, float r) {
  float dif[3] = {spos[0] - ppos[0], spos[1] - ppos[1], spos[2] - ppos[2]};
  float dist = dot3(dif, n) - r;
  for (int i = 0; i < 3; i++) pos[i] = spos[i] - n[i] * (r + 0.5f * dist);
  return dist;
}

// collision_primitive_core.py:114-143
__device__ __forceinline__ float sphere_sphere(float* pos, float* n, const float* p1, float r1, const float* p2, float r2) {
  float dir[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  float dist = sqrtf(dot3(dir, dir));
  if (dist == 0.0f) { n[0] = 1.0f; n[1] = 0.0f; n[2] = 0.0f; }
  else { n[0] = dir[0] / dist; n[1] = dir[1] / dist; n[2] = dir[2] / dist; }
  dist = dist - (r1 + r2);
  for (int i = 0; i < 3; i++) pos[i] = p1[i] + n[i] * (r1 + 0.5f * dist);
  return dist;
}

// math.py:268-273
__device__ __forceinline__ void closest_segment_point(float* r, const float* a, const float* b, const float* pt) {
  float ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, pa[3] = {pt[0] - a[0], pt[1] - a[1], pt[2] - a[2]};
  float t = dot3(pa, ab) / (dot3(ab, ab) + 1e-6f);
  t = clampf(t, 0.0f, 1.0f);
  for (int i = 0; i < 3; i++) r[i] = a[i] + t * ab[i];
}

// collision_primitive_core.py:181-308
__device__ __forceinline__ void capsule_capsule(Con2& out, const float* p1, const float* ax1, float r1, float hl1, const float* p2,
                                const float* ax2, float r2, float hl2, float margin) {
  float a1[3], a2[3], dif[3];
  for (int i = 0; i < 3; i++) { a1[i] = ax1[i] * hl1; a2[i] = ax2[i] * hl2; dif[i] = p1[i] - p2[i]; }
  float ma = dot3(a1, a1), mb = -dot3(a1, a2), mc = dot3(a2, a2);
  float u = -dot3(a1, dif), v = dot3(a2, dif);
  float det = ma * mc - mb * mb;
  out.n = 0;
  float v1[3], v2[3], pos[3], nrm[3];
  if (fabsf(det) >= MJW_MINVAL) {
    float inv = 1.0f / det;
    float x1 = (mc * u - mb * v) * inv, x2 = (ma * v - mb * u) * inv;
    if (x1 > 1.0f) { x1 = 1.0f; x2 = (v - mb) / mc; }
    else if (x1 < -1.0f) { x1 = -1.0f; x2 = (v + mb) / mc; }
    if (x2 > 1.0f) { x2 = 1.0f; x1 = clampf((u - mb) / ma, -1.0f, 1.0f); }
    else if (x2 < -1.0f) { x2 = -1.0f; x1 = clampf((u + mb) / ma, -1.0f, 1.0f); }
    for (int i = 0; i < 3; i++) { v1[i] = p1[i] + a1[i] * x1; v2[i] = p2[i] + a2[i] * x2; }
    float dist = sphere_sphere(pos, nrm, v1, r1, v2, r2);
    if (dist <= margin) {
      out.dist[0] = dist;
      for (int i = 0; i < 3; i++) out.pos[0][i] = pos[i];
      make_frame(out.frame[0], nrm);
      out.n = 1;
    }
    return;
  }
  int cnt = 0;
#pragma unroll
  for (int t = 0; t < 4; t++) {
    if (t >= 2 && cnt >= 2) break;
    float x;
    if (t == 0) { x = clampf((v - mb) / mc, -1.0f, 1.0f); for (int i = 0; i < 3; i++) { v1[i] = p1[i] + a1[i]; v2[i] = p2[i] + a2[i] * x; } }
    else if (t == 1) { x = clampf((v + mb) / mc, -1.0f, 1.0f); for (int i = 0; i < 3; i++) { v1[i] = p1[i] - a1[i]; v2[i] = p2[i] + a2[i] * x; } }
    else if (t == 2) { x = clampf((u - mb) / ma, -1.0f, 1.0f); for (int i = 0; i < 3; i++) { v2[i] = p2[i] + a2[i]; v1[i] = p1[i] + a1[i] * x; } }
    else { x = clampf((u + mb) / ma, -1.0f, 1.0f); for (int i = 0; i < 3; i++) { v2[i] = p2[i] - a2[i]; v1[i] = p1[i] + a1[i] * x; } }
    float dist = sphere_sphere(pos, nrm, v1, r1, v2, r2);
    if (dist <= margin) {
      // slot index kept compile-time (no scratch): slot 0 first, then slot 1
      if (cnt == 0) {
        out.dist[0] = dist;
        for (int i = 0; i < 3; i++) out.pos[0][i] = pos[i];
        make_frame(out.frame[0], nrm);
      } else {
        out.dist[1] = dist;
        for (int i = 0; i < 3; i++) out.pos[1][i] = pos[i];
        make_frame(out.frame[1], nrm);
      }
      cnt++;
    }
  }
  out.n = cnt;
}

// collision_primitive_core.py:311-361
__device__ __forceinline__ void plane_capsule(Con2& out, const float* n, const float* ppos, const float* cpos, const float* axis, float r, float hl) {
  float nd = dot3(n, axis);
  float tmp[3] = {axis[0] - n[0] * nd, axis[1] - n[1] * nd, axis[2] - n[2] * nd};
  float bn = sqrtf(dot3(tmp, tmp));
  float b[3];
  if (bn == 0.0f) { b[0] = tmp[0]; b[1] = tmp[1]; b[2] = tmp[2]; }
  else { b[0] = tmp[0] / bn; b[1] = tmp[1] / bn; b[2] = tmp[2] / bn; }
  if (bn < 0.5f) {
    if (-0.5f < n[1] && n[1] < 0.5f) { b[0] = 0.0f; b[1] = 1.0f; b[2] = 0.0f; }
    else { b[0] = 0.0f; b[1] = 0.0f; b[2] = 1.0f; }
  }
  float c[3];
  cross3(c, n, b);
  float e1[3], e2[3];
  for (int i = 0; i < 3; i++) { e1[i] = cpos[i] + axis[i] * hl; e2[i] = cpos[i] - axis[i] * hl; }
  out.dist[0] = plane_sphere(out.pos[0], n, ppos, e1, r);
  out.dist[1] = plane_sphere(out.pos[1], n, ppos, e2, r);
  for (int k = 0; k < 2; k++) {
    out.frame[k][0] = n[0]; out.frame[k][1] = n[1]; out.frame[k][2] = n[2];
    out.frame[k][3] = b[0]; out.frame[k][4] = b[1]; out.frame[k][5] = b[2];
    out.frame[k][6] = c[0]; out.frame[k][7] = c[1]; out.frame[k][8] = c[2];
  }
  out.n = 2;
}

// collision_primitive_core.py:395-443: corner k (bit i of k selects +/- size[i]) against the plane
__device__ __forceinline__ float plane_box_corner(int k, const float* n, const float* ppos, const float* bpos, const float* bmat,
                                                  const float* bsize, float* pos) {
  float dif[3] = {bpos[0] - ppos[0], bpos[1] - ppos[1], bpos[2] - ppos[2]};
  float center_dist = dot3(dif, n);
  float cl[3] = {(k & 1) ? bsize[0] : -bsize[0], (k & 2) ? bsize[1] : -bsize[1], (k & 4) ? bsize[2] : -bsize[2]};
  float corner[3];
  matvec3(corner, bmat, cl);
  float cdist = center_dist + dot3(n, corner);
  for (int i = 0; i < 3; i++) pos[i] = corner[i] + bpos[i] - 0.5f * n[i] * cdist;
  return cdist;
}

// a[i] for a runtime i in 0..2 without dynamic register indexing (keeps the arrays in VGPRs)
__device__ __forceinline__ float sel3(const float* a, int i) { return i == 0 ? a[0] : (i == 1 ? a[1] : a[2]); }

__device__ __forceinline__ void mat_t_vec3(float* r, const float* M, const float* v) {
  for (int i = 0; i < 3; i++) r[i] = M[i] * v[0] + M[3 + i] * v[1] + M[6 + i] * v[2];
}

// collision_primitive_core.py:1103-1155
__device__ __forceinline__ float sphere_box(float* pos, float* nrm, const float* spos, float r, const float* bpos, const float* brot,
                            const float* bsize) {
  float dif[3] = {spos[0] - bpos[0], spos[1] - bpos[1], spos[2] - bpos[2]}, center[3], clamped[3], tmp[3];
  mat_t_vec3(center, brot, dif);
  for (int i = 0; i < 3; i++) { clamped[i] = fmaxf(-bsize[i], fminf(bsize[i], center[i])); tmp[i] = clamped[i] - center[i]; }
  float dist = sqrtf(dot3(tmp, tmp));
  float cdir[3] = {tmp[0], tmp[1], tmp[2]};
  if (dist != 0.0f) for (int i = 0; i < 3; i++) cdir[i] = tmp[i] / dist;
  float lp[3], dst;
  if (dist <= MJW_MINVAL) {
    float closest = 2.0f * (bsize[0] + bsize[1] + bsize[2]);
    int k = 0;
    for (int i = 0; i < 6; i++) {
      float fd = fabsf(((i & 1) ? 1.0f : -1.0f) * bsize[i >> 1] - center[i >> 1]);
      if (closest > fd) { closest = fd; k = i; }
    }
    const float sgn = (k & 1) ? -1.0f : 1.0f;
    float nearest[3] = {(k >> 1) == 0 ? sgn : 0.0f, (k >> 1) == 1 ? sgn : 0.0f, (k >> 1) == 2 ? sgn : 0.0f};
    for (int i = 0; i < 3; i++) lp[i] = center[i] + nearest[i] * (r - closest) / 2.0f;
    matvec3(nrm, brot, nearest);
    dst = -closest - r;
  } else {
    for (int i = 0; i < 3; i++) lp[i] = 0.5f * (clamped[i] + (center[i] + cdir[i] * r));
    matvec3(nrm, brot, cdir);
    dst = dist - r;
  }
  float w3[3];
  matvec3(w3, brot, lp);
  for (int i = 0; i < 3; i++) pos[i] = bpos[i] + w3[i];
  return dst;
}

// collision_primitive_core.py:1158-1480 (MuJoCo's capsule-box): up to 2 contacts
__device__ __forceinline__ void capsule_box(Con2& out, const float* cpos, const float* cax, float cr, float chl, const float* bpos, const float* brot,
                            const float* bsize) {
  float dif[3] = {cpos[0] - bpos[0], cpos[1] - bpos[1], cpos[2] - bpos[2]}, pos[3], axis[3], ha[3];
  mat_t_vec3(pos, brot, dif);
  mat_t_vec3(axis, brot, cax);
  for (int i = 0; i < 3; i++) ha[i] = axis[i] * chl;
  const int axisdir = (ha[0] > 0.0f) + 2 * (ha[1] > 0.0f) + 4 * (ha[2] > 0.0f);
  float bestdist = 1.0e32f, bestsegmentpos = -12.0f;
  int cltype = -4, clface = -12;
  // faces closest to one capsule end
  for (int i = -1; i < 2; i += 2) {
    float tip[3], bp[3];
    for (int k = 0; k < 3; k++) { tip[k] = pos[k] + (float)i * ha[k]; bp[k] = tip[k]; }
    int n_out = 0, ax_out = -1;
    for (int j = 0; j < 3; j++) {
      if (bp[j] < -bsize[j]) { n_out++; ax_out = j; bp[j] = -bsize[j]; }
      else if (bp[j] > bsize[j]) { n_out++; ax_out = j; bp[j] = bsize[j]; }
    }
    if (n_out > 1) continue;
    float dd[3] = {bp[0] - tip[0], bp[1] - tip[1], bp[2] - tip[2]};
    float dist = dot3(dd, dd);
    if (dist < bestdist) { bestdist = dist; bestsegmentpos = (float)i; cltype = -2 + i; clface = ax_out; }
  }
  // box edges
  int clcorner = -123, cledge = -123;
  float bestboxpos = 0.0f;
  for (int i = 0; i < 8; i++) {
    for (int j = 0; j < 3; j++) {
      if (i & (1 << j)) continue;
      float bpt[3] = {(i & 1) ? bsize[0] : -bsize[0], (i & 2) ? bsize[1] : -bsize[1], (i & 4) ? bsize[2] : -bsize[2]};
      bpt[j] = 0.0f;
      float df[3] = {bpt[0] - pos[0], bpt[1] - pos[1], bpt[2] - pos[2]};
      float u = -bsize[j] * df[j], v = dot3(ha, df);
      float ma = bsize[j] * bsize[j], mb = -bsize[j] * ha[j], mc = chl * chl;
      float det = ma * mc - mb * mb;
      if (fabsf(det) < MJW_MINVAL) continue;
      float idet = 1.0f / det;
      float x1 = (mc * u - mb * v) * idet, x2 = (ma * v - mb * u) * idet;
      int s1 = 1, s2 = 1;
      if (x1 > 1.0f) { x1 = 1.0f; s1 = 2; x2 = safe_div(v - mb, mc); }
      else if (x1 < -1.0f) { x1 = -1.0f; s1 = 0; x2 = safe_div(v + mb, mc); }
      const bool x2_over = x2 > 1.0f;
      if (x2_over || x2 < -1.0f) {
        if (x2_over) { x2 = 1.0f; s2 = 2; x1 = safe_div(u - mb, ma); }
        else { x2 = -1.0f; s2 = 0; x1 = safe_div(u + mb, ma); }
        if (x1 > 1.0f) { x1 = 1.0f; s1 = 2; }
        else if (x1 < -1.0f) { x1 = -1.0f; s1 = 0; }
      }
      for (int k = 0; k < 3; k++) df[k] -= ha[k] * x2;
      df[j] += bsize[j] * x1;
      const int ct = s1 * 3 + s2;
      float dsq = dot3(df, df);
      if (dsq < bestdist - MJW_MINVAL) {
        bestdist = dsq; bestsegmentpos = x2; bestboxpos = x1;
        clcorner = i + (1 << j) * (ct / 6);
        cledge = j;
        cltype = ct;
      }
    }
  }
  out.n = 0;
  if (cltype == -4) return;
  float secondpos = -4.0f;
  int c1;
  if (cltype >= 0 && cltype / 3 != 1) {  // closest to a box corner
    c1 = axisdir ^ clcorner;
    if (c1 != 0 && c1 != 7) {
      int mul, ax = 0, ax1 = 0, ax2 = 0;
      if (c1 == 1 || c1 == 2 || c1 == 4) mul = 1;
      else { mul = -1; c1 = 7 - c1; }
      if (c1 == 1) { ax = 0; ax1 = 1; ax2 = 2; }
      else if (c1 == 2) { ax = 1; ax1 = 2; ax2 = 0; }
      else if (c1 == 4) { ax = 2; ax1 = 0; ax2 = 1; }
      if (sel3(axis, ax) * sel3(axis, ax) > 0.5f) {
        float mm = 2.0f * safe_div(sel3(bsize, ax), fabsf(sel3(ha, ax)));
        secondpos = fminf(1.0f - (float)mul * bestsegmentpos, mm);
      } else {
        float mm = 2.0f * fminf(safe_div(sel3(bsize, ax1), fabsf(sel3(ha, ax1))), safe_div(sel3(bsize, ax2), fabsf(sel3(ha, ax2))));
        secondpos = -fminf(1.0f + (float)mul * bestsegmentpos, mm);
      }
      secondpos *= (float)mul;
    }
  } else if (cltype >= 0 && cltype / 3 == 1) {  // on a box edge
    c1 = axisdir ^ clcorner;
    c1 &= 7 - (1 << cledge);
    if (c1 == 1 || c1 == 2 || c1 == 4) {
      int ax1 = 0, ax2 = 0, ax = cledge, mul;
      if (cledge == 0) { ax1 = 1; ax2 = 2; }
      if (cledge == 1) { ax1 = 2; ax2 = 0; }
      if (cledge == 2) { ax1 = 0; ax2 = 1; }
      if (fabsf(sel3(axis, ax1)) > fabsf(sel3(axis, ax2))) ax1 = ax2;
      ax2 = 3 - ax - ax1;
      if (c1 & (1 << ax2)) { mul = 1; secondpos = 1.0f - bestsegmentpos; }
      else { mul = -1; secondpos = 1.0f + bestsegmentpos; }
      float e1 = 2.0f * safe_div(sel3(bsize, ax2), fabsf(sel3(ha, ax2)));
      secondpos = fminf(e1, secondpos);
      float e2 = (((axisdir & (1 << ax)) != 0) == ((c1 & (1 << ax2)) != 0)) ? 1.0f - bestboxpos : 1.0f + bestboxpos;
      e1 = sel3(bsize, ax) * safe_div(e2, fabsf(sel3(ha, ax)));
      secondpos = fminf(e1, secondpos);
      secondpos *= (float)mul;
    }
  } else if (clface != -1) {  // a capsule end closest to a face
    const int mul = cltype == -3 ? 1 : -1;
    secondpos = 2.0f;
    float tmp1[3] = {pos[0] - ha[0] * mul, pos[1] - ha[1] * mul, pos[2] - ha[2] * mul};
    for (int i = 0; i < 3; i++) {
      if (i == clface) continue;
      float ha_r = safe_div((float)mul, ha[i]);
      float e1 = (bsize[i] - tmp1[i]) * ha_r;
      if (0.0f < e1 && e1 < secondpos) secondpos = e1;
      e1 = (-bsize[i] - tmp1[i]) * ha_r;
      if (0.0f < e1 && e1 < secondpos) secondpos = e1;
    }
    secondpos *= (float)mul;
  }
  float l[3], g[3], nrm[3];
  for (int i = 0; i < 3; i++) l[i] = pos[i] + ha[i] * bestsegmentpos;
  matvec3(g, brot, l);
  for (int i = 0; i < 3; i++) g[i] += bpos[i];
  out.dist[0] = sphere_box(out.pos[0], nrm, g, cr, bpos, brot, bsize);
  make_frame(out.frame[0], nrm);
  out.n = 1;
  if (secondpos > -3.0f) {
    for (int i = 0; i < 3; i++) l[i] = pos[i] + ha[i] * (secondpos + bestsegmentpos);
    matvec3(g, brot, l);
    for (int i = 0; i < 3; i++) g[i] += bpos[i];
    out.dist[1] = sphere_box(out.pos[1], nrm, g, cr, bpos, brot, bsize);
    make_frame(out.frame[1], nrm);
    out.n = 2;
  }
}

// collision_driver.py:217-271
__device__ __forceinline__ bool obb_filter(const float* c1, const float* c2, const float* s1, const float* s2, float margin, const float* xp1,
                           const float* xp2, const float* xm1, const float* xm2) {
  float xc0[3], xc1[3];
  matvec3(xc0, xm1, c1);
  matvec3(xc1, xm2, c2);
  for (int i = 0; i < 3; i++) { xc0[i] += xp1[i]; xc1[i] += xp2[i]; }
  for (int j = 0; j < 2; j++) {
    const float* xmj = j == 0 ? xm1 : xm2;
    for (int k = 0; k < 3; k++) {
      float nk[3] = {xmj[k], xmj[3 + k], xmj[6 + k]};
      float proj0 = dot3(xc0, nk), proj1 = dot3(xc1, nk);
      float rad[2];
      for (int i = 0; i < 2; i++) {
        const float* xmi = i == 0 ? xm1 : xm2;
        const float* size = i == 0 ? s1 : s2;
        float n0[3] = {xmi[0], xmi[3], xmi[6]}, n1[3] = {xmi[1], xmi[4], xmi[7]}, n2[3] = {xmi[2], xmi[5], xmi[8]};
        rad[i] = fabsf(size[0] * dot3(n0, nk)) + fabsf(size[1] * dot3(n1, nk)) + fabsf(size[2] * dot3(n2, nk));
      }
      if (rad[0] + rad[1] + margin < fabsf(proj1 - proj0)) return false;
    }
  }
  return true;
}

// collision_driver.py:116-213
__device__ __forceinline__ bool aabb_filter(const float* c1, const float* c2, const float* s1, const float* s2, float margin, const float* xp1,
                            const float* xp2, const float* xm1, const float* xm2) {
  float cen1[3], cen2[3];
  matvec3(cen1, xm1, c1);
  matvec3(cen2, xm2, c2);
  for (int i = 0; i < 3; i++) { cen1[i] += xp1[i]; cen2[i] += xp2[i]; }
  float mx1[3] = {-MJW_MAXVAL, -MJW_MAXVAL, -MJW_MAXVAL}, mn1[3] = {MJW_MAXVAL, MJW_MAXVAL, MJW_MAXVAL};
  float mx2[3] = {-MJW_MAXVAL, -MJW_MAXVAL, -MJW_MAXVAL}, mn2[3] = {MJW_MAXVAL, MJW_MAXVAL, MJW_MAXVAL};
  for (int c = 0; c < 8; c++) {
    float sg0 = (c & 4) ? 1.0f : -1.0f, sg1 = (c & 2) ? 1.0f : -1.0f, sg2 = (c & 1) ? 1.0f : -1.0f;
    float cr1[3] = {sg0 * s1[0], sg1 * s1[1], sg2 * s1[2]}, cr2[3] = {sg0 * s2[0], sg1 * s2[1], sg2 * s2[2]}, p1[3], p2[3];
    matvec3(p1, xm1, cr1);
    matvec3(p2, xm2, cr2);
    for (int a = 0; a < 3; a++) {
      mx1[a] = fmaxf(mx1[a], p1[a]); mn1[a] = fminf(mn1[a], p1[a]);
      mx2[a] = fmaxf(mx2[a], p2[a]); mn2[a] = fminf(mn2[a], p2[a]);
    }
  }
  for (int a = 0; a < 3; a++) {
    if (cen1[a] + mx1[a] + margin < cen2[a] + mn2[a]) return false;
    if (cen2[a] + mx2[a] + margin < cen1[a] + mn1[a]) return false;
  }
  return true;
}

// collision_core.py:235-341: an explicit <pair> (pairid > -1, nxn_pairid[.][0]) supplies every parameter
// (:270-277); otherwise the geoms' parameters are mixed.  solreffriction (elliptic friction rows) is
// non-zero for explicit pairs only; `solreffriction` may be null where the caller reads it from the pair.
__device__ __forceinline__ void contact_params(const mjw_model_t& m, int wid, int g1, int g2, int pairid, float* margin, float* gap,
                                               int* condim, float* friction, float* solref, float* solimp,
                                               float* solreffriction = nullptr) {
  if (pairid > -1) {
    *margin = MR(pair_margin)[pairid];
    *gap = MR(pair_gap)[pairid];
    *condim = m.pair_dim[pairid];
    for (int i = 0; i < 5; i++) friction[i] = fmaxf(MJW_MINMU, MR(pair_friction)[5 * pairid + i]);
    for (int i = 0; i < 2; i++) solref[i] = MR(pair_solref)[2 * pairid + i];
    for (int i = 0; i < 5; i++) solimp[i] = MR(pair_solimp)[5 * pairid + i];
    if (solreffriction)
      for (int i = 0; i < 2; i++) solreffriction[i] = MR(pair_solreffriction)[2 * pairid + i];
    return;
  }
  if (solreffriction) solreffriction[0] = solreffriction[1] = 0.0f;
  const float* geom_solmix = MR(geom_solmix);
  const float* geom_friction = MR(geom_friction);
  const float* geom_solref = MR(geom_solref);
  const float* geom_solimp = MR(geom_solimp);
  const float* geom_margin = MR(geom_margin);
  const float* geom_gap = MR(geom_gap);
  float s1 = geom_solmix[g1], s2 = geom_solmix[g2];
  int c1 = m.geom_condim[g1], c2 = m.geom_condim[g2];
  int p1 = m.geom_priority[g1], p2 = m.geom_priority[g2];
  float mix, fr[3];
  if (p1 > p2) { mix = 1.0f; *condim = c1; for (int i = 0; i < 3; i++) fr[i] = geom_friction[3 * g1 + i]; }
  else if (p2 > p1) { mix = 0.0f; *condim = c2; for (int i = 0; i < 3; i++) fr[i] = geom_friction[3 * g2 + i]; }
  else {
    mix = safe_div(s1, s1 + s2);
    if (s1 < MJW_MINVAL && s2 < MJW_MINVAL) mix = 0.5f;
    else if (s1 < MJW_MINVAL && s2 >= MJW_MINVAL) mix = 0.0f;
    else if (s1 >= MJW_MINVAL && s2 < MJW_MINVAL) mix = 1.0f;
    *condim = c1 > c2 ? c1 : c2;
    for (int i = 0; i < 3; i++) fr[i] = fmaxf(geom_friction[3 * g1 + i], geom_friction[3 * g2 + i]);
  }
  friction[0] = fr[0]; friction[1] = fr[0]; friction[2] = fr[1]; friction[3] = fr[2]; friction[4] = fr[2];
  const float* sr1 = geom_solref + 2 * g1;
  const float* sr2 = geom_solref + 2 * g2;
  if (sr1[0] > 0.0f && sr2[0] > 0.0f) {
    for (int i = 0; i < 2; i++) solref[i] = mix * sr1[i] + (1.0f - mix) * sr2[i];
  } else {
    for (int i = 0; i < 2; i++) solref[i] = fminf(sr1[i], sr2[i]);
  }
  for (int i = 0; i < 5; i++) solimp[i] = mix * geom_solimp[5 * g1 + i] + (1.0f - mix) * geom_solimp[5 * g2 + i];
  *margin = geom_margin[g1] + geom_margin[g2];
  *gap = geom_gap[g1] + geom_gap[g2];
  for (int i = 0; i < 5; i++) friction[i] = fmaxf(MJW_MINMU, friction[i]);
}

// collision_primitive_core.py:519-613 plane_cylinder candidate k
__device__ __forceinline__ void plane_cylinder_k(int k, const float* n, const float* pp, const float* cc, const float* cax, float r, float hh, float* dist,
                                 float* pos) {
  float axis[3] = {cax[0], cax[1], cax[2]};
  float prjaxis = dot3(n, axis);
  if (prjaxis > 0.0f) {
    for (int i = 0; i < 3; i++) axis[i] = -axis[i];
    prjaxis = -prjaxis;
  }
  const float df[3] = {cc[0] - pp[0], cc[1] - pp[1], cc[2] - pp[2]};
  const float dist0 = dot3(df, n);
  float vec[3];
  for (int i = 0; i < 3; i++) vec[i] = axis[i] * prjaxis - n[i];
  const float len2 = dot3(vec, vec);
  if (len2 >= 1e-12f) {
    const float s = safe_div(r, sqrtf(len2));
    for (int i = 0; i < 3; i++) vec[i] *= s;
  } else {
    vec[0] = r;
    vec[1] = vec[2] = 0.0f;
  }
  const float prjvec = dot3(vec, n);
  for (int i = 0; i < 3; i++) axis[i] *= hh;
  prjaxis *= hh;
  if (k == 0) {
    *dist = dist0 + prjaxis + prjvec;
    for (int i = 0; i < 3; i++) pos[i] = cc[i] + vec[i] + axis[i] - n[i] * (*dist * 0.5f);
  } else if (k == 1) {
    *dist = dist0 - prjaxis + prjvec;
    for (int i = 0; i < 3; i++) pos[i] = cc[i] + vec[i] - axis[i] - n[i] * (*dist * 0.5f);
  } else {
    *dist = dist0 + prjaxis - prjvec * 0.5f;
    float v1[3];
    cross3(v1, vec, axis);
    normalize3(v1);
    const float s = r * sqrtf(3.0f) * 0.5f, sg = k == 2 ? 1.0f : -1.0f;
    for (int i = 0; i < 3; i++) pos[i] = cc[i] + sg * v1[i] * s + axis[i] - vec[i] * 0.5f - n[i] * (*dist * 0.5f);
  }
}

// collision_primitive.py:52-139, 257-277 plane_convex, exhaustive-search branch (the reference takes it
// for meshes without a hull graph; with one it hill-climbs the hull, which reaches the same deepest
// vertex a): the deepest vertex a, then among vertices within 1e-3 of its depth the one farthest from
// a (b), farthest from line ab (c) and from the triangle's other edges (d); each distinct vertex is a
// contact at its own depth.  One thread, serial over the vertices.
static __device__ __noinline__ int plane_mesh(const float* nw, const float* ppos, const float* gpos, const float* R, const float* mv, int nvert, float* dist,
                          float (*pos)[3]) {
  constexpr float HUGE_ = 1e6f;
  const float d0[3] = {ppos[0] - gpos[0], ppos[1] - gpos[1], ppos[2] - gpos[2]};
  float pl[3], n[3];
  for (int i = 0; i < 3; i++) {
    pl[i] = R[i] * d0[0] + R[3 + i] * d0[1] + R[6 + i] * d0[2];
    n[i] = R[i] * nw[0] + R[3 + i] * nw[1] + R[6 + i] * nw[2];
  }
  auto sup = [&](const float* v) { return (pl[0] - v[0]) * n[0] + (pl[1] - v[1]) * n[1] + (pl[2] - v[2]) * n[2]; };
  int idx[4] = {-1, -1, -1, -1};
  float maxs = -HUGE_, a[3] = {0, 0, 0}, b[3] = {0, 0, 0}, c[3] = {0, 0, 0};
  for (int i = 0; i < nvert; i++) {
    const float s = sup(mv + 3 * i);
    if (s > maxs) { maxs = s; idx[0] = i; a[0] = mv[3 * i]; a[1] = mv[3 * i + 1]; a[2] = mv[3 * i + 2]; }
  }
  if (maxs < 0.0f) return 0;
  const float thr = maxs - 1e-3f;
  float best = -HUGE_;
  for (int i = 0; i < nvert; i++) {
    const float* v = mv + 3 * i;
    const float mask = sup(v) > thr ? 0.0f : -HUGE_;
    const float dv[3] = {a[0] - v[0], a[1] - v[1], a[2] - v[2]};
    const float dd = dot3(dv, dv) + mask;
    if (dd > best) { idx[1] = i; best = dd; b[0] = v[0]; b[1] = v[1]; b[2] = v[2]; }
  }
  float ab[3], t[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
  cross3(ab, n, t);
  best = -HUGE_;
  for (int i = 0; i < nvert; i++) {
    const float* v = mv + 3 * i;
    const float mask = sup(v) > thr ? 0.0f : -HUGE_;
    const float ap[3] = {a[0] - v[0], a[1] - v[1], a[2] - v[2]};
    const float dd = fabsf(dot3(ap, ab)) + mask;
    if (dd > best) { idx[2] = i; best = dd; c[0] = v[0]; c[1] = v[1]; c[2] = v[2]; }
  }
  float ac[3], bc[3], t1[3] = {a[0] - c[0], a[1] - c[1], a[2] - c[2]}, t2[3] = {b[0] - c[0], b[1] - c[1], b[2] - c[2]};
  cross3(ac, n, t1);
  cross3(bc, n, t2);
  best = -HUGE_;
  for (int i = 0; i < nvert; i++) {
    const float* v = mv + 3 * i;
    const float mask = sup(v) > thr ? 0.0f : -HUGE_;
    const float ap[3] = {a[0] - v[0], a[1] - v[1], a[2] - v[2]}, bp[3] = {b[0] - v[0], b[1] - v[1], b[2] - v[2]};
    const float dd = (fabsf(dot3(ap, ac)) + mask) + (fabsf(dot3(bp, bc)) + mask);
    if (dd > best) { idx[3] = i; best = dd; }
  }
  int cnt = 0;
  for (int i = 3; i >= 0; i--) {
    int count = 0;
    for (int j = 0; j <= i; j++) count += idx[j] == idx[i];
    if (count != 1) continue;
    const float* v = mv + 3 * idx[i];
    const float dd = -sup(v);
    for (int k = 0; k < 3; k++) pos[cnt][k] = gpos[k] + R[3 * k] * v[0] + R[3 * k + 1] * v[1] + R[3 * k + 2] * v[2] - 0.5f * dd * nw[k];
    dist[cnt] = dd;
    cnt++;
  }
  return cnt;
}

// collision_primitive_core.py:364-392 plane_ellipsoid: the ellipsoid's support point against the plane
// normal (in the unit-sphere frame of the ellipsoid), the contact at the middle of the penetration
__device__ __forceinline__ float plane_ellipsoid(float* pos, const float* n, const float* ppos, const float* epos, const float* R,
                                                 const float* size) {
  float l[3];
  mat_t_vec3(l, R, n);
  for (int i = 0; i < 3; i++) l[i] *= size[i];
  normalize3(l);
  float sl[3] = {-l[0] * size[0], -l[1] * size[1], -l[2] * size[2]}, w[3];
  matvec3(w, R, sl);
  for (int i = 0; i < 3; i++) pos[i] = epos[i] + w[i];
  const float d[3] = {pos[0] - ppos[0], pos[1] - ppos[1], pos[2] - ppos[2]};
  const float dist = dot3(n, d);
  for (int i = 0; i < 3; i++) pos[i] -= n[i] * dist * 0.5f;
  return dist;
}

// collision_primitive_core.py:446-515 sphere_cylinder: side (sphere vs the axis point at the sphere's
// height), cap (plane of the nearer cap, normal flipped) or rim corner, whichever the sphere centre lies in
__device__ __forceinline__ float sphere_cylinder(float* pos, float* nrm, const float* sp, float sr, const float* cp, const float* ax, float cr,
                                                 float hh) {
  const float vec[3] = {sp[0] - cp[0], sp[1] - cp[1], sp[2] - cp[2]};
  const float x = dot3(vec, ax);
  const float a_proj[3] = {ax[0] * x, ax[1] * x, ax[2] * x};
  float p_proj[3] = {vec[0] - a_proj[0], vec[1] - a_proj[1], vec[2] - a_proj[2]};
  const float p2 = dot3(p_proj, p_proj);
  bool side = fabsf(x) < hh, cap = p2 < cr * cr;
  if (side && cap) {
    if (hh - fabsf(x) < cr - sqrtf(p2)) side = false;
    else cap = false;
  }
  if (side) {
    const float tgt[3] = {cp[0] + a_proj[0], cp[1] + a_proj[1], cp[2] + a_proj[2]};
    return sphere_sphere(pos, nrm, sp, sr, tgt, cr);
  }
  if (cap) {
    const float sg = x > 0.0f ? 1.0f : -1.0f;
    const float pc[3] = {cp[0] + sg * ax[0] * hh, cp[1] + sg * ax[1] * hh, cp[2] + sg * ax[2] * hh};
    const float pn[3] = {sg * ax[0], sg * ax[1], sg * ax[2]};
    const float dist = plane_sphere(pos, pn, pc, sp, sr);
    for (int i = 0; i < 3; i++) nrm[i] = -pn[i];
    return dist;
  }
  const float inv = safe_div(1.0f, sqrtf(p2));
  for (int i = 0; i < 3; i++) p_proj[i] *= cr * inv;
  const float sg = x < 0.0f ? -1.0f : 1.0f;  // wp.sign
  const float corner[3] = {cp[0] + ax[0] * sg * hh + p_proj[0], cp[1] + ax[1] * sg * hh + p_proj[1], cp[2] + ax[2] * sg * hh + p_proj[2]};
  return sphere_sphere(pos, nrm, sp, sr, corner, 0.0f);
}

}  // namespace mjw
