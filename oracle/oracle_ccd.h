/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY (included by oracle.c).
 *
 * Convex collision (GJK distance, EPA penetration, box multi-contact) restated from
 * mujoco_warp/_src/collision_gjk.py and the ccd kernels of collision_convex.py:158-890 (heightfield
 * prisms and the convex pairs of the reference's collision table, collision_driver.py:43-77).
 * Serial, one pair at a time.
 */
#include <stdint.h>

#define CCD_FLOAT_MAX ((real)1e30)
#define CCD_MINVAL ((real)1e-15)
#define CCD_MIN_DIST ((real)1e-10)
#define CCD_MAX_EPAFACES 5
#define CCD_MAX_EPAHORIZON 24
#define CCD_INTERSECT_TOL ((real)0.0000003)
#define CCD_MAX_ITER 64
#define CCD_FACE_DELETED 0x80000000u
#define CCD_FACE_INVALID 0x40000000u

/* collision_gjk.py:34-35 */
static real ccd_face_tol(void) { return cos((real)0.0016); }
static real ccd_edge_tol(void) { return sin((real)0.0016); }

typedef struct {
  real pos[3], rot[9], size[3], margin;
  int type;
  const real* vert; /* mesh vertices in the geom frame (GEOM_MESH) */
  int nvert;
  const real* prism; /* GEOM_HFIELD: the 6 prism vertices (heightfield frame); pos = the prism center */
  /* GEOM_MESH polygon data (mesh_poly*, offset to this mesh: pnormal / pvadr / pvnum by its polygon address,
   * pmapadr / pmapnum by its vertex address; pvert / pmap are the model's arrays, holding mesh-local vertex /
   * polygon ids); pnormal == NULL: no polygon data (no mesh multi-contact) */
  const real* pnormal;
  const int *pvadr, *pvnum, *pvert, *pmapadr, *pmapnum, *pmap;
} ccd_geom;

/* multi-contact workspace bounds (the reference sizes its buffers by the model's nmaxpolygon / nmaxmeshdeg) */
#define CCD_MAXPOLY 128
#define CCD_MAXDEG 64

typedef struct {
  int vertex_index;
  real point[3];
} ccd_sp;

static inline real ccd_sign(real x) { return x < 0 ? -1 : 1; } /* wp.sign */

/* collision_gjk.py:97-190 support (primitive types) */
static ccd_sp ccd_support(const ccd_geom* g, const real* dir) {
  ccd_sp sp;
  if (g->type == GEOM_HFIELD) { /* collision_gjk.py:178-187: first strict maximum over the prism, no pose */
    real best = -CCD_FLOAT_MAX;
    sp.vertex_index = dir[2] < 0 ? -2 : -3;
    sp.point[0] = sp.point[1] = sp.point[2] = 0;
    for (int i = 0; i < 6; i++) {
      const real* v = g->prism + 3 * i;
      real dd = v[0] * dir[0] + v[1] * dir[1] + v[2] * dir[2];
      if (dd > best) { best = dd; sp.point[0] = v[0]; sp.point[1] = v[1]; sp.point[2] = v[2]; }
    }
    if (g->margin > 0)
      for (int i = 0; i < 3; i++) sp.point[i] += dir[i] * (0.5 * g->margin);
    return sp;
  }
  sp.vertex_index = -1;
  real ld[3], res[3] = {0, 0, 0};
  for (int i = 0; i < 3; i++) ld[i] = g->rot[i] * dir[0] + g->rot[3 + i] * dir[1] + g->rot[6 + i] * dir[2];
  if (g->type == GEOM_SPHERE) {
    for (int i = 0; i < 3; i++) sp.point[i] = g->pos[i] + (g->size[0] + 0.5 * g->margin) * dir[i];
    return sp;
  }
  if (g->type == GEOM_BOX) {
    real t[3] = {ccd_sign(ld[0]), ccd_sign(ld[1]), ccd_sign(ld[2])};
    for (int i = 0; i < 3; i++) res[i] = t[i] * g->size[i];
    sp.vertex_index = (t[0] > 0) + 2 * (t[1] > 0) + 4 * (t[2] > 0);
  } else if (g->type == GEOM_CAPSULE) {
    for (int i = 0; i < 3; i++) res[i] = ld[i] * g->size[0];
    res[2] += ccd_sign(ld[2]) * g->size[1];
  } else if (g->type == GEOM_ELLIPSOID) {
    for (int i = 0; i < 3; i++) res[i] = ld[i] * g->size[i];
    normalize3(res);
    for (int i = 0; i < 3; i++) res[i] *= g->size[i];
  } else if (g->type == GEOM_CYLINDER) {
    real dd = sqrt(ld[0] * ld[0] + ld[1] * ld[1]);
    if (dd > CCD_MINVAL) { res[0] = ld[0] * g->size[0] / dd; res[1] = ld[1] * g->size[0] / dd; }
    res[2] = ccd_sign(ld[2]) * g->size[1];
  } else if (g->type == GEOM_MESH) { /* collision_gjk.py:136-151: exhaustive, first strict maximum */
    real best = -CCD_FLOAT_MAX;
    for (int i = 0; i < g->nvert; i++) {
      const real* v = g->vert + 3 * i;
      real dd = v[0] * ld[0] + v[1] * ld[1] + v[2] * ld[2];
      if (dd > best) { best = dd; sp.vertex_index = i; res[0] = v[0]; res[1] = v[1]; res[2] = v[2]; }
    }
  }
  for (int i = 0; i < 3; i++) sp.point[i] = g->rot[3 * i] * res[0] + g->rot[3 * i + 1] * res[1] + g->rot[3 * i + 2] * res[2] + g->pos[i];
  if (g->margin > 0)
    for (int i = 0; i < 3; i++) sp.point[i] += dir[i] * (0.5 * g->margin);
  return sp;
}

static inline real det3v(const real* a, const real* b, const real* c) {
  real t[3];
  cross3(t, b, c);
  return dot3(a, t);
}

static inline int same_sign(real a, real b) {
  if (a > 0 && b > 0) return 1;
  if (a < 0 && b < 0) return -1;
  return 0;
}

/* collision_gjk.py:279-284 */
static void project_origin_line(real* r, const real* v1, const real* v2) {
  real diff[3] = {v2[0] - v1[0], v2[1] - v1[1], v2[2] - v1[2]};
  real scl = -(dot3(v2, diff) / dot3(diff, diff));
  for (int i = 0; i < 3; i++) r[i] = v2[i] + scl * diff[i];
}

/* collision_gjk.py:286-315: returns 1 on degenerate input */
static int project_origin_plane(real* r, const real* v1, const real* v2, const real* v3) {
  real d21[3], d31[3], d32[3], n[3];
  for (int i = 0; i < 3; i++) { d21[i] = v2[i] - v1[i]; d31[i] = v3[i] - v1[i]; d32[i] = v3[i] - v2[i]; r[i] = 0; }
  cross3(n, d32, d21);
  real nv = dot3(n, v2), nn = dot3(n, n);
  if (nn == 0) return 1;
  if (nv != 0 && nn > CCD_MINVAL) { for (int i = 0; i < 3; i++) r[i] = (nv / nn) * n[i]; return 0; }
  cross3(n, d21, d31);
  nv = dot3(n, v1); nn = dot3(n, n);
  if (nn == 0) return 1;
  if (nv != 0 && nn > CCD_MINVAL) { for (int i = 0; i < 3; i++) r[i] = (nv / nn) * n[i]; return 0; }
  cross3(n, d31, d32);
  nv = dot3(n, v3); nn = dot3(n, n);
  for (int i = 0; i < 3; i++) r[i] = (nv / nn) * n[i];
  return 0;
}

/* collision_gjk.py:539-559 */
static void S1D(real* out, const real* s1, const real* s2) {
  real p[3];
  project_origin_line(p, s1, s2);
  real mu_max = 0;
  int index = 0;
  for (int i = 0; i < 3; i++) {
    real mu = s1[i] - s2[i];
    if (fabs(mu) >= fabs(mu_max)) { mu_max = mu; index = i; }
  }
  real C1 = p[index] - s2[index], C2 = s1[index] - p[index];
  if (same_sign(mu_max, C1) && same_sign(mu_max, C2)) { out[0] = C1 / mu_max; out[1] = C2 / mu_max; }
  else { out[0] = 0; out[1] = 1; }
}

/* collision_gjk.py:394-536 */
static void S2D(real* out, const real* s1, const real* s2, const real* s3) {
  real p[3];
  if (project_origin_plane(p, s1, s2, s3)) {
    real v[2];
    S1D(v, s1, s2);
    out[0] = v[0]; out[1] = v[1]; out[2] = 0;
    return;
  }
  real M14 = s2[1] * s3[2] - s2[2] * s3[1] - s1[1] * s3[2] + s1[2] * s3[1] + s1[1] * s2[2] - s1[2] * s2[1];
  real M24 = s2[0] * s3[2] - s2[2] * s3[0] - s1[0] * s3[2] + s1[2] * s3[0] + s1[0] * s2[2] - s1[2] * s2[0];
  real M34 = s2[0] * s3[1] - s2[1] * s3[0] - s1[0] * s3[1] + s1[1] * s3[0] + s1[0] * s2[1] - s1[1] * s2[0];
  real Mmax;
  int x, y;
  real mu1 = fabs(M14), mu2 = fabs(M24), mu3 = fabs(M34);
  if (mu1 >= mu2 && mu1 >= mu3) { Mmax = M14; x = 1; y = 2; }
  else if (mu2 >= mu3) { Mmax = M24; x = 0; y = 2; }
  else { Mmax = M34; x = 0; y = 1; }
  real a[2] = {s1[x], s1[y]}, b[2] = {s2[x], s2[y]}, c[2] = {s3[x], s3[y]}, o[2] = {p[x], p[y]};
  real C31 = o[0] * b[1] + o[1] * c[0] + b[0] * c[1] - o[0] * c[1] - o[1] * b[0] - c[0] * b[1];
  real C32 = o[0] * c[1] + o[1] * a[0] + c[0] * a[1] - o[0] * a[1] - o[1] * c[0] - a[0] * c[1];
  real C33 = o[0] * a[1] + o[1] * b[0] + a[0] * b[1] - o[0] * b[1] - o[1] * a[0] - b[0] * a[1];
  int comp1 = same_sign(Mmax, C31), comp2 = same_sign(Mmax, C32), comp3 = same_sign(Mmax, C33);
  if (comp1 && comp2 && comp3) { out[0] = C31 / Mmax; out[1] = C32 / Mmax; out[2] = C33 / Mmax; return; }
  real dmin = CCD_FLOAT_MAX, sc[2], xx[3];
  out[0] = out[1] = out[2] = 0;
  if (!comp1) {
    S1D(sc, s2, s3);
    for (int i = 0; i < 3; i++) xx[i] = sc[0] * s2[i] + sc[1] * s3[i];
    out[0] = 0; out[1] = sc[0]; out[2] = sc[1];
    dmin = dot3(xx, xx);
  }
  if (!comp2) {
    S1D(sc, s1, s3);
    for (int i = 0; i < 3; i++) xx[i] = sc[0] * s1[i] + sc[1] * s3[i];
    real dd = dot3(xx, xx);
    if (dd < dmin) { out[0] = sc[0]; out[1] = 0; out[2] = sc[1]; dmin = dd; }
  }
  if (!comp3) {
    S1D(sc, s1, s2);
    for (int i = 0; i < 3; i++) xx[i] = sc[0] * s1[i] + sc[1] * s2[i];
    real dd = dot3(xx, xx);
    if (dd < dmin) { out[0] = sc[0]; out[1] = sc[1]; out[2] = 0; }
  }
}

/* collision_gjk.py:318-391 */
static void S3D(real* out, const real* s1, const real* s2, const real* s3, const real* s4) {
  real C41 = -det3v(s2, s3, s4), C42 = det3v(s1, s3, s4), C43 = -det3v(s1, s2, s4), C44 = det3v(s1, s2, s3);
  real mdet = C41 + C42 + C43 + C44;
  int c1 = same_sign(mdet, C41), c2 = same_sign(mdet, C42), c3 = same_sign(mdet, C43), c4 = same_sign(mdet, C44);
  if (c1 && c2 && c3 && c4) { out[0] = C41 / mdet; out[1] = C42 / mdet; out[2] = C43 / mdet; out[3] = C44 / mdet; return; }
  real dmin = CCD_FLOAT_MAX, sc[3], xx[3];
  out[0] = out[1] = out[2] = out[3] = 0;
  if (!c1) {
    S2D(sc, s2, s3, s4);
    for (int i = 0; i < 3; i++) xx[i] = sc[0] * s2[i] + sc[1] * s3[i] + sc[2] * s4[i];
    out[0] = 0; out[1] = sc[0]; out[2] = sc[1]; out[3] = sc[2];
    dmin = dot3(xx, xx);
  }
  if (!c2) {
    S2D(sc, s1, s3, s4);
    for (int i = 0; i < 3; i++) xx[i] = sc[0] * s1[i] + sc[1] * s3[i] + sc[2] * s4[i];
    real dd = dot3(xx, xx);
    if (dd < dmin) { out[0] = sc[0]; out[1] = 0; out[2] = sc[1]; out[3] = sc[2]; dmin = dd; }
  }
  if (!c3) {
    S2D(sc, s1, s2, s4);
    for (int i = 0; i < 3; i++) xx[i] = sc[0] * s1[i] + sc[1] * s2[i] + sc[2] * s4[i];
    real dd = dot3(xx, xx);
    if (dd < dmin) { out[0] = sc[0]; out[1] = sc[1]; out[2] = 0; out[3] = sc[2]; dmin = dd; }
  }
  if (!c4) {
    S2D(sc, s1, s2, s3);
    for (int i = 0; i < 3; i++) xx[i] = sc[0] * s1[i] + sc[1] * s2[i] + sc[2] * s3[i];
    real dd = dot3(xx, xx);
    if (dd < dmin) { out[0] = sc[0]; out[1] = sc[1]; out[2] = sc[2]; out[3] = 0; }
  }
}

typedef struct {
  real dist;
  real x1[3], x2[3];
  int dim;
  real simplex[4][3], simplex1[4][3], simplex2[4][3];
  int index1[4], index2[4];
} gjk_result;

static void lin_comb(real* v, int n, const real* coefs, real mat[4][3]) {
  for (int i = 0; i < 3; i++) {
    real s = coefs[0] * mat[0][i];
    for (int k = 1; k < n; k++) s += coefs[k] * mat[k][i];
    v[i] = s;
  }
}

/* collision_gjk.py:562-685 */
static gjk_result gjk(real tolerance, int iterations, const ccd_geom* g1, const ccd_geom* g2, const real* x1_0, const real* x2_0,
                      real cutoff, int is_discrete) {
  gjk_result r;
  memset(&r, 0, sizeof(r));
  real cutoff2 = cutoff * cutoff, tol2 = tolerance * tolerance;
  real epsilon = is_discrete ? 0 : 0.5 * tol2;
  real coords[4] = {0, 0, 0, 0};
  int n = 0;
  real xk[3] = {x1_0[0] - x2_0[0], x1_0[1] - x2_0[1], x1_0[2] - x2_0[2]};
  real xnorm_old = CCD_FLOAT_MAX;
  for (int it = 0; it < iterations; it++) {
    real xnorm = dot3(xk, xk);
    if (xnorm < tol2 || fabs(xnorm_old - xnorm) < tol2) break;
    xnorm_old = xnorm;
    real sq = sqrt(xnorm);
    real dneg[3] = {xk[0] / sq, xk[1] / sq, xk[2] / sq}, dpos[3] = {-dneg[0], -dneg[1], -dneg[2]};
    ccd_sp s1 = ccd_support(g1, dpos), s2 = ccd_support(g2, dneg);
    for (int i = 0; i < 3; i++) {
      r.simplex1[n][i] = s1.point[i];
      r.simplex2[n][i] = s2.point[i];
      r.simplex[n][i] = s1.point[i] - s2.point[i];
    }
    r.index1[n] = s1.vertex_index;
    r.index2[n] = s2.vertex_index;
    real vs = dot3(xk, r.simplex[n]);
    if (cutoff == 0) {
      if (vs > 0) { r.dim = 0; r.dist = CCD_FLOAT_MAX; return r; }
    } else if (cutoff < CCD_FLOAT_MAX) {
      if (vs > 0 && (vs * vs / xnorm) >= cutoff2) { r.dim = 0; r.dist = CCD_FLOAT_MAX; return r; }
    }
    real dk[3] = {xk[0] - r.simplex[n][0], xk[1] - r.simplex[n][1], xk[2] - r.simplex[n][2]};
    if (dot3(xk, dk) < epsilon) break;
    int nn = n + 1;
    if (nn == 4) S3D(coords, r.simplex[0], r.simplex[1], r.simplex[2], r.simplex[3]);
    else if (nn == 3) { S2D(coords, r.simplex[0], r.simplex[1], r.simplex[2]); coords[3] = 0; }
    else if (nn == 2) { S1D(coords, r.simplex[0], r.simplex[1]); coords[2] = coords[3] = 0; }
    else { coords[0] = 1; coords[1] = coords[2] = coords[3] = 0; }
    n = 0;
    for (int i = 0; i < 4; i++) {
      if (coords[i] == 0) continue;
      memcpy(r.simplex[n], r.simplex[i], sizeof(r.simplex[n]));
      memcpy(r.simplex1[n], r.simplex1[i], sizeof(r.simplex1[n]));
      memcpy(r.simplex2[n], r.simplex2[i], sizeof(r.simplex2[n]));
      r.index1[n] = r.index1[i];
      r.index2[n] = r.index2[i];
      coords[n] = coords[i];
      n++;
    }
    if (n < 1) break;
    real xn[3];
    lin_comb(xn, n, coords, r.simplex);
    if (fabs(xn[0] - xk[0]) < CCD_MINVAL && fabs(xn[1] - xk[1]) < CCD_MINVAL && fabs(xn[2] - xk[2]) < CCD_MINVAL) break;
    memcpy(xk, xn, sizeof(xk));
    if (n == 4) break;
  }
  if (n == 0) { memcpy(r.x1, x1_0, 3 * sizeof(real)); memcpy(r.x2, x2_0, 3 * sizeof(real)); }
  else { lin_comb(r.x1, n, coords, r.simplex1); lin_comb(r.x2, n, coords, r.simplex2); }
  r.dist = sqrt(dot3(xk, xk));
  r.dim = n;
  return r;
}

/* EPA polytope (collision_gjk.py:57-76) */
typedef struct {
  int status, nvert, nface, nhorizon;
  int cap_vert, cap_face;
  real vert[2 * (10 + 2 * CCD_MAX_ITER)][3];
  int vert_index[2 * (10 + 2 * CCD_MAX_ITER)];
  uint32_t face[6 + CCD_MAX_EPAFACES * CCD_MAX_ITER];
  real face_pr[6 + CCD_MAX_EPAFACES * CCD_MAX_ITER][3];
  real face_norm2[6 + CCD_MAX_EPAFACES * CCD_MAX_ITER];
  uint32_t horizon[CCD_MAX_EPAHORIZON];
} polytope;

static void face_verts(uint32_t f, int* v) { v[0] = f & 0x3FF; v[1] = (f >> 10) & 0x3FF; v[2] = (f >> 20) & 0x3FF; }

static void pvert(const polytope* pt, int v, real* out) {
  for (int i = 0; i < 3; i++) out[i] = pt->vert[2 * v][i] - pt->vert[2 * v + 1][i];
}

/* collision_gjk.py:194-213 */
static real attach_face(polytope* pt, int idx, int v1, int v2, int v3) {
  if (pt->nface == pt->cap_face) return 0;
  real p1[3], p2[3], p3[3], r[3];
  pvert(pt, v1, p1); pvert(pt, v2, p2); pvert(pt, v3, p3);
  if (project_origin_plane(r, p3, p2, p1)) return 0;
  pt->face[idx] = (uint32_t)(v1 + (v2 << 10) + (v3 << 20));
  memcpy(pt->face_pr[idx], r, sizeof(r));
  pt->face_norm2[idx] = dot3(r, r);
  return pt->face_norm2[idx];
}

/* collision_gjk.py:216-230 */
static void epa_support(polytope* pt, int idx, const ccd_geom* g1, const ccd_geom* g2, const real* dir) {
  real nd[3] = {-dir[0], -dir[1], -dir[2]};
  ccd_sp s1 = ccd_support(g1, dir), s2 = ccd_support(g2, nd);
  memcpy(pt->vert[2 * idx], s1.point, 3 * sizeof(real));
  memcpy(pt->vert[2 * idx + 1], s2.point, 3 * sizeof(real));
  pt->vert_index[2 * idx] = s1.vertex_index;
  pt->vert_index[2 * idx + 1] = s2.vertex_index;
}

/* collision_gjk.py:701-741 */
static void tri_affine_coord(real* out, const real* v1, const real* v2, const real* v3, const real* p) {
  real M14 = v2[1] * v3[2] - v2[2] * v3[1] - v1[1] * v3[2] + v1[2] * v3[1] + v1[1] * v2[2] - v1[2] * v2[1];
  real M24 = v2[0] * v3[2] - v2[2] * v3[0] - v1[0] * v3[2] + v1[2] * v3[0] + v1[0] * v2[2] - v1[2] * v2[0];
  real M34 = v2[0] * v3[1] - v2[1] * v3[0] - v1[0] * v3[1] + v1[1] * v3[0] + v1[0] * v2[1] - v1[1] * v2[0];
  real Mmax;
  int x, y;
  real mu1 = fabs(M14), mu2 = fabs(M24), mu3 = fabs(M34);
  if (mu1 >= mu2 && mu1 >= mu3) { Mmax = M14; x = 1; y = 2; }
  else if (mu2 >= mu3) { Mmax = M24; x = 0; y = 2; }
  else { Mmax = M34; x = 0; y = 1; }
  real C31 = p[x] * v2[y] + p[y] * v3[x] + v2[x] * v3[y] - p[x] * v3[y] - p[y] * v2[x] - v3[x] * v2[y];
  real C32 = p[x] * v3[y] + p[y] * v1[x] + v3[x] * v1[y] - p[x] * v1[y] - p[y] * v3[x] - v1[x] * v3[y];
  real C33 = p[x] * v1[y] + p[y] * v2[x] + v1[x] * v2[y] - p[x] * v2[y] - p[y] * v1[x] - v2[x] * v1[y];
  out[0] = C31 / Mmax; out[1] = C32 / Mmax; out[2] = C33 / Mmax;
}

/* collision_gjk.py:744-758 */
static int tri_point_intersect(const real* v1, const real* v2, const real* v3, const real* p) {
  real c[3];
  tri_affine_coord(c, v1, v2, v3, p);
  if (c[0] < 0 || c[1] < 0 || c[2] < 0) return 0;
  real d[3];
  for (int i = 0; i < 3; i++) d[i] = v1[i] * c[0] + v2[i] * c[1] + v3[i] * c[2] - p[i];
  return sqrt(dot3(d, d)) < CCD_MINVAL;
}

/* collision_gjk.py:688-698 */
static int same_side(const real* p0, const real* p1, const real* p2, const real* p3) {
  real a[3], b[3], n[3], c[3], m0[3] = {-p0[0], -p0[1], -p0[2]};
  for (int i = 0; i < 3; i++) { a[i] = p1[i] - p0[i]; b[i] = p2[i] - p0[i]; c[i] = p3[i] - p0[i]; }
  cross3(n, a, b);
  real d1 = dot3(n, c), d2 = dot3(n, m0);
  return (d1 > 0 && d2 > 0) || (d1 < 0 && d2 < 0);
}
static int test_tetra(const real* p0, const real* p1, const real* p2, const real* p3) {
  return same_side(p0, p1, p2, p3) && same_side(p1, p2, p3, p0) && same_side(p2, p3, p0, p1) && same_side(p3, p0, p1, p2);
}

/* collision_gjk.py:761-797: reset the GJK simplex to polytope vertices v1 v2 v3 */
static void replace_simplex3(gjk_result* r, const polytope* pt, int v1, int v2, int v3) {
  int vs[3] = {v1, v2, v3};
  for (int k = 0; k < 3; k++) {
    for (int i = 0; i < 3; i++) {
      r->simplex1[k][i] = pt->vert[2 * vs[k]][i];
      r->simplex2[k][i] = pt->vert[2 * vs[k] + 1][i];
      r->simplex[k][i] = r->simplex1[k][i] - r->simplex2[k][i];
    }
    r->index1[k] = pt->vert_index[2 * vs[k]];
    r->index2[k] = pt->vert_index[2 * vs[k] + 1];
  }
  r->dim = 3;
}

/* collision_gjk.py:800-819 */
static void rotmat120(real* R, const real* axis) {
  real n = sqrt(dot3(axis, axis));
  real u1 = axis[0] / n, u2 = axis[1] / n, u3 = axis[2] / n;
  real s = 0.86602540378, c = -0.5;
  R[0] = c + u1 * u1 * (1 - c); R[1] = u1 * u2 * (1 - c) - u3 * s; R[2] = u1 * u3 * (1 - c) + u2 * s;
  R[3] = u2 * u1 * (1 - c) + u3 * s; R[4] = c + u2 * u2 * (1 - c); R[5] = u2 * u3 * (1 - c) - u1 * s;
  R[6] = u1 * u3 * (1 - c) - u2 * s; R[7] = u2 * u3 * (1 - c) + u1 * s; R[8] = c + u3 * u3 * (1 - c);
}

/* collision_gjk.py:822-832 */
static int ray_triangle(const real* v1, const real* v2, const real* v3, const real* v4, const real* v5) {
  real a[3], b[3], c[3], d[3];
  for (int i = 0; i < 3; i++) { a[i] = v3[i] - v1[i]; b[i] = v4[i] - v1[i]; c[i] = v2[i] - v1[i]; d[i] = v5[i] - v1[i]; }
  real vol1 = det3v(a, b, c), vol2 = det3v(b, d, c), vol3 = det3v(d, a, c);
  if (vol1 >= 0 && vol2 >= 0 && vol3 >= 0) return 1;
  if (vol1 <= 0 && vol2 <= 0 && vol3 <= 0) return -1;
  return 0;
}

/* collision_gjk.py:840-858 */
static int add_edge(polytope* pt, int e1, int e2) {
  int n = pt->nhorizon;
  if (n < 0) return -1;
  uint32_t edge = (uint32_t)(((e1 < e2 ? e1 : e2) << 10) | (e1 > e2 ? e1 : e2));
  for (int i = 0; i < n; i++) {
    if (edge == pt->horizon[i]) { pt->horizon[i] = pt->horizon[n - 1]; return n - 1; }
  }
  if (n == CCD_MAX_EPAHORIZON) return -1;
  pt->horizon[n] = edge;
  return n + 1;
}

/* collision_gjk.py:936-1023 */
static int polytope2(polytope* pt, gjk_result* r, const ccd_geom* g1, const ccd_geom* g2) {
  real diff[3];
  for (int i = 0; i < 3; i++) diff[i] = r->simplex[1][i] - r->simplex[0][i];
  real value = CCD_FLOAT_MAX;
  int index = 0;
  for (int i = 0; i < 3; i++)
    if (fabs(diff[i]) < value) { value = fabs(diff[i]); index = i; }
  real e[3] = {0, 0, 0}, d1[3], d2[3], d3[3], R[9];
  e[index] = 1;
  cross3(d1, e, diff);
  rotmat120(R, diff);
  matvec3(d2, R, d1);
  matvec3(d3, R, d2);
  memcpy(pt->vert[0], r->simplex1[0], 3 * sizeof(real)); memcpy(pt->vert[1], r->simplex2[0], 3 * sizeof(real));
  memcpy(pt->vert[2], r->simplex1[1], 3 * sizeof(real)); memcpy(pt->vert[3], r->simplex2[1], 3 * sizeof(real));
  pt->vert_index[0] = r->index1[0]; pt->vert_index[1] = r->index2[0];
  pt->vert_index[2] = r->index1[1]; pt->vert_index[3] = r->index2[1];
  real n1 = sqrt(dot3(d1, d1)), n2 = sqrt(dot3(d2, d2)), n3 = sqrt(dot3(d3, d3));
  real u1[3] = {d1[0] / n1, d1[1] / n1, d1[2] / n1}, u2[3] = {d2[0] / n2, d2[1] / n2, d2[2] / n2}, u3[3] = {d3[0] / n3, d3[1] / n3, d3[2] / n3};
  epa_support(pt, 2, g1, g2, u1);
  epa_support(pt, 3, g1, g2, u2);
  epa_support(pt, 4, g1, g2, u3);
  static const int F[6][3] = {{0, 2, 3}, {0, 4, 2}, {0, 3, 4}, {1, 3, 2}, {1, 2, 4}, {1, 4, 3}};
  for (int k = 0; k < 6; k++) {
    if (attach_face(pt, k, F[k][0], F[k][1], F[k][2]) < CCD_MIN_DIST) {
      replace_simplex3(r, pt, F[k][0], F[k][1], F[k][2]);
      return -1;
    }
  }
  real v2[3], v3[3], v4[3];
  pvert(pt, 2, v2); pvert(pt, 3, v3); pvert(pt, 4, v4);
  if (!ray_triangle(r->simplex[0], r->simplex[1], v2, v3, v4)) return 1;
  pt->nvert = 5;
  pt->nface = 6;
  return 0;
}

/* collision_gjk.py:1026-1111 */
static int polytope3(polytope* pt, real dist, const gjk_result* r, const ccd_geom* g1, const ccd_geom* g2) {
  real a[3], b[3], n[3];
  for (int i = 0; i < 3; i++) { a[i] = r->simplex[1][i] - r->simplex[0][i]; b[i] = r->simplex[2][i] - r->simplex[0][i]; }
  cross3(n, a, b);
  if (sqrt(dot3(n, n)) < CCD_MINVAL) return 2;
  for (int k = 0; k < 3; k++) {
    memcpy(pt->vert[2 * k], r->simplex1[k], 3 * sizeof(real));
    memcpy(pt->vert[2 * k + 1], r->simplex2[k], 3 * sizeof(real));
    pt->vert_index[2 * k] = r->index1[k];
    pt->vert_index[2 * k + 1] = r->index2[k];
  }
  real nn[3] = {-n[0], -n[1], -n[2]};
  epa_support(pt, 3, g1, g2, nn);
  epa_support(pt, 4, g1, g2, n);
  real v4[3], v5[3];
  pvert(pt, 3, v4); pvert(pt, 4, v5);
  const real *v1 = r->simplex[0], *v2 = r->simplex[1], *v3 = r->simplex[2];
  if (tri_point_intersect(v1, v2, v3, v4)) return 3;
  if (tri_point_intersect(v1, v2, v3, v5)) return 4;
  if (dist > 1e-5 && !test_tetra(v1, v2, v3, v4) && !test_tetra(v1, v2, v3, v5)) return 5;
  static const int F[6][3] = {{4, 0, 1}, {4, 2, 0}, {4, 1, 2}, {3, 1, 0}, {3, 0, 2}, {3, 2, 1}};
  for (int k = 0; k < 6; k++)
    if (attach_face(pt, k, F[k][0], F[k][1], F[k][2]) < CCD_MIN_DIST) return 6 + k;
  pt->nvert = 5;
  pt->nface = 6;
  return 0;
}

/* collision_gjk.py:1114-1168 */
static int polytope4(polytope* pt, gjk_result* r) {
  for (int k = 0; k < 4; k++) {
    memcpy(pt->vert[2 * k], r->simplex1[k], 3 * sizeof(real));
    memcpy(pt->vert[2 * k + 1], r->simplex2[k], 3 * sizeof(real));
    pt->vert_index[2 * k] = r->index1[k];
    pt->vert_index[2 * k + 1] = r->index2[k];
  }
  static const int F[4][3] = {{0, 1, 2}, {0, 3, 1}, {0, 2, 3}, {3, 2, 1}};
  for (int k = 0; k < 4; k++) {
    if (attach_face(pt, k, F[k][0], F[k][1], F[k][2]) < CCD_MIN_DIST) {
      replace_simplex3(r, pt, F[k][0], F[k][1], F[k][2]);
      return -1;
    }
  }
  if (!test_tetra(r->simplex[0], r->simplex[1], r->simplex[2], r->simplex[3])) return 12;
  pt->nvert = 4;
  pt->nface = 4;
  return 0;
}

/* collision_gjk.py:2173-2186 / 914-921: the heightfield-side witness under x2 on the prism's top triangle
 * (vertical projection inside it, else onto the horizontal plane through the nearest corner) */
static real hfield_top_witness(const ccd_geom* g1, const real* x2, real* x1) {
  const real *a = g1->prism + 9, *b = g1->prism + 12, *c = g1->prism + 15;
  real co[3];
  tri_affine_coord(co, a, b, c, x2);
  if (co[0] > 0 && co[1] > 0 && co[2] > 0) {
    for (int i = 0; i < 3; i++) x1[i] = co[0] * a[i] + co[1] * b[i] + co[2] * c[i];
  } else {
    const real* p = c;
    if (co[1] > 0) p = b;
    if (co[0] > 0) p = a;
    real dz = x2[2] - p[2];
    x1[0] = x2[0]; x1[1] = x2[1]; x1[2] = x2[2] - dz;
  }
  real dd[3] = {x1[0] - x2[0], x1[1] - x2[1], x1[2] - x2[2]};
  return -sqrt(dot3(dd, dd));
}

/* collision_gjk.py:861-933 */
static real epa_witness(const polytope* pt, int fidx, const ccd_geom* g1, const ccd_geom* g2, real* x1, real* x2) {
  int f[3];
  face_verts(pt->face[fidx], f);
  real v1[3], v2[3], v3[3], c[3];
  pvert(pt, f[0], v1); pvert(pt, f[1], v2); pvert(pt, f[2], v3);
  tri_affine_coord(c, v1, v2, v3, pt->face_pr[fidx]);
  for (int i = 0; i < 3; i++) {
    x2[i] = pt->vert[2 * f[0] + 1][i] * c[0] + pt->vert[2 * f[1] + 1][i] * c[1] + pt->vert[2 * f[2] + 1][i] * c[2];
    x1[i] = pt->vert[2 * f[0]][i] * c[0] + pt->vert[2 * f[1]][i] * c[1] + pt->vert[2 * f[2]][i] * c[2];
  }
  int i1 = pt->vert_index[2 * f[0]], i2 = pt->vert_index[2 * f[1]], i3 = pt->vert_index[2 * f[2]];
  if (g1->type == GEOM_HFIELD && (i1 != i2 || i1 != i3)) { /* :886-922 a face across the prism's top and bottom */
    ccd_sp sp;
    if (g2->type == GEOM_CAPSULE || g2->type == GEOM_SPHERE) {
      ccd_geom g = *g2;
      g.margin = 0;
      g.size[0] = 0;
      sp = ccd_support(&g, x2);
      for (int i = 0; i < 3; i++) x2[i] = sp.point[i];
      x2[2] -= 0.5 * g2->margin + g2->size[0];
    } else {
      normalize3(x2);
      sp = ccd_support(g2, x2);
      for (int i = 0; i < 3; i++) x2[i] = sp.point[i];
    }
    return hfield_top_witness(g1, x2, x1);
  }
  return -sqrt(pt->face_norm2[fidx]);
}

/* collision_gjk.py:1201-1328; returns the face index or -1 */
static int epa(real tolerance, int iterations, polytope* pt, const ccd_geom* g1, const ccd_geom* g2, int is_discrete, real* dist,
               real* x1, real* x2) {
  real upper = CCD_FLOAT_MAX, upper2 = CCD_FLOAT_MAX;
  int idx = -1, pidx = -1;
  real epsilon = is_discrete ? 1e-15 : tolerance;
  int nvalid = pt->nface;
  if (iterations > 1000) iterations = 1000;
  for (int it = 0; it < iterations; it++) {
    pidx = idx;
    idx = -1;
    real lower2 = CCD_FLOAT_MAX;
    for (int i = 0; i < pt->nface; i++)
      if (!(pt->face[i] & (CCD_FACE_DELETED | CCD_FACE_INVALID)) && pt->face_norm2[i] < lower2) { idx = i; lower2 = pt->face_norm2[i]; }
    if (lower2 > upper2 || idx < 0) { idx = pidx; break; }
    if (lower2 <= 0) break;
    real lower = sqrt(lower2);
    int wi = pt->nvert;
    real dir[3] = {pt->face_pr[idx][0] / lower, pt->face_pr[idx][1] / lower, pt->face_pr[idx][2] / lower};
    epa_support(pt, wi, g1, g2, dir);
    real w[3];
    pvert(pt, wi, w);
    pt->nvert++;
    real upper_k = dot3(dir, w);
    if (upper_k < upper) { upper = upper_k; upper2 = upper * upper; }
    if (upper - lower < epsilon) break;
    if (is_discrete) {
      int rep = 0;
      for (int i = 0; i < pt->nvert - 1; i++)
        if (pt->vert_index[2 * i] == pt->vert_index[2 * wi] && pt->vert_index[2 * i + 1] == pt->vert_index[2 * wi + 1]) { rep = 1; break; }
      if (rep) break;
    }
    nvalid--;
    pt->face[idx] |= CCD_FACE_DELETED;
    int f[3];
    face_verts(pt->face[idx], f);
    pt->nhorizon = add_edge(pt, f[0], f[1]);
    pt->nhorizon = add_edge(pt, f[1], f[2]);
    pt->nhorizon = add_edge(pt, f[2], f[0]);
    if (pt->nhorizon == -1) { idx = -1; break; }
    for (int i = 0; i < pt->nface; i++) {
      if (pt->face[i] & CCD_FACE_DELETED) continue;
      if (dot3(pt->face_pr[i], w) - pt->face_norm2[i] > 1e-10) {
        if (!(pt->face[i] & (CCD_FACE_DELETED | CCD_FACE_INVALID))) nvalid--;
        pt->face[i] |= CCD_FACE_DELETED;
        face_verts(pt->face[i], f);
        pt->nhorizon = add_edge(pt, f[0], f[1]);
        pt->nhorizon = add_edge(pt, f[1], f[2]);
        pt->nhorizon = add_edge(pt, f[2], f[0]);
        if (pt->nhorizon == -1) { idx = -1; break; }
      }
    }
    for (int i = 0; i < pt->nhorizon; i++) {
      int e0 = pt->horizon[i] & 0x3FF, e1 = (pt->horizon[i] >> 10) & 0x3FF;
      real d2 = attach_face(pt, pt->nface, wi, e0, e1);
      if (d2 == 0) { idx = -1; break; }
      pt->nface++;
      if (d2 >= lower2 && d2 <= upper2) nvalid++;
      else pt->face[pt->nface - 1] |= CCD_FACE_INVALID;
    }
    if (nvalid == 0 || idx == -1) break;
    pt->nhorizon = 0;
  }
  if (idx > -1) {
    *dist = epa_witness(pt, idx, g1, g2, x1, x2);
    return idx;
  }
  *dist = 0;
  return -1;
}

/* ---- box multi-contact (collision_gjk.py:1331-2150, box branches) ---- */
static real area4(const real* a, const real* b, const real* c, const real* d) {
  real t1[3], t2[3], c1[3], c2[3];
  for (int i = 0; i < 3; i++) { t1[i] = a[i] - d[i]; t2[i] = d[i] - b[i]; }
  cross3(c1, t1, t2);
  for (int i = 0; i < 3; i++) { t1[i] = b[i] - c[i]; t2[i] = c[i] - a[i]; }
  cross3(c2, t1, t2);
  for (int i = 0; i < 3; i++) c1[i] += c2[i];
  return 0.5 * sqrt(dot3(c1, c1));
}

static void polygon_quad(int* res, real poly[][3], int np) {
  int b = 1, c = 2, d = 3;
  res[0] = 0; res[1] = b; res[2] = c; res[3] = d;
  real m = area4(poly[0], poly[b], poly[c], poly[d]);
  for (int a = 0; a < np; a++) {
    while (1) {
      real mn = area4(poly[a], poly[b], poly[c], poly[(d + 1) % np]);
      if (mn <= m) break;
      m = mn; d = (d + 1) % np;
      res[0] = a; res[1] = b; res[2] = c; res[3] = d;
      while (1) {
        mn = area4(poly[a], poly[b], poly[(c + 1) % np], poly[d]);
        if (mn <= m) break;
        m = mn; c = (c + 1) % np;
        res[0] = a; res[1] = b; res[2] = c; res[3] = d;
      }
      while (1) {
        mn = area4(poly[a], poly[(b + 1) % np], poly[c], poly[d]);
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

/* collision_gjk.py:1377-1400 */
static int feature_dim(const int* face, const polytope* pt, int offset, int* fi, real fv[3][3]) {
  int v1i = pt->vert_index[2 * face[0] + offset], v2i = pt->vert_index[2 * face[1] + offset], v3i = pt->vert_index[2 * face[2] + offset];
  fi[0] = v1i; fi[1] = v2i; fi[2] = v3i;
  for (int k = 0; k < 3; k++) memcpy(fv[k], pt->vert[2 * face[k] + offset], 3 * sizeof(real));
  if (v1i != v2i) return (v3i == v1i || v3i == v2i) ? 2 : 3;
  fi[1] = v3i;
  memcpy(fv[1], pt->vert[2 * face[2] + offset], 3 * sizeof(real));
  return v1i != v3i ? 2 : 1;
}

static void matvec3r(real* r, const real* M, real x, real y, real z) {
  for (int i = 0; i < 3; i++) r[i] = M[3 * i] * x + M[3 * i + 1] * y + M[3 * i + 2] * z;
}

/* collision_gjk.py:1577-1607 */
static int box_normals2(const real* mat, const real* n, real nout[][3], int* iout) {
  static const real FN[6][3] = {{1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1}};
  real ln[3];
  for (int i = 0; i < 3; i++) ln[i] = mat[i] * n[0] + mat[3 + i] * n[1] + mat[6 + i] * n[2];
  normalize3(ln);
  for (int i = 0; i < 6; i++) {
    if (dot3(ln, FN[i]) > ccd_face_tol()) {
      matvec3r(nout[0], mat, FN[i][0], FN[i][1], FN[i][2]);
      iout[0] = i;
      return 1;
    }
  }
  return 0;
}

/* collision_gjk.py:1610-1681 */
static int box_normals(int dim, const int* fi, const real* mat, const real* dir, real nout[][3], int* iout) {
  int v1 = fi[0], v2 = fi[1], v3 = fi[2];
  if (dim == 3) {
    int c = 0;
    real x = (real)((v1 & 1) && (v2 & 1) && (v3 & 1)) - (real)(!(v1 & 1) && !(v2 & 1) && !(v3 & 1));
    real y = (real)((v1 & 2) && (v2 & 2) && (v3 & 2)) - (real)(!(v1 & 2) && !(v2 & 2) && !(v3 & 2));
    real z = (real)((v1 & 4) && (v2 & 4) && (v3 & 4)) - (real)(!(v1 & 4) && !(v2 & 4) && !(v3 & 4));
    matvec3r(nout[0], mat, x, y, z);
    real sgn = x + y + z;
    if (x != 0) iout[c++] = 0;
    if (y != 0) iout[c++] = 2;
    if (z != 0) iout[c++] = 4;
    if (sgn == -1) iout[0] = iout[0] + 1;
    if (c == 1) return 1;
    return box_normals2(mat, dir, nout, iout);
  }
  if (dim == 2) {
    int c = 0;
    real x = (real)((v1 & 1) && (v2 & 1)) - (real)(!(v1 & 1) && !(v2 & 1));
    real y = (real)((v1 & 2) && (v2 & 2)) - (real)(!(v1 & 2) && !(v2 & 2));
    real z = (real)((v1 & 4) && (v2 & 4)) - (real)(!(v1 & 4) && !(v2 & 4));
    if (x != 0) { matvec3r(nout[c], mat, x, 0, 0); iout[c] = x > 0 ? 0 : 1; c++; }
    if (y != 0) { matvec3r(nout[c], mat, 0, y, 0); iout[c] = y > 0 ? 2 : 3; c++; }
    if (z != 0) { matvec3r(nout[c], mat, 0, 0, z); iout[c] = z > 0 ? 4 : 5; c++; }
    if (c == 1 || c == 2) return c;
    return box_normals2(mat, dir, nout, iout);
  }
  if (dim == 1) {
    real x = (v1 & 1) ? 1 : -1, y = (v1 & 2) ? 1 : -1, z = (v1 & 4) ? 1 : -1;
    matvec3r(nout[0], mat, x, 0, 0);
    matvec3r(nout[1], mat, 0, y, 0);
    matvec3r(nout[2], mat, 0, 0, z);
    iout[0] = x > 0 ? 0 : 1; iout[1] = y > 0 ? 2 : 3; iout[2] = z > 0 ? 4 : 5;
    return 3;
  }
  return 0;
}

/* collision_gjk.py:1684-1719 */
static int box_edge_normals(int dim, const real* mat, const real* pos, const real* size, const real* v1, const real* v2, int v1i,
                            real nout[][3], real endvert[][3]) {
  if (dim == 2) {
    memcpy(endvert[0], v2, 3 * sizeof(real));
    for (int i = 0; i < 3; i++) nout[0][i] = v2[i] - v1[i];
    normalize3(nout[0]);
    return 1;
  }
  if (dim == 1) {
    real x = (v1i & 1) ? size[0] : -size[0], y = (v1i & 2) ? size[1] : -size[1], z = (v1i & 4) ? size[2] : -size[2];
    real p[3][3] = {{-x, y, z}, {x, -y, z}, {x, y, -z}};
    for (int k = 0; k < 3; k++) {
      matvec3r(endvert[k], mat, p[k][0], p[k][1], p[k][2]);
      for (int i = 0; i < 3; i++) { endvert[k][i] += pos[i]; nout[k][i] = endvert[k][i] - v1[i]; }
      normalize3(nout[k]);
    }
    return 3;
  }
  return 0;
}

/* collision_gjk.py:1722-1762 */
static int box_face(const real* mat, const real* pos, const real* s, int idx, real fo[][3]) {
  static const real SG[6][4][3] = {
    {{1, 1, 1}, {1, 1, -1}, {1, -1, -1}, {1, -1, 1}},   {{-1, 1, -1}, {-1, 1, 1}, {-1, -1, 1}, {-1, -1, -1}},
    {{-1, 1, -1}, {1, 1, -1}, {1, 1, 1}, {-1, 1, 1}},   {{-1, -1, 1}, {1, -1, 1}, {1, -1, -1}, {-1, -1, -1}},
    {{-1, 1, 1}, {1, 1, 1}, {1, -1, 1}, {-1, -1, 1}},   {{1, 1, -1}, {-1, 1, -1}, {-1, -1, -1}, {1, -1, -1}}};
  if (idx < 0 || idx > 5) return 0;
  for (int k = 0; k < 4; k++) {
    matvec3r(fo[k], mat, SG[idx][k][0] * s[0], SG[idx][k][1] * s[1], SG[idx][k][2] * s[2]);
    for (int i = 0; i < 3; i++) fo[k][i] += pos[i];
  }
  return 4;
}

/* test hook (tests/test_multiccd.py): when set, every clipped polygon of more than 4 vertices that
   polygon_quad searches is appended to the log as (np, the quad it kept, np x 3 coordinates), ORC_POLYLOG_STRIDE
   reals per record, so that a test can enumerate the quads the greedy search reaches when near-equal areas
   compare either way.  Single-threaded callers only. */
#define ORC_POLYLOG_STRIDE (5 + 3 * 2 * CCD_MAXPOLY)
static real* g_polylog = NULL;
static int g_polylog_cap = 0, g_polylog_n = 0;
void orc_polylog(real* buf, int cap) {
  g_polylog = buf;
  g_polylog_cap = cap;
  g_polylog_n = 0;
}
int orc_polylog_count(void) { return g_polylog_n; }
int orc_polylog_stride(void) { return ORC_POLYLOG_STRIDE; }

/* collision_gjk.py:1815-1909 */
static int polygon_clip(real face1[][3], int nface1, real face2[][3], int nface2, const real* n, const real* dir, real w1[4][3],
                        real w2[4][3]) {
  if (nface1 < 3) return 0;
  static real pn[CCD_MAXPOLY][3], pd[CCD_MAXPOLY], bufA[2 * CCD_MAXPOLY][3], bufB[2 * CCD_MAXPOLY][3];
#ifdef _OPENMP
#pragma omp threadprivate(pn, pd, bufA, bufB)
#endif
  real(*poly)[3] = bufA;
  real(*clip)[3] = bufB;
  for (int i = 0; i < nface1; i++) {
    const real* v1 = face1[i];
    const real* v2 = face1[(i + 1) % nface1];
    real v3[3], a[3], b[3];
    for (int k = 0; k < 3; k++) { v3[k] = v1[k] + n[k]; a[k] = v2[k] - v1[k]; b[k] = v3[k] - v1[k]; }
    cross3(pn[i], a, b);
    pd[i] = dot3(pn[i], v1);
  }
  int np = nface2, nc = 0;
  for (int i = 0; i < nface2; i++) memcpy(poly[i], face2[i], 3 * sizeof(real));
  for (int e = 0; e < nface1; e++) {
    for (int i = 0; i < np; i++) {
      const real* P = poly[i];
      const real* Q = poly[(i + 1) % np];
      real dP[3], dQ[3];
      for (int k = 0; k < 3; k++) { dP[k] = P[k] - face1[e][k]; dQ[k] = Q[k] - face1[e][k]; }
      int in1 = dot3(dP, pn[e]) > -1e-10, in2 = dot3(dQ, pn[e]) > -1e-10;
      if (!in1 && !in2) continue;
      if (nc >= 2 * CCD_MAXPOLY - 2) break;
      if (in1 && in2) { memcpy(clip[nc++], Q, 3 * sizeof(real)); continue; }
      real PQ[3] = {Q[0] - P[0], Q[1] - P[1], Q[2] - P[2]};
      real dt = dot3(pn[e], PQ);
      real t = fabs(dt) < 1e-10 ? CCD_FLOAT_MAX : (pd[e] - dot3(pn[e], P)) / dt;
      if (t > -CCD_INTERSECT_TOL && t < 1 + CCD_INTERSECT_TOL) {
        t = clampr(t, 0, 1);
        for (int k = 0; k < 3; k++) clip[nc][k] = P[k] + t * PQ[k];
        nc++;
      }
      if (in2) memcpy(clip[nc++], Q, 3 * sizeof(real));
    }
    real(*tmp)[3] = poly;
    poly = clip;
    clip = tmp;
    np = nc;
    nc = 0;
  }
  if (np < 1) return 0;
  if (np > 4) {
    int q[4];
    polygon_quad(q, poly, np);
    if (g_polylog && g_polylog_n < g_polylog_cap) {
      real* rec = g_polylog + (long)ORC_POLYLOG_STRIDE * g_polylog_n++;
      rec[0] = (real)np;
      for (int i = 0; i < 4; i++) rec[1 + i] = (real)q[i];
      for (int i = 0; i < np; i++)
        for (int k = 0; k < 3; k++) rec[5 + 3 * i + k] = poly[i][k];
    }
    for (int i = 0; i < 4; i++)
      for (int k = 0; k < 3; k++) { w2[i][k] = poly[q[i]][k]; w1[i][k] = w2[i][k] - dir[k]; }
    return 4;
  }
  for (int i = 0; i < np; i++)
    for (int k = 0; k < 3; k++) { w2[i][k] = poly[i][k]; w1[i][k] = w2[i][k] - dir[k]; }
  return np;
}

/* collision_gjk.py:1427-1456 _intersect1 / _intersect2: up to two common entries, in a1's order */
static int mesh_intersect(const int* a1, int n1, const int* a2, int n2, int* res) {
  int count = 0;
  for (int i = 0; i < n1; i++)
    for (int j = 0; j < n2; j++)
      if (a1[i] == a2[j]) {
        res[count++] = a1[i];
        if (count == 2) return 2;
      }
  return count;
}

/* collision_gjk.py:1460-1527 _mesh_normals: the polygon normals a feature of up to 3 mesh vertices can lie on */
static int mesh_normals(int dim, const int* fi, const ccd_geom* g, real nout[][3], int* iout) {
  const int* mp = g->pmap;
  const int v1 = fi[0], v2 = fi[1], v3 = fi[2];
  int edge[2], face[2], n;
  if (dim == 3) {
    n = mesh_intersect(mp + g->pmapadr[v1], g->pmapnum[v1], mp + g->pmapadr[v2], g->pmapnum[v2], edge);
    if (n == 0) return 0;
    n = mesh_intersect(edge, n, mp + g->pmapadr[v3], g->pmapnum[v3], face);
    if (n == 0) return 0;
    const real* pn = g->pnormal + 3 * face[0];
    matvec3r(nout[0], g->rot, pn[0], pn[1], pn[2]);
    iout[0] = face[0];
    return 1;
  }
  if (dim == 2) {
    n = mesh_intersect(mp + g->pmapadr[v1], g->pmapnum[v1], mp + g->pmapadr[v2], g->pmapnum[v2], edge);
    for (int i = 0; i < n; i++) {
      const real* pn = g->pnormal + 3 * edge[i];
      matvec3r(nout[i], g->rot, pn[0], pn[1], pn[2]);
      iout[i] = edge[i];
    }
    return n;
  }
  if (dim == 1) {
    const int num = g->pmapnum[v1];
    for (int i = 0; i < num && i < CCD_MAXDEG; i++) {
      const int idx = mp[g->pmapadr[v1] + i];
      const real* pn = g->pnormal + 3 * idx;
      matvec3r(nout[i], g->rot, pn[0], pn[1], pn[2]);
      iout[i] = idx;
    }
    return num;
  }
  return 0;
}

/* collision_gjk.py:1530-1574 _mesh_edge_normals: directions of the edges along a feature's vertex v1 */
static int mesh_edge_normals(int dim, const ccd_geom* g, const real* v1, const real* v2, int v1i, real nout[][3], real endvert[][3]) {
  if (dim == 2) {
    memcpy(endvert[0], v2, 3 * sizeof(real));
    real t[3] = {v2[0] - v1[0], v2[1] - v1[1], v2[2] - v1[2]};
    normalize3(t);
    memcpy(nout[0], t, sizeof(t));
    return 1;
  }
  if (dim == 1) {
    const int num = g->pmapnum[v1i];
    for (int i = 0; i < num && i < CCD_MAXDEG; i++) {
      const int idx = g->pmap[g->pmapadr[v1i] + i];
      const int adr = g->pvadr[idx], nv = g->pvnum[idx];
      for (int j = 0; j < nv; j++) {
        if (g->pvert[adr + j] != v1i) continue;
        const int k = j == 0 ? nv - 1 : j - 1;
        const real* vk = g->vert + 3 * g->pvert[adr + k];
        matvec3r(endvert[i], g->rot, vk[0], vk[1], vk[2]);
        for (int c = 0; c < 3; c++) endvert[i][c] += g->pos[c];
        real t[3] = {endvert[i][0] - v1[0], endvert[i][1] - v1[1], endvert[i][2] - v1[2]};
        normalize3(t);
        memcpy(nout[i], t, sizeof(t));
      }
    }
    return num;
  }
  return 0;
}

/* collision_gjk.py:1765-1787 _mesh_face: polygon idx in world coordinates, its loop reversed */
static int mesh_face(const ccd_geom* g, int idx, real fo[][3]) {
  const int adr = g->pvadr[idx], nv = g->pvnum[idx];
  int j = 0;
  for (int i = nv - 1; i >= 0; i--, j++) {
    const real* v = g->vert + 3 * g->pvert[adr + i];
    matvec3r(fo[j], g->rot, v[0], v[1], v[2]);
    for (int c = 0; c < 3; c++) fo[j][c] += g->pos[c];
  }
  return nv;
}

/* collision_gjk.py:1929-2150 multicontact (boxes and meshes with polygon data) */
static int multicontact(const polytope* pt, int fidx, const real* x1, const real* x2, const ccd_geom* g1, const ccd_geom* g2,
                        real w1[4][3], real w2[4][3]) {
  memcpy(w1[0], x1, 3 * sizeof(real));
  memcpy(w2[0], x2, 3 * sizeof(real));
  int face[3];
  face_verts(pt->face[fidx], face);
  int fi1[3], fi2[3];
  real fv1[3][3], fv2[3][3];
  int nface1 = feature_dim(face, pt, 0, fi1, fv1);
  int nface2 = feature_dim(face, pt, 1, fi2, fv2);
  real dir[3] = {x2[0] - x1[0], x2[1] - x1[1], x2[2] - x1[2]}, dneg[3] = {-dir[0], -dir[1], -dir[2]};
  static real n1[CCD_MAXDEG][3], n2[CCD_MAXDEG][3], endvert[CCD_MAXDEG][3], f1[CCD_MAXPOLY][3], f2[CCD_MAXPOLY][3];
  static int idx1[CCD_MAXDEG], idx2[CCD_MAXDEG];
#ifdef _OPENMP
#pragma omp threadprivate(n1, n2, endvert, f1, f2, idx1, idx2)
#endif
  int nn1 = g1->type == GEOM_BOX ? box_normals(nface1, fi1, g1->rot, dneg, n1, idx1) : mesh_normals(nface1, fi1, g1, n1, idx1);
  int nn2 = g2->type == GEOM_BOX ? box_normals(nface2, fi2, g2->rot, dir, n2, idx2) : mesh_normals(nface2, fi2, g2, n2, idx2);
  int edge1 = 0, edge2 = 0, ri = 0, rj = 0, found = 0;
  for (int i = 0; i < nn1 && !found; i++)
    for (int j = 0; j < nn2; j++)
      if (dot3(n1[i], n2[j]) < -ccd_face_tol()) { ri = i; rj = j; found = 1; break; }
  if (!found) {
    if (nface1 < 3 && nface1 <= nface2) {
      nn1 = g1->type == GEOM_BOX ? box_edge_normals(nface1, g1->rot, g1->pos, g1->size, fv1[0], fv1[1], fi1[0], n1, endvert)
                                 : mesh_edge_normals(nface1, g1, fv1[0], fv1[1], fi1[0], n1, endvert);
      for (int i = 0; i < nn2 && !found; i++) /* _aligned_face_edge(n1 edges, n2 faces) */
        for (int j = 0; j < nn1; j++)
          if (fabs(dot3(n1[j], n2[i])) < ccd_edge_tol()) { ri = j; rj = i; found = 1; break; }
      if (!found) return 1;
      edge1 = 1;
    } else if (nface2 < 3) {
      nn2 = g2->type == GEOM_BOX ? box_edge_normals(nface2, g2->rot, g2->pos, g2->size, fv2[0], fv2[1], fi2[0], n2, endvert)
                                 : mesh_edge_normals(nface2, g2, fv2[0], fv2[1], fi2[0], n2, endvert);
      for (int i = 0; i < nn1 && !found; i++) /* _aligned_face_edge(n2 edges, n1 faces) */
        for (int j = 0; j < nn2; j++)
          if (fabs(dot3(n2[j], n1[i])) < ccd_edge_tol()) { ri = j; rj = i; found = 1; break; }
      if (!found) return 1;
      edge2 = 1;
    } else {
      return 1;
    }
  }
  int nf1, nf2;
  if (edge1) {
    memcpy(f1[0], pt->vert[2 * face[0]], 3 * sizeof(real));
    memcpy(f1[1], endvert[ri], 3 * sizeof(real));
    nf1 = 2;
  } else {
    const int ind = edge2 ? idx1[rj] : idx1[ri];
    nf1 = g1->type == GEOM_BOX ? box_face(g1->rot, g1->pos, g1->size, ind, f1) : mesh_face(g1, ind, f1);
  }
  if (edge2) {
    memcpy(f2[0], pt->vert[2 * face[0] + 1], 3 * sizeof(real));
    memcpy(f2[1], endvert[ri], 3 * sizeof(real));
    nf2 = 2;
  } else {
    nf2 = g2->type == GEOM_BOX ? box_face(g2->rot, g2->pos, g2->size, idx2[rj], f2) : mesh_face(g2, idx2[rj], f2);
  }
  real dl = sqrt(dot3(dir, dir)), ad[3];
  if (edge1) {
    for (int i = 0; i < 3; i++) ad[i] = dl * n2[rj][i];
    return polygon_clip(f2, nf2, f1, nf1, n2[rj], ad, w1, w2);
  }
  if (edge2) {
    for (int i = 0; i < 3; i++) ad[i] = -dl * n1[rj][i];
    return polygon_clip(f1, nf1, f2, nf2, n1[rj], ad, w1, w2);
  }
  for (int i = 0; i < 3; i++) ad[i] = dl * n2[rj][i];
  return polygon_clip(f1, nf1, f2, nf2, n1[ri], ad, w1, w2);
}

/* collision_gjk.py:2200-2345 ccd: distance (or penetration depth) of one convex pair and its first
 * witness points.  Returns the reference's ncon (1, or 0 when EPA fails with FLOAT_MAX); *idx is the
 * EPA face for box multi-contact (-1 otherwise); the polytope stays in `pt` for multicontact_box.
 * Geoms carry their margin (the caller sets it, collision_convex.py:770-771). */
static int ccd_raw(const ccd_geom* g1in, const ccd_geom* g2in, real tolerance, real cutoff, int gjk_iter, int epa_iter, polytope* pt,
                   real* dist, real* x1, real* x2, int* idx, ccd_geom* g1out, ccd_geom* g2out) {
  ccd_geom g1 = *g1in, g2 = *g2in;
  *idx = -1;
  /* collision_gjk.py:91-94, 2226: boxes and meshes are discrete */
  int discrete = (g1.type == GEOM_BOX || g1.type == GEOM_MESH || g1.type == GEOM_HFIELD) &&
                 (g2.type == GEOM_BOX || g2.type == GEOM_MESH || g2.type == GEOM_HFIELD) && g1.margin == 0 && g2.margin == 0;
  real full1 = 0, full2 = 0, size1 = 0, size2 = 0;
  if (g1.type == GEOM_SPHERE || g1.type == GEOM_CAPSULE) {
    size1 = g1.size[0]; full1 = size1 + 0.5 * g1.margin; g1.margin = 0; g1.size[0] = 0;
  }
  if (g2.type == GEOM_SPHERE || g2.type == GEOM_CAPSULE) {
    size2 = g2.size[0]; full2 = size2 + 0.5 * g2.margin; g2.margin = 0; g2.size[0] = 0;
  }
  *g1out = g1;
  *g2out = g2;
  gjk_result r;
  if (size1 + size2 > 0) {
    cutoff += full1 + full2;
    r = gjk(tolerance, gjk_iter, &g1, &g2, g1.pos, g2.pos, cutoff, discrete);
    if (r.dist > tolerance) { /* shallow penetration: inflate (collision_gjk.py:194-213 _inflate) */
      if (r.dist == CCD_FLOAT_MAX) {
        *dist = r.dist;
        memcpy(x1, r.x1, 3 * sizeof(real));
        memcpy(x2, r.x2, 3 * sizeof(real));
        return 1;
      }
      if (g1.type == GEOM_HFIELD) { /* collision_gjk.py:2160-2187: a simplex touching the prism's top and bottom */
        int side = 0;
        for (int i = 1; i < r.dim; i++) side |= r.index1[i] != r.index1[0];
        if (side) {
          ccd_sp sp = ccd_support(&g2, r.x2); /* geom2 still shrunk to its point / segment */
          memcpy(x2, sp.point, 3 * sizeof(real));
          x2[2] -= full2;
          *dist = hfield_top_witness(&g1, x2, x1);
          return 1;
        }
      }
      real n[3] = {r.x2[0] - r.x1[0], r.x2[1] - r.x1[1], r.x2[2] - r.x1[2]};
      normalize3(n);
      for (int i = 0; i < 3; i++) { x1[i] = r.x1[i] + (full1 > 0 ? full1 * n[i] : 0); x2[i] = r.x2[i] - (full2 > 0 ? full2 * n[i] : 0); }
      *dist = r.dist - (full1 + full2);
      return 1;
    }
    g1.margin = full1 - size1; g1.size[0] = size1;
    g2.margin = full2 - size2; g2.size[0] = size2;
    cutoff -= full1 + full2;
  }
  *g1out = g1;
  *g2out = g2;
  r = gjk(tolerance, gjk_iter, &g1, &g2, g1.pos, g2.pos, cutoff, discrete);
  *dist = r.dist;
  memcpy(x1, r.x1, 3 * sizeof(real));
  memcpy(x2, r.x2, 3 * sizeof(real));
  if (r.dist > tolerance || r.dim < 2) return 1;
  memset(pt, 0, sizeof(*pt));
  pt->cap_vert = 10 + 2 * epa_iter;
  pt->cap_face = 6 + CCD_MAX_EPAFACES * epa_iter;
  int status;
  if (r.dim == 2) {
    status = polytope2(pt, &r, &g1, &g2);
    if (status == -1) status = polytope3(pt, r.dist, &r, &g1, &g2);
  } else if (r.dim == 4) {
    status = polytope4(pt, &r);
    if (status == -1) status = polytope3(pt, r.dist, &r, &g1, &g2);
  } else {
    status = polytope3(pt, r.dist, &r, &g1, &g2);
  }
  if (status) return 1; /* origin on the boundary: not penetrating */
  int f = epa(tolerance, epa_iter, pt, &g1, &g2, discrete, dist, x1, x2);
  if (f == -1) {
    *dist = CCD_FLOAT_MAX;
    for (int i = 0; i < 3; i++) x1[i] = x2[i] = 0;
    return 0;
  }
  /* collision_gjk.py:2336-2345: multicontact needs no margin and boxes or meshes (with polygon data,
   * collision_convex.py:810-818); the caller applies MULTICCD (box-box always, collision_convex.py:809) */
  if (g1.margin != 0 || g2.margin != 0) f = -1;
  if (!((g1.type == GEOM_BOX || g1.type == GEOM_MESH) && (g2.type == GEOM_BOX || g2.type == GEOM_MESH))) f = -1;
  if ((g1.type == GEOM_MESH && !g1.pnormal) || (g2.type == GEOM_MESH && !g2.pnormal)) f = -1;
  *idx = f;
  return 1;
}

/* MULTICCD of the model being collided (opt.enableflags), set by the caller around ccd_pair */
static int ccd_multiccd = 0;
#ifdef _OPENMP
#pragma omp threadprivate(ccd_multiccd)
#endif

static polytope* ccd_polytope(void) {
  static polytope pt_store;
#ifdef _OPENMP
#pragma omp threadprivate(pt_store)
#endif
  return &pt_store;
}

/* collision_convex.py:763-852 (eval_ccd_write_contact): contacts of one convex pair.  Returns the number
 * of contacts (0 when not penetrating), all at distance *dist (already corrected by +margin) with normal
 * `normal` (unnormalized; the frame is make_frame(normal)). */
static int ccd_pair_cut(const ccd_geom* g1in, const ccd_geom* g2in, real tolerance, int gjk_iter, int epa_iter, real margin,
                        real cutoff, real* dist_out, real* normal, real pts[4][3]);
static int ccd_pair(const ccd_geom* g1in, const ccd_geom* g2in, real tolerance, int gjk_iter, int epa_iter, real margin,
                    real* dist_out, real* normal, real pts[4][3]) {
  return ccd_pair_cut(g1in, g2in, tolerance, gjk_iter, epa_iter, margin, 0, dist_out, normal, pts);
}

/* cutoff > 0: collision sensors (collision_convex.py:772-776, cutoff 1e32), separated pairs reported too */
static int ccd_pair_cut(const ccd_geom* g1in, const ccd_geom* g2in, real tolerance, int gjk_iter, int epa_iter, real margin,
                        real cutoff, real* dist_out, real* normal, real pts[4][3]) {
  polytope* pt = ccd_polytope();
  ccd_geom g1 = *g1in, g2 = *g2in, h1, h2;
  g1.margin = margin;
  g2.margin = margin;
  real d, x1[3], x2[3];
  int idx;
  if (!ccd_raw(&g1, &g2, tolerance, cutoff, gjk_iter, epa_iter, pt, &d, x1, x2, &idx, &h1, &h2)) return 0;
  if (d >= 0 && cutoff == 0) return 0;
  d += margin;
  *dist_out = d;
  real w1[4][3], w2[4][3];
  int n = 1;
  memcpy(w1[0], x1, sizeof(x1));
  memcpy(w2[0], x2, sizeof(x2));
  /* collision_convex.py:809: box-box always, box-mesh / mesh-mesh under MULTICCD (g*->multiccd) */
  const int boxbox = g1.type == GEOM_BOX && g2.type == GEOM_BOX;
  if (idx > -1 && (boxbox || ccd_multiccd)) n = multicontact(pt, idx, x1, x2, &h1, &h2, w1, w2);
  for (int i = 0; i < n; i++)
    for (int k = 0; k < 3; k++) pts[i][k] = 0.5 * (w1[i][k] + w2[i][k]);
  for (int k = 0; k < 3; k++) normal[k] = w1[0][k] - w2[0][k];
  return n;
}

/* ---- heightfields: collision_convex.py:55-154 _hfield_filter and 158-697 ccd_hfield_kernel ----
 * One heightfield (g1, frame hpos / hmat) against a convex geom2 (world frame).  Every triangular prism
 * of the grid cells under geom2's bounds goes through ccd() (cached: distance, world position, world
 * normal); then contact 0 = the minimum distance, 1 = the farthest from it, 2 = the farthest from their
 * line, 3 = the farthest from the triangle's other edges (each only while the previous one exists and lies
 * at least 1e-3 away).  Returns the number of points written to dist / pos / nrm. */
#define HF_MAXCON 50 /* mjMAXCONPAIR */
static int hfield_pair(const real* hpos, const real* hmat, const real* hsize, int nrow, int ncol, const real* hdata,
                       const ccd_geom* g2w, real grbound, real fmargin, real margin, real tolerance, int gjk_iter, int epa_iter,
                       real dist[4], real pos[4][3], real nrm[4][3]) {
  real dp[3] = {g2w->pos[0] - hpos[0], g2w->pos[1] - hpos[1], g2w->pos[2] - hpos[2]}, lp[3];
  for (int i = 0; i < 3; i++) lp[i] = hmat[i] * dp[0] + hmat[3 + i] * dp[1] + hmat[6 + i] * dp[2];
  for (int i = 0; i < 2; i++)
    if (hsize[i] < lp[i] - grbound - fmargin || -hsize[i] > lp[i] + grbound + fmargin) return 0;
  if (hsize[2] < lp[2] - grbound - fmargin) return 0;
  if (-hsize[3] > lp[2] + grbound + fmargin) return 0;
  ccd_geom g2 = *g2w;
  memcpy(g2.pos, lp, sizeof(lp));
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) g2.rot[3 * i + j] = hmat[i] * g2w->rot[j] + hmat[3 + i] * g2w->rot[3 + j] + hmat[6 + i] * g2w->rot[6 + j];
  g2.margin = 0;
  real ext[6];
  for (int k = 0; k < 6; k++) {
    real dir[3] = {0, 0, 0};
    dir[k >> 1] = (k & 1) ? -1 : 1;
    ext[k] = ccd_support(&g2, dir).point[k >> 1];
  }
  real xmax = ext[0], xmin = ext[1], ymax = ext[2], ymin = ext[3], zmax = ext[4], zmin = ext[5];
  if (xmin - fmargin > hsize[0] || xmax + fmargin < -hsize[0] || ymin - fmargin > hsize[1] || ymax + fmargin < -hsize[1] ||
      zmin - fmargin > hsize[2] || zmax + fmargin < -hsize[3])
    return 0;
  real x_scale = 0.5 * (real)(ncol - 1) / hsize[0], y_scale = 0.5 * (real)(nrow - 1) / hsize[1];
  int cmin = (int)floor((xmin + hsize[0]) * x_scale), cmax = (int)ceil((xmax + hsize[0]) * x_scale);
  int rmin = (int)floor((ymin + hsize[1]) * y_scale), rmax = (int)ceil((ymax + hsize[1]) * y_scale);
  if (cmin < 0) cmin = 0;
  if (cmax > ncol - 1) cmax = ncol - 1;
  if (rmin < 0) rmin = 0;
  if (rmax > nrow - 1) rmax = nrow - 1;
  real dx = (2 * hsize[0]) / (real)(ncol - 1), dy = (2 * hsize[1]) / (real)(nrow - 1);
  real prism[6][3];
  memset(prism, 0, sizeof(prism));
  for (int i = 0; i < 3; i++) prism[i][2] = -hsize[3];
  g2.margin = margin;
  ccd_geom g1;
  memset(&g1, 0, sizeof(g1));
  for (int i = 0; i < 3; i++) g1.rot[4 * i] = 1;
  g1.type = GEOM_HFIELD;
  g1.prism = &prism[0][0];
  real cd[HF_MAXCON], cp[HF_MAXCON][3], cn[HF_MAXCON][3];
  int count = 0, min_id = -1;
  real min_dist = 1e10; /* MJ_MAXVAL */
  polytope* pt = ccd_polytope();
  for (int r = rmin; r < rmax; r++) {
    for (int c = cmin; c <= cmax; c++) {
      for (int i = 0; i < 2; i++) {
        if (c > cmin && count >= HF_MAXCON) continue; /* overflow: the reference drops the prism */
        memmove(prism[0], prism[1], 2 * sizeof(prism[0]));
        memmove(prism[3], prism[4], 2 * sizeof(prism[0]));
        real x = dx * (real)c - hsize[0], y = dy * (real)(r + i) - hsize[1];
        prism[2][0] = prism[5][0] = x;
        prism[2][1] = prism[5][1] = y;
        prism[5][2] = hdata[(r + i) * ncol + c] * hsize[2] + margin;
        if (c == cmin) continue; /* the first column only seeds the prism */
        if (prism[3][2] < zmin && prism[4][2] < zmin && prism[5][2] < zmin) continue;
        for (int k = 0; k < 3; k++)
          g1.pos[k] = (prism[0][k] + prism[1][k] + prism[2][k] + prism[3][k] + prism[4][k] + prism[5][k]) * (1.0 / 6.0);
        real d, x1[3], x2[3];
        int idx;
        ccd_geom h1, h2;
        if (!ccd_raw(&g1, &g2, tolerance, 0, gjk_iter, epa_iter, pt, &d, x1, x2, &idx, &h1, &h2)) continue;
        real pl[3] = {0.5 * (x1[0] + x2[0]), 0.5 * (x1[1] + x2[1]), 0.5 * (x1[2] + x2[2])};
        real nl[3] = {x1[0] - x2[0], x1[1] - x2[1], x1[2] - x2[2]};
        normalize3(nl);
        cd[count] = d;
        for (int k = 0; k < 3; k++) {
          cp[count][k] = hmat[3 * k] * pl[0] + hmat[3 * k + 1] * pl[1] + hmat[3 * k + 2] * pl[2] + hpos[k];
          cn[count][k] = hmat[3 * k] * nl[0] + hmat[3 * k + 1] * nl[1] + hmat[3 * k + 2] * nl[2];
        }
        if (d < min_dist) { min_dist = d; min_id = count; }
        count++;
      }
    }
  }
  real mpos[3] = {1e10, 1e10, 1e10}, mnrm[3] = {1e10, 1e10, 1e10};
  if (min_id >= 0) { memcpy(mpos, cp[min_id], sizeof(mpos)); memcpy(mnrm, cn[min_id], sizeof(mnrm)); }
  int n = 0;
  dist[n] = min_dist; memcpy(pos[n], mpos, sizeof(mpos)); memcpy(nrm[n], mnrm, sizeof(mnrm)); n++;
  const real min_next = 1.0e-3;
  int id1 = -1;
  real dist1 = -1e10;
  for (int i = 0; i < count; i++) {
    if (i == min_id) continue;
    real t[3] = {cp[i][0] - mpos[0], cp[i][1] - mpos[1], cp[i][2] - mpos[2]};
    real dd = sqrt(dot3(t, t));
    if (dd > dist1) { id1 = i; dist1 = dd; }
  }
  if (id1 == -1 || (0 < dist1 && dist1 < min_next)) return n;
  dist[n] = cd[id1]; memcpy(pos[n], cp[id1], sizeof(mpos)); memcpy(nrm[n], cn[id1], sizeof(mnrm)); n++;
  real t1[3] = {mpos[0] - cp[id1][0], mpos[1] - cp[id1][1], mpos[2] - cp[id1][2]}, dmin1[3];
  cross3(dmin1, mnrm, t1);
  int id2 = -1;
  real dist12 = -1e10;
  for (int i = 0; i < count; i++) {
    if (i == min_id || i == id1) continue;
    real u[3] = {cp[i][0] - mpos[0], cp[i][1] - mpos[1], cp[i][2] - mpos[2]};
    real dd = fabs(dot3(u, dmin1));
    if (dd > dist12) { id2 = i; dist12 = dd; }
  }
  if (id2 == -1 || (0 < dist12 && dist12 < min_next)) return n;
  dist[n] = cd[id2]; memcpy(pos[n], cp[id2], sizeof(mpos)); memcpy(nrm[n], cn[id2], sizeof(mnrm)); n++;
  real a0[3] = {mpos[0] - cp[id2][0], mpos[1] - cp[id2][1], mpos[2] - cp[id2][2]};
  real a1[3] = {cp[id1][0] - cp[id2][0], cp[id1][1] - cp[id2][1], cp[id1][2] - cp[id2][2]}, vmin2[3], v12[3];
  cross3(vmin2, mnrm, a0);
  cross3(v12, mnrm, a1);
  int id3 = -1;
  real dist3 = -1e10;
  for (int i = 0; i < count; i++) {
    if (i == min_id || i == id1 || i == id2) continue;
    real u[3] = {cp[i][0] - mpos[0], cp[i][1] - mpos[1], cp[i][2] - mpos[2]};
    real v[3] = {cp[id1][0] - cp[i][0], cp[id1][1] - cp[i][1], cp[id1][2] - cp[i][2]};
    real dd = fabs(dot3(u, vmin2)) + fabs(dot3(v, v12));
    if (dd > dist3) { id3 = i; dist3 = dd; }
  }
  if (id3 == -1 || (0 < dist3 && dist3 < min_next)) return n;
  dist[n] = cd[id3]; memcpy(pos[n], cp[id3], sizeof(mpos)); memcpy(nrm[n], cn[id3], sizeof(mnrm)); n++;
  return n;
}
