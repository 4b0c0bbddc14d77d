/* Spatial tendons for the CPU oracle (test infrastructure only -- never the product path).
 *
 * Restates the reference's tendon wrapping geometry (util_misc.py:30-450: is_intersect, length_circle,
 * wrap_circle, wrap_inside, wrap) and the spatial tendon length / Jacobian (smooth.py:3172-3465: site-site
 * segments, site-geom-site wraps, pulley scaling io.py:491-497) and its time derivative for the armature
 * bias (smooth.py:1590-1932).  Included by oracle.c after its vector helpers. */

#define WRAP_JOINT 1
#define WRAP_PULLEY 2
#define WRAP_SITE 3
#define WRAP_SPHERE 4
#define WRAP_CYLINDER 5

/* util_misc.py:30-56 */
static int wrap_is_intersect(const real* p1, const real* p2, const real* p3, const real* p4) {
  real det = (p4[1] - p3[1]) * (p2[0] - p1[0]) - (p4[0] - p3[0]) * (p2[1] - p1[1]);
  if (fabs(det) < MINVAL) return 0;
  real a = ((p4[0] - p3[0]) * (p1[1] - p3[1]) - (p4[1] - p3[1]) * (p1[0] - p3[0])) / det;
  real b = ((p2[0] - p1[0]) * (p1[1] - p3[1]) - (p2[1] - p1[1]) * (p1[0] - p3[0])) / det;
  return a >= 0 && a <= 1 && b >= 0 && b <= 1;
}

static real norm2d(const real* v) { return sqrt(v[0] * v[0] + v[1] * v[1]); }

/* util_misc.py:76-100 */
static real wrap_length_circle(const real* p0, const real* p1, int ind, real radius) {
  real n0 = norm2d(p0), n1 = norm2d(p1);
  real a0[2] = {0, 0}, a1[2] = {0, 0};
  if (n0 > 0) { a0[0] = p0[0] / n0; a0[1] = p0[1] / n0; }
  if (n1 > 0) { a1[0] = p1[0] / n1; a1[1] = p1[1] / n1; }
  real angle = acos(clampr(a0[0] * a1[0] + a0[1] * a1[1], -1, 1));
  real cross = p0[1] * p1[0] - p0[0] * p1[1];
  if ((cross > 0 && ind != 0) || (cross < 0 && ind == 0)) angle = 2 * M_PI - angle;
  return radius * angle;
}

/* util_misc.py:103-198: returns the arc length or -1, tangent points in q0 / q1 */
static real wrap_circle(const real* end, const real* side, real radius, real* q0, real* q1) {
  const int valid_side = norm2d(side) < MAXVAL;
  const real sq0 = end[0] * end[0] + end[1] * end[1], sq1 = end[2] * end[2] + end[3] * end[3], sqr = radius * radius;
  q0[0] = q0[1] = q1[0] = q1[1] = MAXVAL;
  if (sq0 < sqr || sq1 < sqr || radius < MINVAL) return -1;
  real dif[2] = {end[2] - end[0], end[3] - end[1]};
  real dd = dif[0] * dif[0] + dif[1] * dif[1];
  if (dd < MINVAL) return -1;
  real a = clampr(-(dif[0] * end[0] + dif[1] * end[1]) / dd, 0, 1);
  real tmp[2] = {a * dif[0] + end[0], a * dif[1] + end[1]};
  if (tmp[0] * tmp[0] + tmp[1] * tmp[1] > sqr && (!valid_side || side[0] * tmp[0] + side[1] * tmp[1] >= 0)) return -1;
  real s0 = sqrt(sq0 - sqr), s1 = sqrt(sq1 - sqr);
  real sol00[2] = {safe_div(end[0] * sqr + radius * end[1] * s0, sq0), safe_div(end[1] * sqr - radius * end[0] * s0, sq0)};
  real sol01[2] = {safe_div(end[2] * sqr - radius * end[3] * s1, sq1), safe_div(end[3] * sqr + radius * end[2] * s1, sq1)};
  real sol10[2] = {safe_div(end[0] * sqr - radius * end[1] * s0, sq0), safe_div(end[1] * sqr + radius * end[0] * s0, sq0)};
  real sol11[2] = {safe_div(end[2] * sqr + radius * end[3] * s1, sq1), safe_div(end[3] * sqr - radius * end[2] * s1, sq1)};
  real good0, good1;
  if (valid_side) {
    real m0[2] = {sol00[0] + sol01[0], sol00[1] + sol01[1]}, m1[2] = {sol10[0] + sol11[0], sol10[1] + sol11[1]};
    real n0 = norm2d(m0), n1 = norm2d(m1);
    good0 = n0 > 0 ? (m0[0] * side[0] + m0[1] * side[1]) / n0 : 0;
    good1 = n1 > 0 ? (m1[0] * side[0] + m1[1] * side[1]) / n1 : 0;
  } else {
    real d0[2] = {sol00[0] - sol01[0], sol00[1] - sol01[1]}, d1[2] = {sol10[0] - sol11[0], sol10[1] - sol11[1]};
    good0 = -(d0[0] * d0[0] + d0[1] * d0[1]);
    good1 = -(d1[0] * d1[0] + d1[1] * d1[1]);
  }
  const real e0[2] = {end[0], end[1]}, e1[2] = {end[2], end[3]};
  if (wrap_is_intersect(e0, sol00, e1, sol01)) good0 = -10000;
  if (wrap_is_intersect(e0, sol10, e1, sol11)) good1 = -10000;
  const real *p0, *p1;
  int ind;
  if (good0 > good1) { p0 = sol00; p1 = sol01; ind = 0; }
  else { p0 = sol10; p1 = sol11; ind = 1; }
  if (wrap_is_intersect(e0, p0, e1, p1)) return -1;
  q0[0] = p0[0]; q0[1] = p0[1]; q1[0] = p1[0]; q1[1] = p1[1];
  return wrap_length_circle(p0, p1, ind, radius);
}

/* util_misc.py:201-323: inside wrap (sidesite within the geom); one tangent point, Newton on
 * asin(A z) + asin(B z) - 2 asin(z) + G = 0 */
static real wrap_inside(const real* end, real radius, real* q0, real* q1) {
  const int maxiter = 20;
  const real zinit = 1.0 - 1.0e-7, tol = 1.0e-6;
  q0[0] = q0[1] = q1[0] = q1[1] = MAXVAL;
  const real e0[2] = {end[0], end[1]}, e1[2] = {end[2], end[3]};
  real len0 = norm2d(e0), len1 = norm2d(e1);
  real dif[2] = {e1[0] - e0[0], e1[1] - e0[1]};
  real dd = dif[0] * dif[0] + dif[1] * dif[1];
  if (len0 <= radius || len1 <= radius || radius < MINVAL || len0 < MINVAL || len1 < MINVAL) return -1;
  if (dd > MINVAL) {
    real a = -(dif[0] * e0[0] + dif[1] * e0[1]) / dd;
    real c[2] = {e0[0] + a * dif[0], e0[1] + a * dif[1]};
    if (a > 0 && a < 1 && norm2d(c) <= radius) return -1;
  }
  real mid[2] = {0.5 * (e0[0] + e1[0]), 0.5 * (e0[1] + e1[1])}, nm = norm2d(mid);
  real pnt[2] = {nm > 0 ? mid[0] / nm * radius : 0, nm > 0 ? mid[1] / nm * radius : 0};
  q0[0] = q1[0] = pnt[0];
  q0[1] = q1[1] = pnt[1];
  real A = safe_div(radius, len0), B = safe_div(radius, len1);
  real cosG = safe_div(len0 * len0 + len1 * len1 - dd, 2 * len0 * len1);
  if (cosG < -1 + MINVAL) return -1;
  if (cosG > 1 - MINVAL) return 0;
  real G = acos(cosG), z = zinit;
  real f = asin(A * z) + asin(B * z) - 2 * asin(z) + G;
  if (f > 0) return 0;
  int it = 0;
  while (it < maxiter && fabs(f) > tol) {
    real sz = z * z;
    real df = A / maxr(MINVAL, sqrt(1 - sz * A * A)) + B / maxr(MINVAL, sqrt(1 - sz * B * B)) - 2 / maxr(MINVAL, sqrt(1 - sz));
    if (df > -MINVAL) return 0;
    real z1 = z - safe_div(f, df);
    if (z1 > z) return 0;
    z = z1;
    f = asin(A * z) + asin(B * z) - 2 * asin(z) + G;
    if (f > tol) return 0;
    it++;
  }
  if (it >= maxiter) return 0;
  const real* vec;
  real ang;
  if (end[0] * end[3] - end[1] * end[2] > 0) { vec = e0; ang = asin(z) - asin(A * z); }
  else { vec = e1; ang = asin(z) - asin(B * z); }
  real nv_ = norm2d(vec), v[2] = {nv_ > 0 ? vec[0] / nv_ : 0, nv_ > 0 ? vec[1] / nv_ : 0};
  q0[0] = q1[0] = radius * (cos(ang) * v[0] - sin(ang) * v[1]);
  q0[1] = q1[1] = radius * (sin(ang) * v[0] + cos(ang) * v[1]);
  return 0;
}

/* util_misc.py:326-450: wrap segment x0-x1 around a sphere / infinite cylinder at pos / mat (row-major);
 * side = sidesite position or MAXVAL.  Returns arc length or -1, world wrap points in w0 / w1. */
static real wrap_geom(const real* x0, const real* x1, const real* pos, const real* mat, real radius, int type, const real* side,
                      real* w0, real* w1) {
  for (int i = 0; i < 3; i++) w0[i] = w1[i] = MAXVAL;
  real d0[3], d1[3], p0[3], p1[3];
  for (int i = 0; i < 3; i++) { d0[i] = x0[i] - pos[i]; d1[i] = x1[i] - pos[i]; }
  rt_vec(p0, mat, d0);
  rt_vec(p1, mat, d1);
  if (sqrt(dot3(p0, p0)) < MINVAL || sqrt(dot3(p1, p1)) < MINVAL) return -1;
  real axis0[3], axis1[3];
  if (type == WRAP_SPHERE) {
    normalize_with_norm(axis0, p0);
    real c[3], normal[3];
    cross3(c, p0, p1);
    real nrm = normalize_with_norm(normal, c);
    if (nrm < MINVAL) {
      real ab[3] = {fabs(axis0[0]), fabs(axis0[1]), fabs(axis0[2])};
      int i = 0;
      if (ab[1] > ab[0] && ab[1] > ab[2]) i = 1;
      if (ab[2] > ab[0] && ab[2] > ab[1]) i = 2;
      real a1[3] = {1, 1, 1};
      a1[i] = 0;
      cross3(c, axis0, a1);
      normalize_with_norm(normal, c);
    }
    cross3(c, normal, axis0);
    normalize_with_norm(axis1, c);
  } else {
    axis0[0] = 1; axis0[1] = 0; axis0[2] = 0;
    axis1[0] = 0; axis1[1] = 1; axis1[2] = 0;
  }
  real end[4] = {dot3(p0, axis0), dot3(p0, axis1), dot3(p1, axis0), dot3(p1, axis1)};
  const int valid_side = sqrt(dot3(side, side)) < MAXVAL;
  real sidepnt[3] = {0, 0, 0}, sproj[2] = {MAXVAL, MAXVAL};
  if (valid_side) {
    real ds[3] = {side[0] - pos[0], side[1] - pos[1], side[2] - pos[2]};
    rt_vec(sidepnt, mat, ds);
    real sp[2] = {dot3(sidepnt, axis0), dot3(sidepnt, axis1)}, n = norm2d(sp);
    sproj[0] = n > 0 ? sp[0] / n * radius : 0;
    sproj[1] = n > 0 ? sp[1] / n * radius : 0;
  }
  real q0[2], q1[2], wlen;
  if (valid_side && sqrt(dot3(sidepnt, sidepnt)) < radius) wlen = wrap_inside(end, radius, q0, q1);
  else wlen = wrap_circle(end, sproj, radius, q0, q1);
  if (wlen < 0) return -1;
  real r0[3], r1[3];
  for (int i = 0; i < 3; i++) {
    r0[i] = axis0[i] * q0[0] + axis1[i] * q0[1];
    r1[i] = axis0[i] * q1[0] + axis1[i] * q1[1];
  }
  if (type == WRAP_CYLINDER) {
    real L0 = sqrt((p0[0] - r0[0]) * (p0[0] - r0[0]) + (p0[1] - r0[1]) * (p0[1] - r0[1]));
    real L1 = sqrt((p1[0] - r1[0]) * (p1[0] - r1[0]) + (p1[1] - r1[1]) * (p1[1] - r1[1]));
    r0[2] = p0[2] + (p1[2] - p0[2]) * safe_div(L0, L0 + wlen + L1);
    r1[2] = p0[2] + (p1[2] - p0[2]) * safe_div(L0 + wlen, L0 + wlen + L1);
    wlen = sqrt(wlen * wlen + (r1[2] - r0[2]) * (r1[2] - r0[2]));
  }
  r_vec(w0, mat, r0);
  r_vec(w1, mat, r1);
  for (int i = 0; i < 3; i++) { w0[i] += pos[i]; w1[i] += pos[i]; }
  return wlen;
}

/* smooth.py:3126-3170 (_accumulate_jac_chain): J[rowadr + k] += scale vec . (cdof_lin + cdof_ang x offset)
 * for every dof k of the body chain from `body` to the root */
static void ten_jac_chain(const orc_model* m, const orc_data* d, int t, int body, const real* pnt, const real* vec, real scale) {
  const int ra = m->ten_J_rowadr[t], rn = m->ten_J_rownnz[t];
  const real* sc = d->subtree_com + 3 * m->body_rootid[body];
  real off[3] = {pnt[0] - sc[0], pnt[1] - sc[1], pnt[2] - sc[2]};
  for (int b = body; b > 0; b = m->body_parentid[b])
    for (int dof = m->body_dofadr[b]; dof < m->body_dofadr[b] + m->body_dofnum[b]; dof++) {
      const real* cd = d->cdof + 6 * dof;
      real c[3], jp[3];
      cross3(c, cd, off);
      for (int i = 0; i < 3; i++) jp[i] = cd[3 + i] + c[i];
      for (int k = 0; k < rn; k++)
        if (m->ten_J_colind[ra + k] == dof) { d->ten_J[ra + k] += scale * dot3(jp, vec); break; }
    }
}

static real ten_segment(const orc_model* m, const orc_data* d, int t, const real* p0, int b0, const real* p1, int b1, real scale) {
  real dif[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]}, vec[3];
  real len = normalize_with_norm(vec, dif);
  if (len < MINVAL) { vec[0] = 1; vec[1] = 0; vec[2] = 0; }
  if (b0 != b1) {
    ten_jac_chain(m, d, t, b0, p0, vec, -scale);
    ten_jac_chain(m, d, t, b1, p1, vec, scale);
  }
  return len;
}

static real pulley_divisor(const orc_model* m, int t, int w) {
  real s = 1;
  for (int p = m->tendon_adr[t]; p <= w; p++)
    if (m->wrap_type[p] == WRAP_PULLEY) s = 1.0 / m->wrap_prm[p];
  return s;
}

/* smooth.py:3172-3465: length and (sparse) Jacobian of spatial tendon t; ten_J row already zeroed */
static real spatial_tendon(const orc_model* m, orc_data* d, int t) {
  const int a = m->tendon_adr[t], n = m->tendon_num[t];
  real L = 0;
  int j = 0;
  while (j < n - 1) {
    const int t0 = m->wrap_type[a + j], t1 = m->wrap_type[a + j + 1];
    if (t0 == WRAP_PULLEY || t1 == WRAP_PULLEY) { j++; continue; }
    const int s0 = m->wrap_objid[a + j];
    const real* p0 = d->site_xpos + 3 * s0;
    const int b0 = m->site_bodyid[s0];
    if (t1 == WRAP_SPHERE || t1 == WRAP_CYLINDER) {
      const int g = m->wrap_objid[a + j + 1], s1 = m->wrap_objid[a + j + 2], gb = m->geom_bodyid[g];
      const real* p1 = d->site_xpos + 3 * s1;
      const int b1 = m->site_bodyid[s1];
      const real sc = pulley_divisor(m, t, a + j + 1);
      const int sid = (int)lround(m->wrap_prm[a + j + 1]);
      real side[3] = {MAXVAL, MAXVAL, MAXVAL}, g0[3], g1[3];
      if (sid >= 0) memcpy(side, d->site_xpos + 3 * sid, sizeof(side));
      real wl = wrap_geom(p0, p1, d->geom_xpos + 3 * g, d->geom_xmat + 9 * g, m->geom_size[3 * g], t1, side, g0, g1);
      if (wl >= 0) {
        real l0 = ten_segment(m, d, t, p0, b0, g0, gb, sc);
        real l1 = ten_segment(m, d, t, g1, gb, p1, b1, sc);
        L += (l0 + wl + l1) * sc;
      } else {
        L += ten_segment(m, d, t, p0, b0, p1, b1, sc) * sc;
      }
      j += 2;
    } else {
      const int s1 = m->wrap_objid[a + j + 1];
      const real sc = pulley_divisor(m, t, a + j);
      L += ten_segment(m, d, t, p0, b0, d->site_xpos + 3 * s1, m->site_bodyid[s1], sc) * sc;
      j++;
    }
  }
  return L;
}

/* smooth.py:1590-1653 (_accumulate_jac_dot_chain) */
static void ten_jacdot_chain(const orc_model* m, const orc_data* d, int t, int body, const real* off, const real* pvel, const real* dpnt,
                             const real* dvel, real scale, real* Jdot) {
  const int ra = m->ten_J_rowadr[t], rn = m->ten_J_rownnz[t];
  for (int b = body; b > 0; b = m->body_parentid[b])
    for (int dof = m->body_dofadr[b]; dof < m->body_dofadr[b] + m->body_dofnum[b]; dof++) {
      int k = 0;
      while (k < rn && m->ten_J_colind[ra + k] != dof) k++;
      if (k == rn) continue;
      const real* cd = d->cdof + 6 * dof;
      real cdd[6];
      const int jid = m->dof_jntid[dof], jt = m->jnt_type[jid];
      if (jt == JNT_BALL || (jt == JNT_FREE && dof >= m->jnt_dofadr[jid] + 3)) motion_cross(cdd, d->cvel + 6 * b, cd);
      else memcpy(cdd, d->cdof_dot + 6 * dof, sizeof(cdd));
      real c1[3], c2[3], c3[3], jpd[3], jp[3];
      cross3(c1, cdd, off);
      cross3(c2, cd, pvel);
      cross3(c3, cd, off);
      for (int i = 0; i < 3; i++) {
        jpd[i] = cdd[3 + i] + c1[i] + c2[i];
        jp[i] = cd[3 + i] + c3[i];
      }
      Jdot[k] += (dot3(jpd, dpnt) + dot3(jp, dvel)) * scale;
    }
}

static void point_vel(const orc_data* d, int body, const real* off, real* v) {
  const real* cv = d->cvel + 6 * body;
  real c[3];
  cross3(c, off, cv);
  for (int i = 0; i < 3; i++) v[i] = cv[3 + i] - c[i];
}

/* smooth.py:1656-1932 (_tendon_dot, tendon_bias): qfrc += armature J (Jdot qvel) for spatial tendons; as
 * the reference, a site-geom-site wrap ends the Jdot accumulation of its tendon (segments before it count) */
static void tendon_bias(const orc_model* m, orc_data* d, real* qfrc) {
  for (int t = 0; t < m->ntendon; t++) {
    const real arm = m->tendon_armature[t];
    const int a = m->tendon_adr[t], n = m->tendon_num[t];
    if (arm == 0 || m->wrap_type[a] == WRAP_JOINT) continue;
    const int ra = m->ten_J_rowadr[t], rn = m->ten_J_rownnz[t];
    real Jdot[64];
    if (rn > 64) abort();
    for (int k = 0; k < rn; k++) Jdot[k] = 0;
    real divisor = 1;
    for (int j = 0; j < n - 1; j++) {
      const int t0 = m->wrap_type[a + j], t1 = m->wrap_type[a + j + 1];
      if (t0 == WRAP_PULLEY || t1 == WRAP_PULLEY) {
        if (t0 == WRAP_PULLEY) divisor = m->wrap_prm[a + j];
        continue;
      }
      if (t1 == WRAP_SPHERE || t1 == WRAP_CYLINDER) break;
      const int s0 = m->wrap_objid[a + j], s1 = m->wrap_objid[a + j + 1];
      const int b0 = m->site_bodyid[s0], b1 = m->site_bodyid[s1];
      if (b0 == b1) continue;
      const real *p0 = d->site_xpos + 3 * s0, *p1 = d->site_xpos + 3 * s1;
      const real *sc0 = d->subtree_com + 3 * m->body_rootid[b0], *sc1 = d->subtree_com + 3 * m->body_rootid[b1];
      real off0[3], off1[3], v0[3], v1[3], dif[3], dpnt[3], dvel[3];
      for (int i = 0; i < 3; i++) { off0[i] = p0[i] - sc0[i]; off1[i] = p1[i] - sc1[i]; dif[i] = p1[i] - p0[i]; }
      point_vel(d, b0, off0, v0);
      point_vel(d, b1, off1, v1);
      real nrm = normalize_with_norm(dpnt, dif);
      for (int i = 0; i < 3; i++) dvel[i] = v1[i] - v0[i];
      real dt = dot3(dpnt, dvel);
      for (int i = 0; i < 3; i++) dvel[i] = nrm > MINVAL ? (dvel[i] - dpnt[i] * dt) / nrm : 0;
      real inv = safe_div(1.0, divisor);
      ten_jacdot_chain(m, d, t, b0, off0, v0, dpnt, dvel, -inv, Jdot);
      ten_jacdot_chain(m, d, t, b1, off1, v1, dpnt, dvel, inv, Jdot);
    }
    real coef = 0;
    for (int k = 0; k < rn; k++) coef += Jdot[k] * d->qvel[m->ten_J_colind[ra + k]];
    for (int k = 0; k < rn; k++) qfrc[m->ten_J_colind[ra + k]] += d->ten_J[ra + k] * arm * coef;
  }
}
