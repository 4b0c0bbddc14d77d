/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY (see oracle.h header comment).
 *
 * Serial, per-world restatement of mujoco_warp's `step` (forward.py:1003-1018)
 * for the primitive-geom, dense-Jacobian path: kinematics -> com_pos ->
 * camlight -> crb/qM -> collision (NXN + primitive narrowphase) ->
 * make_constraint -> transmission -> velocity -> passive -> rne -> actuation ->
 * acceleration (Cholesky factor/solve) -> CG / Newton solver -> Euler.
 * Every function cites the reference file:line it follows.  Worlds are
 * independent; orc_step() runs them in an OpenMP loop (CPU baseline leg).
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define MINVAL ((real)1e-15)
#define MAXVAL ((real)1e10)
#define MINIMP ((real)0.0001)
#define MAXIMP ((real)0.9999)
#define MINMU ((real)1e-5)

enum { JNT_FREE = 0, JNT_BALL = 1, JNT_SLIDE = 2, JNT_HINGE = 3 };
enum { GEOM_PLANE = 0, GEOM_HFIELD = 1, GEOM_SPHERE = 2, GEOM_CAPSULE = 3, GEOM_ELLIPSOID = 4, GEOM_CYLINDER = 5, GEOM_BOX = 6, GEOM_MESH = 7 };
enum { DSBL_CONSTRAINT = 1, DSBL_EQUALITY = 2, DSBL_FRICTIONLOSS = 4, DSBL_LIMIT = 8, DSBL_CONTACT = 16,
       DSBL_SPRING = 32, DSBL_DAMPER = 64, DSBL_GRAVITY = 128, DSBL_CLAMPCTRL = 256, DSBL_WARMSTART = 512,
       DSBL_FILTERPARENT = 1024, DSBL_ACTUATION = 2048, DSBL_REFSAFE = 4096, DSBL_SENSOR = 8192, DSBL_EULERDAMP = 1 << 15 };
enum { ENBL_MULTICCD = 16 };
enum { CNSTR_EQUALITY = 0, CNSTR_FRICTION_DOF = 1, CNSTR_LIMIT_JOINT = 3, CNSTR_CONTACT_FRICTIONLESS = 5, CNSTR_CONTACT_PYRAMIDAL = 6,
       CNSTR_CONTACT_ELLIPTIC = 7 };
enum { CONE_PYRAMIDAL = 0, CONE_ELLIPTIC = 1 };
enum { STATE_SATISFIED = 0, STATE_QUADRATIC = 1, STATE_LINEARNEG = 2, STATE_LINEARPOS = 3, STATE_CONE = 4 };
enum { SOLVER_CG = 1, SOLVER_NEWTON = 2 };
enum { INT_EULER = 0, INT_RK4 = 1, INT_IMPLICITFAST = 3 };
enum { CAM_FIXED = 0, CAM_TRACK = 1, CAM_TRACKCOM = 2, CAM_TARGETBODY = 3, CAM_TARGETBODYCOM = 4 };
enum { GAIN_FIXED = 0, GAIN_AFFINE = 1, GAIN_MUSCLE = 2 };
enum { DYN_NONE = 0, DYN_INTEGRATOR = 1, DYN_FILTER = 2, DYN_FILTEREXACT = 3, DYN_MUSCLE = 4, DYN_USER = 5 };
enum { EQ_CONNECT = 0, EQ_WELD = 1, EQ_JOINT = 2, EQ_TENDON = 3, EQ_FLEX = 4 };
enum { OBJ_UNKNOWN = 0, OBJ_BODY = 1, OBJ_XBODY = 2, OBJ_GEOM = 5, OBJ_SITE = 6, OBJ_CAMERA = 7 };
enum { INTEGRATOR_EULER = 0, INTEGRATOR_RK4 = 1, INTEGRATOR_IMPLICIT = 2, INTEGRATOR_IMPLICITFAST = 3 };
enum { BIAS_NONE = 0, BIAS_AFFINE = 1, BIAS_MUSCLE = 2 };
enum { TRN_JOINT = 0, TRN_JOINTINPARENT = 1, TRN_SLIDERCRANK = 2, TRN_TENDON = 3, TRN_SITE = 4, TRN_BODY = 5 };
enum { CNSTR_FRICTION_TENDON = 2, CNSTR_LIMIT_TENDON = 4 };
enum { FILTER_PLANE = 1, FILTER_SPHERE = 2, FILTER_AABB = 4, FILTER_OBB = 8 };

/* =============================================================================================
 * math helpers (mujoco_warp/_src/math.py)
 * ============================================================================================= */
static inline real dot3(const real* a, const real* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline void cross3(real* r, const real* a, const real* b) {
  real t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static inline real clampr(real x, real lo, real hi) { return x < lo ? lo : (x > hi ? hi : x); }
static inline real maxr(real a, real b) { return a > b ? a : b; }
static inline real minr(real a, real b) { return a < b ? a : b; }
static inline real safe_div(real x, real y) { return x / (y != 0 ? y : MINVAL); } /* math.py:317-319 */

/* wp.normalize: zero vector stays zero */
static inline void normalize3(real* v) {
  real n = sqrt(dot3(v, v));
  if (n > 0) { v[0] /= n; v[1] /= n; v[2] /= n; } else { v[0] = v[1] = v[2] = 0; }
}
static inline void normalize4(real* q) {
  real n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n > 0) { q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n; } else { q[0] = q[1] = q[2] = q[3] = 0; }
}

/* math.py:23-30 */
static void mul_quat(real* r, const real* u, const real* v) {
  real t0 = u[0] * v[0] - u[1] * v[1] - u[2] * v[2] - u[3] * v[3];
  real t1 = u[0] * v[1] + u[1] * v[0] + u[2] * v[3] - u[3] * v[2];
  real t2 = u[0] * v[2] - u[1] * v[3] + u[2] * v[0] + u[3] * v[1];
  real t3 = u[0] * v[3] + u[1] * v[2] - u[2] * v[1] + u[3] * v[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}

/* math.py:44-49 */
static void rot_vec_quat(real* r, const real* vec, const real* q) {
  real s = q[0], u[3] = {q[1], q[2], q[3]}, c[3];
  real uv = dot3(u, vec), uu = dot3(u, u);
  cross3(c, u, vec);
  real t[3];
  for (int i = 0; i < 3; i++) t[i] = 2 * (uv * u[i]) + (s * s - uu) * vec[i] + 2 * s * c[i];
  r[0] = t[0]; r[1] = t[1]; r[2] = t[2];
}

/* math.py:52-56 */
static void axis_angle_to_quat(real* q, const real* axis, real angle) {
  real s = sin(angle * (real)0.5), c = cos(angle * (real)0.5);
  q[0] = c; q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}

/* math.py:59-83 (row-major 3x3) */
static void quat_to_mat(real* m, const real* q) {
  real q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  real q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3], q22 = q[2] * q[2];
  real q23 = q[2] * q[3], q33 = q[3] * q[3];
  m[0] = q00 + q11 - q22 - q33; m[1] = 2 * (q12 - q03); m[2] = 2 * (q13 + q02);
  m[3] = 2 * (q12 + q03); m[4] = q00 - q11 + q22 - q33; m[5] = 2 * (q23 - q01);
  m[6] = 2 * (q13 - q02); m[7] = 2 * (q23 + q01); m[8] = q00 - q11 - q22 + q33;
}

/* math.py:120-130 mju_mulInertVec */
static void inert_vec(real* r, const real* i, const real* v) {
  real t[6];
  t[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  t[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  t[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  t[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  t[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  t[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
  memcpy(r, t, sizeof(t));
}

/* math.py:133-144 */
static void motion_cross(real* r, const real* u, const real* v) {
  real a[3], b[3], c[3];
  cross3(a, u, v);
  cross3(b, u + 3, v);
  cross3(c, u, v + 3);
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
  r[3] = b[0] + c[0]; r[4] = b[1] + c[1]; r[5] = b[2] + c[2];
}

/* math.py:147-158 */
static void motion_cross_force(real* r, const real* v, const real* f) {
  real a[3], b[3], c[3];
  cross3(a, v, f);
  cross3(b, v + 3, f + 3);
  cross3(c, v, f + 3);
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
  r[3] = c[0]; r[4] = c[1]; r[5] = c[2];
}

/* math.py:161-174 */
static void quat_to_vel(real* r, const real* q) {
  real axis[3] = {q[1], q[2], q[3]};
  real s = sqrt(dot3(axis, axis));
  if (s == 0) { r[0] = r[1] = r[2] = 0; return; }
  real speed = 2 * atan2(s, q[0]);
  if (speed > (real)M_PI) speed -= 2 * (real)M_PI;
  for (int i = 0; i < 3; i++) r[i] = axis[i] * speed / s;
}

/* math.py:177-185 */
static void quat_sub(real* r, const real* qa, const real* qb) {
  real qneg[4] = {qb[0], -qb[1], -qb[2], -qb[3]}, qdif[4];
  mul_quat(qdif, qneg, qa);
  quat_to_vel(r, qdif);
}

/* math.py:188-199 */
static void quat_integrate(real* res, const real* qin, const real* vin, real dt) {
  real v[3] = {vin[0], vin[1], vin[2]};
  real n = sqrt(dot3(v, v));
  normalize3(v);
  real qr[4], q[4] = {qin[0], qin[1], qin[2], qin[3]};
  axis_angle_to_quat(qr, v, dt * n);
  normalize4(q);
  mul_quat(res, q, qr);
  normalize4(res);
}

/* math.py:202-213 */
static void orthogonals(real* b, real* c, const real* a) {
  int usey = (-0.5 < a[1]) && (a[1] < 0.5);
  b[0] = 0; b[1] = usey ? 1 : 0; b[2] = usey ? 0 : 1;
  real d = dot3(a, b);
  for (int i = 0; i < 3; i++) b[i] -= a[i] * d;
  normalize3(b);
  if (sqrt(dot3(a, a)) == 0) b[0] = b[1] = b[2] = 0;
  cross3(c, a, b);
}

/* math.py:246-257: rows = (normal, tangent1, tangent2) */
static void make_frame(real* f, const real* ain) {
  real a[3] = {ain[0], ain[1], ain[2]}, b[3], c[3];
  normalize3(a);
  orthogonals(b, c, a);
  f[0] = a[0]; f[1] = a[1]; f[2] = a[2];
  f[3] = b[0]; f[4] = b[1]; f[5] = b[2];
  f[6] = c[0]; f[7] = c[1]; f[8] = c[2];
}

/* math.py:268-281 */
static void closest_segment_point(real* r, const real* a, const real* b, const real* pt) {
  real ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, pa[3] = {pt[0] - a[0], pt[1] - a[1], pt[2] - a[2]};
  real t = dot3(pa, ab) / (dot3(ab, ab) + (real)1e-6);
  t = clampr(t, 0, 1);
  for (int i = 0; i < 3; i++) r[i] = a[i] + t * ab[i];
}

static real closest_segment_point_and_dist(real* r, const real* a, const real* b, const real* pt) {
  closest_segment_point(r, a, b, pt);
  real d[3] = {pt[0] - r[0], pt[1] - r[1], pt[2] - r[2]};
  return dot3(d, d);
}

static real normalize_with_norm(real* r, const real* x) {
  real n = sqrt(dot3(x, x));
  if (n == 0) { r[0] = x[0]; r[1] = x[1]; r[2] = x[2]; return 0; }
  r[0] = x[0] / n; r[1] = x[1] / n; r[2] = x[2] / n;
  return n;
}

/* math.py:284-314 */
void orc_closest_segment_to_segment_points(const real* a0, const real* a1, const real* b0, const real* b1,
                                           real* best_a, real* best_b) {
  real da[3] = {a1[0] - a0[0], a1[1] - a0[1], a1[2] - a0[2]}, db[3] = {b1[0] - b0[0], b1[1] - b0[1], b1[2] - b0[2]};
  real dir_a[3], dir_b[3];
  real len_a = normalize_with_norm(dir_a, da), len_b = normalize_with_norm(dir_b, db);
  real ha = len_a * (real)0.5, hb = len_b * (real)0.5;
  real am[3], bm[3], tr[3];
  for (int i = 0; i < 3; i++) { am[i] = a0[i] + dir_a[i] * ha; bm[i] = b0[i] + dir_b[i] * hb; tr[i] = am[i] - bm[i]; }
  real dadb = dot3(dir_a, dir_b), dat = dot3(dir_a, tr), dbt = dot3(dir_b, tr);
  real denom = 1 - dadb * dadb;
  real ota = (-dat + dadb * dbt) / (denom + (real)1e-6);
  real otb = dbt + ota * dadb;
  real ta = clampr(ota, -ha, ha), tb = clampr(otb, -hb, hb);
  real ba[3], bb[3], na[3], nb[3];
  for (int i = 0; i < 3; i++) { ba[i] = am[i] + dir_a[i] * ta; bb[i] = bm[i] + dir_b[i] * tb; }
  real d1 = closest_segment_point_and_dist(na, a0, a1, bb);
  real d2 = closest_segment_point_and_dist(nb, b0, b1, ba);
  if (d1 < d2) { memcpy(best_a, na, 3 * sizeof(real)); memcpy(best_b, bb, 3 * sizeof(real)); }
  else { memcpy(best_a, ba, 3 * sizeof(real)); memcpy(best_b, nb, 3 * sizeof(real)); }
}

/* math.py:322-333 */
int orc_upper_tri_index(int n, int i, int j) { return (i * (2 * n - i - 3)) / 2 + j - 1; }
int orc_upper_trid_index(int n, int i, int j) {
  if (j < i) { int t = i; i = j; j = t; }
  return (i * (2 * n - i - 1)) / 2 + j;
}

/* util_misc.py:59-73 */
real orc_halton(int index, int base) {
  int n0 = index;
  real b = (real)base, f = (real)1 / b, hn = 0;
  while (n0 > 0) {
    int n1 = n0 / base;
    int r = n0 - n1 * base;
    hn += f * (real)r;
    f /= b;
    n0 = n1;
  }
  return hn;
}

/* benchmark.py:41-83 (world ids are global: worldid = world_offset + w) */
void orc_ctrl_noise(const orc_model* m, real* ctrl, const real* center, int ncenter, int step, real std,
                    real rate_, int nworld, int world_offset) {
  for (int w = 0; w < nworld; w++) {
    int worldid = world_offset + w;
    for (int a = 0; a < m->nu; a++) {
      real rate = exp(-m->opt_timestep / rate_);
      real scale = std * sqrt(1 - rate * rate);
      real midpoint = 0, halfrange = 1;
      const real* cr = m->actuator_ctrlrange + 2 * a;
      if (m->actuator_ctrllimited[a]) { midpoint = (real)0.5 * (cr[1] + cr[0]); halfrange = (real)0.5 * (cr[1] - cr[0]); }
      if (ncenter > 0) midpoint = center[a];
      real* c = ctrl + (size_t)w * m->nu + a;
      real v = rate * (*c) + (1 - rate) * midpoint;
      v += scale * halfrange * (2 * orc_halton((step + 1) * (worldid + 1), a + 2) - 1);
      if (m->actuator_ctrllimited[a]) v = clampr(v, cr[0], cr[1]);
      *c = v;
    }
  }
}

/* =============================================================================================
 * per-world view
 * ============================================================================================= */
static void world_view(const orc_model* m, const orc_data* b, int w, orc_data* o) {
  int nq = m->nq, nv = m->nv, nu = m->nu, na = m->na, nbody = m->nbody, njnt = m->njnt;
  int ngeom = m->ngeom, nsite = m->nsite, ncam = m->ncam, nlight = m->nlight, nmocap = m->nmocap, neq = m->neq;
  int njmax = b->njmax, nconmax = b->nconmax, nsensordata = m->nsensordata;
  int nflexvert = m->nflexvert, nflexedge = m->nflexedge, ntendon = m->ntendon, nJten = m->nJten;
  (void)nflexvert; (void)nflexedge; (void)ntendon; (void)nJten;
  (void)nsensordata;
  (void)nq; (void)nv; (void)nu; (void)na; (void)nbody; (void)njnt; (void)ngeom; (void)nsite; (void)ncam;
  (void)nlight; (void)nmocap; (void)njmax; (void)nconmax; (void)neq;
  o->njmax = njmax;
  o->nconmax = nconmax;
#define ORC_OFF(name, n) o->name = b->name + (size_t)w * (size_t)(n);
  ORC_DATA_REAL_ARRAYS(ORC_OFF)
  ORC_DATA_INT_ARRAYS(ORC_OFF)
#undef ORC_OFF
}

/* =============================================================================================
 * smooth.py
 * ============================================================================================= */

/* smooth.py:44-143 (_kinematics_branch) + :146-224 (inertial frames, matrices, geoms, sites) */
static void kinematics(const orc_model* m, orc_data* d) {
  real* xpos = d->xpos;
  real* xquat = d->xquat;
  /* world body */
  xpos[0] = xpos[1] = xpos[2] = 0;
  xquat[0] = 1; xquat[1] = xquat[2] = xquat[3] = 0;
  for (int b = 1; b < m->nbody; b++) {
    int pid = m->body_parentid[b];
    int jntadr = m->body_jntadr[b], jntnum = m->body_jntnum[b];
    if (jntnum == 1 && m->jnt_type[jntadr] == JNT_FREE) {
      int qa = m->jnt_qposadr[jntadr];
      real q[4] = {d->qpos[qa + 3], d->qpos[qa + 4], d->qpos[qa + 5], d->qpos[qa + 6]};
      normalize4(q);
      for (int i = 0; i < 3; i++) xpos[3 * b + i] = d->qpos[qa + i];
      memcpy(xquat + 4 * b, q, sizeof(q));
      for (int i = 0; i < 3; i++) { d->xanchor[3 * jntadr + i] = d->qpos[qa + i]; d->xaxis[3 * jntadr + i] = m->jnt_axis[3 * jntadr + i]; }
      continue;
    }
    real pos[3], quat[4];
    int mocapid = m->body_mocapid[b];
    if (mocapid >= 0) {
      memcpy(pos, d->mocap_pos + 3 * mocapid, 3 * sizeof(real));
      memcpy(quat, d->mocap_quat + 4 * mocapid, 4 * sizeof(real));
    } else {
      memcpy(pos, m->body_pos + 3 * b, 3 * sizeof(real));
      memcpy(quat, m->body_quat + 4 * b, 4 * sizeof(real));
    }
    if (pid >= 0) {
      real t[3];
      rot_vec_quat(t, pos, xquat + 4 * pid);
      for (int i = 0; i < 3; i++) pos[i] = t[i] + xpos[3 * pid + i];
      mul_quat(quat, xquat + 4 * pid, quat);
    }
    for (int k = 0; k < jntnum; k++) {
      int j = jntadr + k;
      int qa = m->jnt_qposadr[j];
      const real* axis = m->jnt_axis + 3 * j;
      const real* jpos = m->jnt_pos + 3 * j;
      real xanchor[3], xaxis[3], t[3];
      rot_vec_quat(t, jpos, quat);
      for (int i = 0; i < 3; i++) xanchor[i] = t[i] + pos[i];
      rot_vec_quat(xaxis, axis, quat);
      int jt = m->jnt_type[j];
      if (jt == JNT_BALL) {
        real ql[4] = {d->qpos[qa], d->qpos[qa + 1], d->qpos[qa + 2], d->qpos[qa + 3]};
        normalize4(ql);
        mul_quat(quat, quat, ql);
        rot_vec_quat(t, jpos, quat);
        for (int i = 0; i < 3; i++) pos[i] = xanchor[i] - t[i];
      } else if (jt == JNT_SLIDE) {
        real dq = d->qpos[qa] - m->qpos0[qa];
        for (int i = 0; i < 3; i++) pos[i] += xaxis[i] * dq;
      } else if (jt == JNT_HINGE) {
        real ql[4];
        axis_angle_to_quat(ql, axis, d->qpos[qa] - m->qpos0[qa]);
        mul_quat(quat, quat, ql);
        rot_vec_quat(t, jpos, quat);
        for (int i = 0; i < 3; i++) pos[i] = xanchor[i] - t[i];
      }
      memcpy(d->xanchor + 3 * j, xanchor, sizeof(xanchor));
      memcpy(d->xaxis + 3 * j, xaxis, sizeof(xaxis));
    }
    normalize4(quat);
    memcpy(xpos + 3 * b, pos, sizeof(pos));
    memcpy(xquat + 4 * b, quat, sizeof(quat));
  }
  for (int b = 0; b < m->nbody; b++) {
    real q[4], t[3];
    quat_to_mat(d->xmat + 9 * b, xquat + 4 * b);
    rot_vec_quat(t, m->body_ipos + 3 * b, xquat + 4 * b);
    for (int i = 0; i < 3; i++) d->xipos[3 * b + i] = xpos[3 * b + i] + t[i];
    mul_quat(q, xquat + 4 * b, m->body_iquat + 4 * b);
    quat_to_mat(d->ximat + 9 * b, q);
  }
  for (int g = 0; g < m->ngeom; g++) {
    int b = m->geom_bodyid[g];
    /* smooth.py:195-198: static world geoms are computed once (at put_data) */
    if (m->body_weldid[b] == 0 && m->body_mocapid[m->body_rootid[b]] == -1) {
      real q[4], t[3];
      /* world frame is identity: pose equals the model pose */
      rot_vec_quat(t, m->geom_pos + 3 * g, xquat + 4 * b);
      for (int i = 0; i < 3; i++) d->geom_xpos[3 * g + i] = xpos[3 * b + i] + t[i];
      mul_quat(q, xquat + 4 * b, m->geom_quat + 4 * g);
      quat_to_mat(d->geom_xmat + 9 * g, q);
      continue;
    }
    real q[4], t[3];
    rot_vec_quat(t, m->geom_pos + 3 * g, xquat + 4 * b);
    for (int i = 0; i < 3; i++) d->geom_xpos[3 * g + i] = xpos[3 * b + i] + t[i];
    mul_quat(q, xquat + 4 * b, m->geom_quat + 4 * g);
    quat_to_mat(d->geom_xmat + 9 * g, q);
  }
  for (int s = 0; s < m->nsite; s++) {
    int b = m->site_bodyid[s];
    real q[4], t[3];
    rot_vec_quat(t, m->site_pos + 3 * s, xquat + 4 * b);
    for (int i = 0; i < 3; i++) d->site_xpos[3 * s + i] = xpos[3 * b + i] + t[i];
    mul_quat(q, xquat + 4 * b, m->site_quat + 4 * s);
    quat_to_mat(d->site_xmat + 9 * s, q);
  }
}

/* smooth.py:463-632 (subtree com, cinert, cdof) */
static void com_pos(const orc_model* m, orc_data* d) {
  int nb = m->nbody;
  real* sc = d->subtree_com;
  for (int b = 0; b < nb; b++)
    for (int i = 0; i < 3; i++) sc[3 * b + i] = d->xipos[3 * b + i] * m->body_mass[b];
  for (int b = nb - 1; b > 0; b--) {
    int p = m->body_parentid[b];
    for (int i = 0; i < 3; i++) sc[3 * p + i] += sc[3 * b + i];
  }
  for (int b = 0; b < nb; b++) {
    real mass = m->body_subtreemass[b];
    if (mass != 0)
      for (int i = 0; i < 3; i++) sc[3 * b + i] /= mass;
  }
  /* _cinert smooth.py:510-553 */
  for (int b = 0; b < nb; b++) {
    const real* mat = d->ximat + 9 * b;
    const real* inert = m->body_inertia + 3 * b;
    real mass = m->body_mass[b];
    real dif[3];
    for (int i = 0; i < 3; i++) dif[i] = d->xipos[3 * b + i] - sc[3 * m->body_rootid[b] + i];
    real tmp[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        real s = 0;
        for (int k = 0; k < 3; k++) s += mat[3 * i + k] * inert[k] * mat[3 * j + k];
        tmp[3 * i + j] = s;
      }
    real* res = d->cinert + 10 * b;
    res[0] = tmp[0] + mass * (dif[1] * dif[1] + dif[2] * dif[2]);
    res[1] = tmp[4] + mass * (dif[0] * dif[0] + dif[2] * dif[2]);
    res[2] = tmp[8] + mass * (dif[0] * dif[0] + dif[1] * dif[1]);
    res[3] = tmp[1] - mass * dif[0] * dif[1];
    res[4] = tmp[2] - mass * dif[0] * dif[2];
    res[5] = tmp[5] - mass * dif[1] * dif[2];
    res[6] = mass * dif[0];
    res[7] = mass * dif[1];
    res[8] = mass * dif[2];
    res[9] = mass;
  }
  /* _cdof smooth.py:556-598 */
  for (int j = 0; j < m->njnt; j++) {
    int b = m->jnt_bodyid[j], da = m->jnt_dofadr[j], jt = m->jnt_type[j];
    const real* xaxis = d->xaxis + 3 * j;
    const real* xmat = d->xmat + 9 * b;
    real off[3];
    for (int i = 0; i < 3; i++) off[i] = sc[3 * m->body_rootid[b] + i] - d->xanchor[3 * j + i];
    real* cd = d->cdof;
    if (jt == JNT_FREE || jt == JNT_BALL) {
      int rot0 = da;
      if (jt == JNT_FREE) {
        for (int k = 0; k < 3; k++) {
          real* r = cd + 6 * (da + k);
          memset(r, 0, 6 * sizeof(real));
          r[3 + k] = 1;
        }
        rot0 = da + 3;
      }
      for (int k = 0; k < 3; k++) {
        real ax[3] = {xmat[k], xmat[3 + k], xmat[6 + k]}; /* column k of xmat */
        real* r = cd + 6 * (rot0 + k);
        r[0] = ax[0]; r[1] = ax[1]; r[2] = ax[2];
        cross3(r + 3, ax, off);
      }
    } else if (jt == JNT_SLIDE) {
      real* r = cd + 6 * da;
      r[0] = r[1] = r[2] = 0;
      r[3] = xaxis[0]; r[4] = xaxis[1]; r[5] = xaxis[2];
    } else {
      real* r = cd + 6 * da;
      r[0] = xaxis[0]; r[1] = xaxis[1]; r[2] = xaxis[2];
      cross3(r + 3, xaxis, off);
    }
  }
}

/* smooth.py:635-803 (camlight) */
static void camlight(const orc_model* m, orc_data* d) {
  for (int c = 0; c < m->ncam; c++) {
    int mode = m->cam_mode[c], b = m->cam_bodyid[c], tgt = m->cam_targetbodyid[c];
    int is_target = (mode == CAM_TARGETBODY) || (mode == CAM_TARGETBODYCOM);
    real* cx = d->cam_xpos + 3 * c;
    real* cm = d->cam_xmat + 9 * c;
    if ((is_target && tgt < 0) || mode == CAM_FIXED) {
      real t[3], q[4];
      rot_vec_quat(t, m->cam_pos + 3 * c, d->xquat + 4 * b);
      for (int i = 0; i < 3; i++) cx[i] = d->xpos[3 * b + i] + t[i];
      mul_quat(q, d->xquat + 4 * b, m->cam_quat + 4 * c);
      quat_to_mat(cm, q);
    } else if (mode == CAM_TRACK) {
      memcpy(cm, m->cam_mat0 + 9 * c, 9 * sizeof(real));
      for (int i = 0; i < 3; i++) cx[i] = d->xpos[3 * b + i] + m->cam_pos0[3 * c + i];
    } else if (mode == CAM_TRACKCOM) {
      memcpy(cm, m->cam_mat0 + 9 * c, 9 * sizeof(real));
      for (int i = 0; i < 3; i++) cx[i] = d->subtree_com[3 * b + i] + m->cam_poscom0[3 * c + i];
    } else {
      real t[3], pos[3], m1[3], m2[3], m3[3];
      rot_vec_quat(t, m->cam_pos + 3 * c, d->xquat + 4 * b);
      for (int i = 0; i < 3; i++) cx[i] = d->xpos[3 * b + i] + t[i];
      const real* tp = (mode == CAM_TARGETBODYCOM) ? d->subtree_com + 3 * tgt : d->xpos + 3 * tgt;
      for (int i = 0; i < 3; i++) { pos[i] = tp[i]; m3[i] = cx[i] - pos[i]; }
      normalize3(m3);
      real z[3] = {0, 0, 1};
      cross3(m1, z, m3);
      normalize3(m1);
      cross3(m2, m3, m1);
      normalize3(m2);
      for (int i = 0; i < 3; i++) { cm[3 * i] = m1[i]; cm[3 * i + 1] = m2[i]; cm[3 * i + 2] = m3[i]; }
    }
  }
  for (int l = 0; l < m->nlight; l++) {
    int mode = m->light_mode[l], b = m->light_bodyid[l], tgt = m->light_targetbodyid[l];
    int is_target = (mode == CAM_TARGETBODY) || (mode == CAM_TARGETBODYCOM);
    real* lx = d->light_xpos + 3 * l;
    real* ld = d->light_xdir + 3 * l;
    if ((is_target && tgt < 0) || mode == CAM_FIXED) {
      real t[3];
      rot_vec_quat(t, m->light_pos + 3 * l, d->xquat + 4 * b);
      for (int i = 0; i < 3; i++) lx[i] = d->xpos[3 * b + i] + t[i];
      rot_vec_quat(ld, m->light_dir + 3 * l, d->xquat + 4 * b);
      if (is_target && tgt < 0) continue; /* smooth.py:732 returns before normalize */
    } else if (mode == CAM_TRACK) {
      memcpy(ld, m->light_dir0 + 3 * l, 3 * sizeof(real));
      for (int i = 0; i < 3; i++) lx[i] = d->xpos[3 * b + i] + m->light_pos0[3 * l + i];
    } else if (mode == CAM_TRACKCOM) {
      memcpy(ld, m->light_dir0 + 3 * l, 3 * sizeof(real));
      for (int i = 0; i < 3; i++) lx[i] = d->subtree_com[3 * b + i] + m->light_poscom0[3 * l + i];
    } else {
      real t[3];
      rot_vec_quat(t, m->light_pos + 3 * l, d->xquat + 4 * b);
      for (int i = 0; i < 3; i++) lx[i] = d->xpos[3 * b + i] + t[i];
      const real* tp = (mode == CAM_TARGETBODYCOM) ? d->subtree_com + 3 * tgt : d->xpos + 3 * tgt;
      for (int i = 0; i < 3; i++) ld[i] = tp[i] - lx[i];
    }
    normalize3(ld);
  }
}

static void matvec3(real* r, const real* M, const real* v);

/* smooth.py:228-258 _flex_vertices, :261-355 _flex_edges (edge length, velocity and the Jacobian of
 * the edge length w.r.t. the two vertex bodies' own dofs -- the reference's "TODO: use Jacobian"
 * form; flexedge_J holds body 1's dofs then body 2's, 6 slots per edge) */
static void flex_kinematics(const orc_model* m, orc_data* d) {
  for (int v = 0; v < m->nflexvert; v++) {
    int b = m->flex_vertbodyid[v], f = m->flex_vertflexid[v];
    if (m->flex_centered[f]) {
      for (int i = 0; i < 3; i++) d->flexvert_xpos[3 * v + i] = d->xpos[3 * b + i];
    } else {
      real t[3];
      matvec3(t, d->xmat + 9 * b, m->flex_vert + 3 * v);
      for (int i = 0; i < 3; i++) d->flexvert_xpos[3 * v + i] = t[i] + d->xpos[3 * b + i];
    }
  }
  for (int f = 0; f < m->nflex; f++) {
    for (int e = m->flex_edgeadr[f]; e < m->flex_edgeadr[f] + m->flex_edgenum[f]; e++) {
      int v[2] = {m->flex_vertadr[f] + m->flex_edge[2 * e], m->flex_vertadr[f] + m->flex_edge[2 * e + 1]};
      const real* p1 = d->flexvert_xpos + 3 * v[0];
      const real* p2 = d->flexvert_xpos + 3 * v[1];
      real vec[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]}, dir[3];
      d->flexedge_length[e] = normalize_with_norm(dir, vec);
      real vel = 0;
      real* J = d->flexedge_J + 6 * e;
      for (int k = 0; k < 6; k++) J[k] = 0;
      int slot = 0;
      for (int s2 = 0; s2 < 2; s2++) {
        int b = m->flex_vertbodyid[v[s2]];
        const real* p = s2 ? p2 : p1;
        real off[3];
        for (int i = 0; i < 3; i++) off[i] = p[i] - d->subtree_com[3 * m->body_rootid[b] + i];
        for (int k = 0; k < m->body_dofnum[b]; k++) {
          int dof = m->body_dofadr[b] + k;
          const real* cd = d->cdof + 6 * dof;
          real c[3], jacp[3];
          cross3(c, cd, off);
          for (int i = 0; i < 3; i++) jacp[i] = cd[3 + i] + c[i];
          real jv = dot3(jacp, dir) * (s2 ? 1 : -1);
          vel += jv * d->qvel[dof];
          J[slot++] = jv;
        }
      }
      d->flexedge_velocity[e] = vel;
    }
  }
}

/* passive.py:566-662 _flex_elasticity and :665-725 _flex_bending, accumulated into qfrc_spring */
/* the local edges of a segment / triangle / tetrahedron, passive.py:606-613 */
static const int flex_ledge[4][6][2] = {{{0}},
                                        {{0, 1}},
                                        {{1, 2}, {2, 0}, {0, 1}},
                                        {{0, 1}, {1, 2}, {2, 0}, {2, 3}, {0, 3}, {1, 3}}};
static const int flex_nledge[4] = {0, 1, 3, 6};

static void flex_passive(const orc_model* m, orc_data* d) {
  for (int f = 0; f < m->nflex; f++) {
    const int dim = m->flex_dim[f], nve = dim + 1, ne = flex_nledge[dim];
    const int(*edges2)[2] = flex_ledge[dim];
    real kD = (m->opt_timestep > 0 && !(m->opt_disableflags & DSBL_DAMPER)) ? m->flex_damping[f] / m->opt_timestep : 0;
    for (int el = 0; el < m->flex_elemnum[f]; el++) {
      int elemid = m->flex_elemadr[f] + el;
      const int* ev = m->flex_elem + m->flex_elemdataadr[f] + nve * el;
      int vb = m->flex_vertadr[f];
      real grad[6][6], elong[6], metric[6][6], force[4][3] = {{0}};
      for (int e = 0; e < ne; e++) {
        const real* x0 = d->flexvert_xpos + 3 * (vb + ev[edges2[e][0]]);
        const real* x1 = d->flexvert_xpos + 3 * (vb + ev[edges2[e][1]]);
        for (int i = 0; i < 3; i++) { grad[e][i] = x0[i] - x1[i]; grad[e][3 + i] = x1[i] - x0[i]; }
        int idx = m->flex_edgeadr[f] + m->flex_elemedge[m->flex_elemedgeadr[f] + ne * el + e];
        real vel = d->flexedge_velocity[idx], def = d->flexedge_length[idx], ref = m->flexedge_length0[idx];
        real prev = def - vel * m->opt_timestep;
        elong[e] = def * def - ref * ref + (def * def - prev * prev) * kD;
      }
      int id = 0;
      for (int a = 0; a < ne; a++)
        for (int b = a; b < ne; b++) { metric[a][b] = metric[b][a] = m->flex_stiffness[21 * elemid + id]; id++; }
      for (int e1 = 0; e1 < ne; e1++)
        for (int e2 = 0; e2 < ne; e2++)
          for (int i = 0; i < 2; i++)
            for (int x = 0; x < 3; x++) force[edges2[e2][i]][x] -= elong[e1] * grad[e2][3 * i + x] * metric[e1][e2];
      for (int k = 0; k < nve; k++) {
        int b = m->flex_vertbodyid[vb + ev[k]];
        if (m->body_dofnum[b] == 0) continue;
        for (int x = 0; x < 3; x++) d->qfrc_spring[m->body_dofadr[b] + x] += force[k][x];
      }
    }
    for (int e = m->flex_edgeadr[f]; e < m->flex_edgeadr[f] + m->flex_edgenum[f]; e++) {
      if (m->flex_edgeflap[2 * e + 1] == -1) continue;
      int vb = m->flex_vertadr[f];
      int v[4] = {vb + m->flex_edge[2 * e], vb + m->flex_edge[2 * e + 1], vb + m->flex_edgeflap[2 * e], vb + m->flex_edgeflap[2 * e + 1]};
      const real* B = m->flex_bending + 17 * e;
      real frc[4][3] = {{0}};
      if (B[16] != 0) {
        const real *v0 = d->flexvert_xpos + 3 * v[0], *v1 = d->flexvert_xpos + 3 * v[1];
        const real *v2 = d->flexvert_xpos + 3 * v[2], *v3 = d->flexvert_xpos + 3 * v[3];
        real a1[3], a2[3], a3[3];
        for (int i = 0; i < 3; i++) { a1[i] = v1[i] - v0[i]; a2[i] = v2[i] - v0[i]; a3[i] = v3[i] - v0[i]; }
        cross3(frc[1], a2, a3);
        cross3(frc[2], a3, a1);
        cross3(frc[3], a1, a2);
        for (int i = 0; i < 3; i++) frc[0][i] = -(frc[1][i] + frc[2][i] + frc[3][i]);
      }
      for (int i = 0; i < 4; i++) {
        int b = m->flex_vertbodyid[v[i]];
        for (int x = 0; x < 3; x++) {
          real fx = 0;
          for (int j = 0; j < 4; j++) fx -= B[4 * i + j] * d->flexvert_xpos[3 * v[j] + x];
          fx -= B[16] * frc[i][x];
          if (m->body_dofnum[b]) d->qfrc_spring[m->body_dofadr[b] + x] += fx;
        }
      }
    }
  }
}

/* smooth.py:806-912 (crb accumulate + dense qM) */
static void crb(const orc_model* m, orc_data* d) {
  int nb = m->nbody, nv = m->nv;
  memcpy(d->crb, d->cinert, (size_t)nb * 10 * sizeof(real));
  for (int b = nb - 1; b > 0; b--) {
    int p = m->body_parentid[b];
    if (p == 0) continue;
    for (int i = 0; i < 10; i++) d->crb[10 * p + i] += d->crb[10 * b + i];
  }
  memset(d->qM, 0, (size_t)nv * nv * sizeof(real));
  for (int i = 0; i < nv; i++) {
    int b = m->dof_bodyid[i];
    real buf[6];
    inert_vec(buf, d->crb + 10 * b, d->cdof + 6 * i);
    real Mii = m->dof_armature[i];
    real s = 0;
    for (int k = 0; k < 6; k++) s += d->cdof[6 * i + k] * buf[k];
    Mii += s;
    d->qM[i * nv + i] = Mii;
    int j = m->dof_parentid[i];
    while (j >= 0) {
      real q = 0;
      for (int k = 0; k < 6; k++) q += d->cdof[6 * j + k] * buf[k];
      d->qM[i * nv + j] += q;
      d->qM[j * nv + i] += q;
      j = m->dof_parentid[j];
    }
  }
}

/* dense Cholesky M = L L^T (wp.tile_cholesky), L stored lower in qLD (row-major, nv x nv) */
static void cholesky(int n, const real* M, real* L) {
  memset(L, 0, (size_t)n * n * sizeof(real));
  for (int j = 0; j < n; j++) {
    real s = M[j * n + j];
    for (int k = 0; k < j; k++) s -= L[j * n + k] * L[j * n + k];
    real ljj = sqrt(s);
    L[j * n + j] = ljj;
    for (int i = j + 1; i < n; i++) {
      real t = M[i * n + j];
      for (int k = 0; k < j; k++) t -= L[i * n + k] * L[j * n + k];
      L[i * n + j] = t / ljj;
    }
  }
}

/* wp.tile_cholesky_solve: x = (L L^T)^-1 y */
static void cholesky_solve(int n, const real* L, const real* y, real* x) {
  real tmp[512];
  real* z = n <= 512 ? tmp : (real*)malloc(n * sizeof(real));
  for (int i = 0; i < n; i++) {
    real s = y[i];
    for (int k = 0; k < i; k++) s -= L[i * n + k] * z[k];
    z[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    real s = z[i];
    for (int k = i + 1; k < n; k++) s -= L[k * n + i] * x[k];
    x[i] = s / L[i * n + i];
  }
  if (z != tmp) free(z);
}

/* sparse path (is_sparse): M = L' D L over the kinematic tree (smooth.py:1003-1064 _factor_i_sparse,
 * the level-scheduled form of MuJoCo's mj_factorM) on dense storage: only ancestor entries are touched,
 * so the cost is O(nv * depth^2).  qLD holds D on the diagonal and L (unit, strictly lower) below it. */
static void factor_tree(const orc_model* m, int n, const real* M, real* L) {
  memcpy(L, M, (size_t)n * n * sizeof(real));
  for (int k = n - 1; k >= 0; k--) {
    for (int i = m->dof_parentid[k]; i >= 0; i = m->dof_parentid[i]) {
      real tmp = L[(size_t)k * n + i] / L[(size_t)k * n + k];
      for (int j = i; j >= 0; j = m->dof_parentid[j]) L[(size_t)i * n + j] -= tmp * L[(size_t)k * n + j];
      L[(size_t)k * n + i] = tmp;
    }
  }
}

/* smooth.py:2813-2846 _solve_LD_sparse: x = (L' D L)^-1 y */
static void solve_tree(const orc_model* m, int n, const real* L, const real* y, real* x) {
  if (x != y) memcpy(x, y, (size_t)n * sizeof(real));
  for (int k = n - 1; k >= 0; k--)
    for (int i = m->dof_parentid[k]; i >= 0; i = m->dof_parentid[i]) x[i] -= L[(size_t)k * n + i] * x[k];
  for (int k = 0; k < n; k++) x[k] /= L[(size_t)k * n + k];
  for (int k = 0; k < n; k++)
    for (int i = m->dof_parentid[k]; i >= 0; i = m->dof_parentid[i]) x[k] -= L[(size_t)k * n + i] * x[i];
}

/* factor_m / solve_m: the dense tile Cholesky or the sparse tree LDL, as the reference dispatches */
static void factor_m(const orc_model* m, int n, const real* M, real* L) {
  if (m->is_sparse) factor_tree(m, n, M, L);
  else cholesky(n, M, L);
}

static void solve_m(const orc_model* m, int n, const real* L, const real* y, real* x) {
  if (m->is_sparse) solve_tree(m, n, L, y, x);
  else cholesky_solve(n, L, y, x);
}

/* smooth.py:2041-2147 (_transmission, joint transmissions; dense moment rows) */
/* smooth.py:3085-3121 (_joint_tendon): fixed tendon length sum coef * qpos, Jacobian coef at the joint's
 * dof, stored in the sparse ten_J layout (ten_J_rowadr / _rownnz / _colind, dofs ascending) */
static real spatial_tendon(const orc_model* m, orc_data* d, int t);

static void tendon(const orc_model* m, orc_data* d) {
  for (int t = 0; t < m->ntendon; t++) {
    real L = 0;
    const int ra = m->ten_J_rowadr[t], rn = m->ten_J_rownnz[t];
    for (int k = 0; k < rn; k++) d->ten_J[ra + k] = 0;
    if (m->wrap_type[m->tendon_adr[t]] != 1) { /* spatial: oracle_tendon.h */
      d->ten_length[t] = spatial_tendon(m, d, t);
      continue;
    }
    for (int w = m->tendon_adr[t]; w < m->tendon_adr[t] + m->tendon_num[t]; w++) {
      const int j = m->wrap_objid[w];
      const real prm = m->wrap_prm[w];
      L += prm * d->qpos[m->jnt_qposadr[j]];
      for (int k = 0; k < rn; k++)
        if (m->ten_J_colind[ra + k] == m->jnt_dofadr[j]) { d->ten_J[ra + k] = prm; break; }
    }
    d->ten_length[t] = L;
  }
}

/* dense row of tendon t's Jacobian */
static void ten_J_dense(const orc_model* m, const orc_data* d, int t, real* J) {
  memset(J, 0, (size_t)m->nv * sizeof(real));
  for (int k = 0; k < m->ten_J_rownnz[t]; k++) J[m->ten_J_colind[m->ten_J_rowadr[t] + k]] = d->ten_J[m->ten_J_rowadr[t] + k];
}

/* smooth.py:916-1000 (_tendon_armature): qM[i][j] += armature J_i J_j for j = i and every ancestor j of i
 * (the ancestor pattern of qM) */
static void tendon_armature(const orc_model* m, orc_data* d) {
  int nv = m->nv;
  for (int t = 0; t < m->ntendon; t++) {
    const real arm = m->tendon_armature[t];
    if (arm == 0) continue;
    const int ra = m->ten_J_rowadr[t], rn = m->ten_J_rownnz[t];
    for (int k = 0; k < rn; k++) {
      const int i = m->ten_J_colind[ra + k];
      const real Ji = d->ten_J[ra + k];
      if (Ji == 0) continue;
      for (int j = i; j >= 0; j = m->dof_parentid[j]) {
        real Jj = 0;
        for (int q = 0; q < rn; q++)
          if (m->ten_J_colind[ra + q] == j) Jj = d->ten_J[ra + q];
        const real v = arm * Jj * Ji;
        d->qM[(size_t)i * nv + j] += v;
        if (i != j) d->qM[(size_t)j * nv + i] += v;
      }
    }
  }
}

static void rt_vec(real* r, const real* R, const real* v);
static void r_vec(real* r, const real* R, const real* v);

static int jac_dof(const orc_model* m, const orc_data* d, const real* point, int bodyid, int dofid, real* jacp, real* jacr);

static int last_dof(const orc_model* m, int body) { return body > 0 ? m->body_dofadr[body] + m->body_dofnum[body] - 1 : -1; }

/* smooth.py:2150-2241 (SLIDERCRANK) and 2274-2442 (SITE): moments over the union of the two bodies' dof
 * chains (SITE with a reference site: above their common ancestor dof only) */
static void site_transmission(const orc_model* m, orc_data* d, int a, real* mom) {
  const real* gear = m->actuator_gear + 6 * a;
  const int trn = m->actuator_trntype[a], id = m->actuator_trnid[2 * a], id2 = m->actuator_trnid[2 * a + 1];
  const real* sx = d->site_xpos + 3 * id;
  real jp[3], jr[3], jp2[3], jr2[3];
  if (trn == TRN_SLIDERCRANK) {
    const real rod = m->actuator_cranklength[a];
    const real* sm = d->site_xmat + 9 * id2;
    const real* sx2 = d->site_xpos + 3 * id2;
    real axis[3] = {sm[2], sm[5], sm[8]}, vec[3] = {sx[0] - sx2[0], sx[1] - sx2[1], sx[2] - sx2[2]};
    real av = dot3(vec, axis), det = av * av + rod * rod - dot3(vec, vec), sdet = 0, length = av;
    const int ok = det > 0;
    if (ok) { sdet = sqrt(det); length = av - sdet; }
    d->actuator_length[a] = length * gear[0];
    real dldv[3], dlda[3];
    for (int i = 0; i < 3; i++) {
      if (ok) {
        const real sc = 1 - safe_div(av, sdet);
        dldv[i] = axis[i] * sc + safe_div(vec[i], sdet);
        dlda[i] = vec[i] * sc;
      } else {
        dldv[i] = axis[i];
        dlda[i] = vec[i];
      }
    }
    int da1 = last_dof(m, m->body_weldid[m->site_bodyid[id]]), da2 = last_dof(m, m->body_weldid[m->site_bodyid[id2]]);
    while (da1 >= 0 || da2 >= 0) {
      const int da = da1 > da2 ? da1 : da2;
      real jacA[3], jac[3];
      jac_dof(m, d, sx2, m->site_bodyid[id2], da, jp2, jr2);
      cross3(jacA, jr2, axis);
      jac_dof(m, d, sx, m->site_bodyid[id], da, jp, jr);
      for (int i = 0; i < 3; i++) jac[i] = jp[i] - jp2[i];
      mom[da] = (dot3(dlda, jacA) + dot3(dldv, jac)) * gear[0];
      if (da1 == da) da1 = m->dof_parentid[da1];
      if (da2 == da) da2 = m->dof_parentid[da2];
    }
    return;
  }
  if (id2 < 0) { /* wrench in the global frame */
    const real* sm = d->site_xmat + 9 * id;
    real wt[3], wr[3];
    r_vec(wt, sm, gear);
    r_vec(wr, sm, gear + 3);
    d->actuator_length[a] = 0;
    for (int da = last_dof(m, m->body_weldid[m->site_bodyid[id]]); da >= 0; da = m->dof_parentid[da]) {
      jac_dof(m, d, sx, m->site_bodyid[id], da, jp, jr);
      mom[da] = dot3(jp, wt) + dot3(jr, wr);
    }
    return;
  }
  const int body = m->site_bodyid[id], bref = m->site_bodyid[id2];
  const real *rx = d->site_xpos + 3 * id2, *rm = d->site_xmat + 9 * id2;
  const int tr = gear[0] != 0 || gear[1] != 0 || gear[2] != 0, rot = gear[3] != 0 || gear[4] != 0 || gear[5] != 0;
  real length = 0, wt[3] = {0, 0, 0}, wr[3] = {0, 0, 0};
  if (tr) {
    real dx[3] = {sx[0] - rx[0], sx[1] - rx[1], sx[2] - rx[2]}, vec[3];
    rt_vec(vec, rm, dx);
    length += dot3(vec, gear);
    r_vec(wt, rm, gear);
  }
  if (rot) {
    real q[4], qr[4], vec[3];
    mul_quat(q, m->site_quat + 4 * id, d->xquat + 4 * body); /* smooth.py:2375-2376 multiplies in this order */
    mul_quat(qr, m->site_quat + 4 * id2, d->xquat + 4 * bref);
    quat_sub(vec, q, qr);
    length += dot3(vec, gear + 3);
    r_vec(wr, rm, gear + 3);
  }
  d->actuator_length[a] = length;
  int da1 = last_dof(m, m->body_weldid[body]), da2 = last_dof(m, m->body_weldid[bref]);
  while (da1 >= 0 || da2 >= 0) {
    const int da = da1 > da2 ? da1 : da2;
    if (da1 == da && da2 == da) break;
    jac_dof(m, d, sx, body, da, jp, jr);
    jac_dof(m, d, rx, bref, da, jp2, jr2);
    real v = 0;
    for (int i = 0; i < 3; i++) {
      if (tr) v += (jp[i] - jp2[i]) * wt[i];
      if (rot) v += (jr[i] - jr2[i]) * wr[i];
    }
    mom[da] = v;
    if (da1 == da) da1 = m->dof_parentid[da1];
    if (da2 == da) da2 = m->dof_parentid[da2];
  }
}

/* smooth.py:2260-2273, 2448-2602 (BODY, adhesion): minus the mean over the body's contacts of the normal
 * direction's Jacobian -- the contact's constraint rows when it is active (pyramid rows weighted 1/(2 npyr)
 * each, i.e. their mean), else normal . (J(pos, b2) - J(pos, b1)) -- zero without contacts */
static void body_transmission(const orc_model* m, orc_data* d, int a, real* mom) {
  const int body = m->actuator_trnid[2 * a], nv = m->nv;
  int ncon = 0;
  d->actuator_length[a] = 0;
  for (int c = 0; c < d->ncon[0]; c++) {
    const int g1 = d->con_geom[2 * c], g2 = d->con_geom[2 * c + 1];
    if (g1 < 0 || g2 < 0) continue;
    const int b1 = m->geom_bodyid[g1], b2 = m->geom_bodyid[g2];
    if (b1 != body && b2 != body) continue;
    ncon++;
    if (d->con_dist[c] < d->con_includemargin[c]) {
      const int dim = d->con_dim[c];
      const int* adr = d->con_efc_address + (size_t)c * 10;
      if (dim == 1 || m->opt_cone == 1) {
        for (int i = 0; i < nv; i++) mom[i] += d->efc_J[(size_t)adr[0] * nv + i];
      } else {
        const int np = dim - 1;
        for (int j = 0; j < 2 * np; j++)
          for (int i = 0; i < nv; i++) mom[i] += d->efc_J[(size_t)adr[j] * nv + i] * (0.5 / np);
      }
    } else {
      const real* pos = d->con_pos + 3 * c;
      const real* n = d->con_frame + 9 * c;
      for (int i = 0; i < nv; i++) {
        real j1[3], j2[3], r[3];
        jac_dof(m, d, pos, b1, i, j1, r);
        jac_dof(m, d, pos, b2, i, j2, r);
        mom[i] += n[0] * (j2[0] - j1[0]) + n[1] * (j2[1] - j1[1]) + n[2] * (j2[2] - j1[2]);
      }
    }
  }
  if (ncon > 0)
    for (int i = 0; i < nv; i++) mom[i] /= -(real)ncon;
}

static void transmission(const orc_model* m, orc_data* d) {
  int nv = m->nv;
  memset(d->actuator_moment, 0, (size_t)m->nu * nv * sizeof(real));
  for (int a = 0; a < m->nu; a++) {
    const real* gear = m->actuator_gear + 6 * a;
    int trn = m->actuator_trntype[a];
    real* mom = d->actuator_moment + (size_t)a * nv;
    if (trn == TRN_TENDON) {
      /* smooth.py:2244-2260: length = ten_length gear0, moment = gear0 ten_J */
      const int t = m->actuator_trnid[2 * a];
      d->actuator_length[a] = d->ten_length[t] * gear[0];
      for (int k = 0; k < m->ten_J_rownnz[t]; k++)
        mom[m->ten_J_colind[m->ten_J_rowadr[t] + k]] = d->ten_J[m->ten_J_rowadr[t] + k] * gear[0];
      continue;
    }
    if (trn == TRN_SITE || trn == TRN_SLIDERCRANK) {
      site_transmission(m, d, a, mom);
      continue;
    }
    if (trn == TRN_BODY) {
      body_transmission(m, d, a, mom);
      continue;
    }
    if (trn == TRN_JOINT || trn == TRN_JOINTINPARENT) {
      int j = m->actuator_trnid[2 * a];
      int jt = m->jnt_type[j], qa = m->jnt_qposadr[j], va = m->jnt_dofadr[j];
      if (jt == JNT_FREE) {
        d->actuator_length[a] = 0;
        if (trn == TRN_JOINTINPARENT) {
          real q[4] = {d->qpos[qa + 3], d->qpos[qa + 4], d->qpos[qa + 5], d->qpos[qa + 6]}, qn[4], ga[3];
          normalize4(q);
          qn[0] = q[0]; qn[1] = -q[1]; qn[2] = -q[2]; qn[3] = -q[3];
          rot_vec_quat(ga, gear + 3, qn);
          for (int i = 0; i < 3; i++) { mom[va + i] = gear[i]; mom[va + 3 + i] = ga[i]; }
        } else {
          for (int i = 0; i < 6; i++) mom[va + i] = gear[i];
        }
      } else if (jt == JNT_BALL) {
        real q[4] = {d->qpos[qa], d->qpos[qa + 1], d->qpos[qa + 2], d->qpos[qa + 3]}, aa[3];
        normalize4(q);
        quat_to_vel(aa, q);
        real ga[3] = {gear[0], gear[1], gear[2]};
        if (trn == TRN_JOINTINPARENT) {
          real qn[4] = {q[0], -q[1], -q[2], -q[3]};
          rot_vec_quat(ga, ga, qn);
        }
        d->actuator_length[a] = dot3(aa, ga);
        for (int i = 0; i < 3; i++) mom[va + i] = ga[i];
      } else {
        d->actuator_length[a] = d->qpos[qa] * gear[0];
        mom[va] = gear[0];
      }
    }
  }
}

/* smooth.py:1935-2038 (com_vel) */
static void com_vel(const orc_model* m, orc_data* d) {
  memset(d->cvel, 0, 6 * sizeof(real));
  memset(d->cdof_dot, 0, (size_t)m->nv * 6 * sizeof(real));
  for (int b = 1; b < m->nbody; b++) {
    int p = m->body_parentid[b];
    real cvel[6];
    memcpy(cvel, d->cvel + 6 * p, sizeof(cvel));
    int dofid = m->body_dofadr[b];
    for (int j = m->body_jntadr[b]; j < m->body_jntadr[b] + m->body_jntnum[b]; j++) {
      int jt = m->jnt_type[j];
      const real* cd = d->cdof;
      if (jt == JNT_FREE) {
        for (int k = 0; k < 3; k++)
          for (int i = 0; i < 6; i++) cvel[i] += cd[6 * (dofid + k) + i] * d->qvel[dofid + k];
        for (int k = 3; k < 6; k++) motion_cross(d->cdof_dot + 6 * (dofid + k), cvel, cd + 6 * (dofid + k));
        for (int k = 3; k < 6; k++)
          for (int i = 0; i < 6; i++) cvel[i] += cd[6 * (dofid + k) + i] * d->qvel[dofid + k];
        dofid += 6;
      } else if (jt == JNT_BALL) {
        for (int k = 0; k < 3; k++) motion_cross(d->cdof_dot + 6 * (dofid + k), cvel, cd + 6 * (dofid + k));
        for (int k = 0; k < 3; k++)
          for (int i = 0; i < 6; i++) cvel[i] += cd[6 * (dofid + k) + i] * d->qvel[dofid + k];
        dofid += 3;
      } else {
        motion_cross(d->cdof_dot + 6 * dofid, cvel, cd + 6 * dofid);
        for (int i = 0; i < 6; i++) cvel[i] += cd[6 * dofid + i] * d->qvel[dofid];
        dofid += 1;
      }
    }
    memcpy(d->cvel + 6 * b, cvel, sizeof(cvel));
  }
}

/* smooth.py:1112-1274 (rne, flg_acc = False) */
static void rne(const orc_model* m, orc_data* d) {
  int nb = m->nbody;
  real* cacc = d->cacc;
  memset(cacc, 0, 6 * sizeof(real));
  if (!(m->opt_disableflags & DSBL_GRAVITY))
    for (int i = 0; i < 3; i++) cacc[3 + i] = -m->opt_gravity[i];
  for (int b = 1; b < nb; b++) {
    int p = m->body_parentid[b];
    real acc[6];
    memcpy(acc, cacc + 6 * p, sizeof(acc));
    for (int k = 0; k < m->body_dofnum[b]; k++) {
      int dof = m->body_dofadr[b] + k;
      for (int i = 0; i < 6; i++) acc[i] += d->cdof_dot[6 * dof + i] * d->qvel[dof];
    }
    memcpy(cacc + 6 * b, acc, sizeof(acc));
  }
  real* cfrc = d->cfrc_int;
  memset(cfrc, 0, 6 * sizeof(real));
  for (int b = 1; b < nb; b++) {
    real f1[6], iv[6], f2[6];
    inert_vec(f1, d->cinert + 10 * b, cacc + 6 * b);
    inert_vec(iv, d->cinert + 10 * b, d->cvel + 6 * b);
    motion_cross_force(f2, d->cvel + 6 * b, iv);
    for (int i = 0; i < 6; i++) cfrc[6 * b + i] = f1[i] + f2[i];
  }
  for (int b = nb - 1; b > 0; b--) {
    int p = m->body_parentid[b];
    for (int i = 0; i < 6; i++) cfrc[6 * p + i] += cfrc[6 * b + i];
  }
  for (int i = 0; i < m->nv; i++) {
    int b = m->dof_bodyid[i];
    real s = 0;
    for (int k = 0; k < 6; k++) s += d->cdof[6 * i + k] * cfrc[6 * b + k];
    d->qfrc_bias[i] = s;
  }
}

/* support.py:174-216 apply_ft (flg_add = False): qfrc = sum over bodies of J(xipos_b)^T (f_b, t_b);
   ft: (nbody, 6) = (force, torque) per body */
static void apply_ft(const orc_model* m, const orc_data* d, const real* ft, real* qfrc) {
  for (int i = 0; i < m->nv; i++) {
    const real* cd = d->cdof + 6 * i;
    const int db = m->dof_bodyid[i];
    real acc = 0;
    for (int b = db; b < m->nbody; b++) {
      const real* f = ft + 6 * b;
      if (f[0] == 0 && f[1] == 0 && f[2] == 0 && f[3] == 0 && f[4] == 0 && f[5] == 0) continue;
      int p = b;
      while (p != 0 && p != db) p = m->body_parentid[p];
      if (p == 0) continue;
      real off[3], c[3];
      for (int k = 0; k < 3; k++) off[k] = d->xipos[3 * b + k] - d->subtree_com[3 * m->body_rootid[b] + k];
      cross3(c, cd, off);
      acc += cd[3] * f[0] + cd[4] * f[1] + cd[5] * f[2] + cd[0] * f[3] + cd[1] * f[4] + cd[2] * f[5] + dot3(c, f);
    }
    qfrc[i] = acc;
  }
}

/* passive.py:246-272 _gravity_force: f_b = -gravity * mass_b * gravcomp_b at xipos_b */
static void gravcomp(const orc_model* m, orc_data* d, real* ft) {
  memset(ft, 0, 6 * m->nbody * sizeof(real));
  for (int b = 1; b < m->nbody; b++) {
    const real gc = m->body_gravcomp[b];
    if (gc == 0) continue;
    for (int k = 0; k < 3; k++) ft[6 * b + k] = -m->opt_gravity[k] * m->body_mass[b] * gc;
  }
  apply_ft(m, d, ft, d->qfrc_gravcomp);
}

/* R^T v and R v for a row-major R (world from local) */
static void rt_vec(real* r, const real* R, const real* v) {
  for (int i = 0; i < 3; i++) r[i] = R[i] * v[0] + R[3 + i] * v[1] + R[6 + i] * v[2];
}
static void r_vec(real* r, const real* R, const real* v) {
  for (int i = 0; i < 3; i++) r[i] = R[3 * i] * v[0] + R[3 * i + 1] * v[1] + R[3 * i + 2] * v[2];
}
static real pow4r(real x) { return x * x * x * x; }

#include "oracle_tendon.h"

/* passive.py:42-59 */
static void fluid_semiaxes(int type, const real* size, real* s) {
  if (type == GEOM_SPHERE) { s[0] = s[1] = s[2] = size[0]; }
  else if (type == GEOM_CAPSULE) { s[0] = s[1] = size[0]; s[2] = size[1] + size[0]; }
  else if (type == GEOM_CYLINDER) { s[0] = s[1] = size[0]; s[2] = size[1]; }
  else { s[0] = size[0]; s[1] = size[1]; s[2] = size[2]; }
}

/* passive.py:276-500 _fluid_force (ellipsoid model per geom with geom_fluid[0] > 0, else the body's
   equivalent inertia box), then support.apply_ft into qfrc_fluid (passive.py:503-532) */
static void fluid(const orc_model* m, orc_data* d, real* ft) {
  const real PI = 3.14159265358979323846;
  const real rho = m->opt_density, mu = m->opt_viscosity;
  const real* wind = m->opt_wind;
  memset(ft, 0, 6 * m->nbody * sizeof(real));
  for (int b = 1; b < m->nbody; b++) {
    const real mass = m->body_mass[b];
    if (mass < MINVAL) continue;
    const real* xipos = d->xipos + 3 * b;
    const real* R = d->ximat + 9 * b;
    const real* ang = d->cvel + 6 * b;
    const real* root = d->subtree_com + 3 * m->body_rootid[b];
    real off[3] = {xipos[0] - root[0], xipos[1] - root[1], xipos[2] - root[2]}, c[3], lin_com[3];
    cross3(c, off, ang);
    for (int k = 0; k < 3; k++) lin_com[k] = d->cvel[6 * b + 3 + k] - c[k];
    real F[3] = {0, 0, 0}, T[3] = {0, 0, 0};
    if (m->body_fluid_ellipsoid[b]) {
      for (int g = m->body_geomadr[b]; g < m->body_geomadr[b] + m->body_geomnum[b]; g++) {
        const real* fl = m->geom_fluid + 12 * g;
        if (fl[0] <= 0) continue;
        real s[3];
        fluid_semiaxes(m->geom_type[g], m->geom_size + 3 * g, s);
        const real* G = d->geom_xmat + 9 * g;
        real dp[3], lp[3], w[3], la[3], ll[3];
        for (int k = 0; k < 3; k++) dp[k] = d->geom_xpos[3 * g + k] - xipos[k];
        cross3(c, ang, dp);
        for (int k = 0; k < 3; k++) lp[k] = lin_com[k] + c[k];
        rt_vec(la, G, ang);
        rt_vec(ll, G, lp);
        rt_vec(w, G, wind);
        for (int k = 0; k < 3; k++) ll[k] -= w[k];
        real tq[3] = {0, 0, 0}, fo[3] = {0, 0, 0};
        if (rho > 0) {  /* added mass */
          real vl[3], va[3], a[3];
          for (int k = 0; k < 3; k++) { vl[k] = rho * fl[6 + k] * ll[k]; va[k] = rho * fl[9 + k] * la[k]; }
          cross3(a, vl, la);
          for (int k = 0; k < 3; k++) fo[k] += a[k];
          cross3(a, vl, ll);
          for (int k = 0; k < 3; k++) tq[k] += a[k];
          cross3(a, va, la);
          for (int k = 0; k < 3; k++) tq[k] += a[k];
        }
        const real vol = 4.0 / 3.0 * PI * s[0] * s[1] * s[2];
        const real dmax = maxr(maxr(s[0], s[1]), s[2]), dmin = minr(minr(s[0], s[1]), s[2]);
        const real dmid = s[0] + s[1] + s[2] - dmax - dmin, Amax = PI * dmax * dmid;
        const real speed = sqrt(dot3(ll, ll));
        real magnus[3];
        cross3(magnus, la, ll);
        for (int k = 0; k < 3; k++) magnus[k] *= fl[5] * rho * vol;
        const real s12 = s[1] * s[2], s20 = s[2] * s[0], s01 = s[0] * s[1];
        const real den = pow4r(s12) * ll[0] * ll[0] + pow4r(s20) * ll[1] * ll[1] + pow4r(s01) * ll[2] * ll[2];
        const real num = s12 * ll[0] * s12 * ll[0] + s20 * ll[1] * s20 * ll[1] + s01 * ll[2] * s01 * ll[2];
        real Aproj = 0, cosa = 0;
        if (num > MINVAL && den > MINVAL) {
          Aproj = PI * sqrt(den / maxr(MINVAL, num));
          if (speed > MINVAL) cosa = num / maxr(MINVAL, speed * den);
        }
        const real nrm[3] = {s12 * s12 * ll[0], s20 * s20 * ll[1], s01 * s01 * ll[2]};
        real kutta[3] = {0, 0, 0};
        if (rho > 0 && fl[4] != 0 && speed > MINVAL) {
          real circ[3];
          cross3(circ, nrm, ll);
          for (int k = 0; k < 3; k++) circ[k] *= fl[4] * rho * cosa * Aproj;
          cross3(kutta, circ, ll);
        }
        const real D = 2.0 / 3.0 * (s[0] + s[1] + s[2]);
        const real Imax = 8.0 / 15.0 * PI * dmid * pow4r(dmax);
        real mv[3];
        for (int k = 0; k < 3; k++) {
          const real II = 8.0 / 15.0 * PI * s[k] * pow4r(maxr(s[(k + 1) % 3], s[(k + 2) % 3]));
          mv[k] = la[k] * (fl[3] * II + fl[2] * (Imax - II));
        }
        const real dlin = mu * 3.0 * PI * D + rho * speed * (Aproj * fl[1] + fl[2] * (Amax - Aproj));
        const real dang = mu * PI * D * D * D + rho * sqrt(dot3(mv, mv));
        for (int k = 0; k < 3; k++) {
          tq[k] = (tq[k] - dang * la[k]) * fl[0];
          fo[k] = (fo[k] + magnus[k] + kutta[k] - dlin * ll[k]) * fl[0];
        }
        real wt[3], wf[3];
        r_vec(wt, G, tq);
        r_vec(wf, G, fo);
        for (int k = 0; k < 3; k++) { T[k] += wt[k]; F[k] += wf[k]; }
      }
    } else {
      real la[3], ll[3], w[3];
      rt_vec(la, R, ang);
      rt_vec(ll, R, lin_com);
      rt_vec(w, R, wind);
      for (int k = 0; k < 3; k++) ll[k] -= w[k];
      real tq[3] = {0, 0, 0}, fo[3] = {0, 0, 0};
      if (mu > 0 || rho > 0) {
        const real* I = m->body_inertia + 3 * b;
        const real box[3] = {sqrt(maxr(MINVAL, I[1] + I[2] - I[0]) * 6 / mass), sqrt(maxr(MINVAL, I[0] + I[2] - I[1]) * 6 / mass),
                             sqrt(maxr(MINVAL, I[0] + I[1] - I[2]) * 6 / mass)};
        if (mu > 0) {
          const real diam = (box[0] + box[1] + box[2]) / 3;
          for (int k = 0; k < 3; k++) { tq[k] = -la[k] * diam * diam * diam * PI * mu; fo[k] = -3 * ll[k] * diam * PI * mu; }
        }
        if (rho > 0) {
          for (int k = 0; k < 3; k++) {
            const int i1 = (k + 1) % 3, i2 = (k + 2) % 3;
            fo[k] -= 0.5 * rho * box[i1] * box[i2] * fabs(ll[k]) * ll[k];
            tq[k] -= box[k] * (pow4r(box[i1]) + pow4r(box[i2])) * fabs(la[k]) * la[k] * rho / 64;
          }
        }
      }
      r_vec(T, R, tq);
      r_vec(F, R, fo);
    }
    for (int k = 0; k < 3; k++) { ft[6 * b + k] = F[k]; ft[6 * b + 3 + k] = T[k]; }
  }
  apply_ft(m, d, ft, d->qfrc_fluid);
}

/* passive.py:728-872 (spring / damper :70-179, tendons :183-252, flex, gravcomp, fluid, _qfrc_passive :535-563) */
static void passive(const orc_model* m, orc_data* d) {
  int nv = m->nv;
  int dsbl_spring = m->opt_disableflags & DSBL_SPRING, dsbl_damper = m->opt_disableflags & DSBL_DAMPER;
  memset(d->qfrc_spring, 0, nv * sizeof(real));
  memset(d->qfrc_damper, 0, nv * sizeof(real));
  memset(d->qfrc_gravcomp, 0, nv * sizeof(real));
  memset(d->qfrc_fluid, 0, nv * sizeof(real));
  if (dsbl_spring && dsbl_damper) { memset(d->qfrc_passive, 0, nv * sizeof(real)); return; }
  for (int j = 0; j < m->njnt; j++) {
    int da = m->jnt_dofadr[j], qa = m->jnt_qposadr[j], jt = m->jnt_type[j];
    real stiff = m->jnt_stiffness[j], damp = m->dof_damping[da];
    int has_s = stiff != 0 && !dsbl_spring, has_d = damp != 0 && !dsbl_damper;
    if (jt == JNT_FREE) {
      if (has_s) {
        for (int i = 0; i < 3; i++) d->qfrc_spring[da + i] = -stiff * (d->qpos[qa + i] - m->qpos_spring[qa + i]);
        real rot[4] = {d->qpos[qa + 3], d->qpos[qa + 4], d->qpos[qa + 5], d->qpos[qa + 6]}, dif[3];
        normalize4(rot);
        quat_sub(dif, rot, m->qpos_spring + qa + 3);
        for (int i = 0; i < 3; i++) d->qfrc_spring[da + 3 + i] = -stiff * dif[i];
      }
      if (has_d)
        for (int i = 0; i < 6; i++) d->qfrc_damper[da + i] = -damp * d->qvel[da + i];
    } else if (jt == JNT_BALL) {
      if (has_s) {
        real rot[4] = {d->qpos[qa], d->qpos[qa + 1], d->qpos[qa + 2], d->qpos[qa + 3]}, dif[3];
        normalize4(rot);
        quat_sub(dif, rot, m->qpos_spring + qa);
        for (int i = 0; i < 3; i++) d->qfrc_spring[da + i] = -stiff * dif[i];
      }
      if (has_d)
        for (int i = 0; i < 3; i++) d->qfrc_damper[da + i] = -damp * d->qvel[da + i];
    } else {
      if (has_s) d->qfrc_spring[da] = -stiff * (d->qpos[qa] - m->qpos_spring[qa]);
      if (has_d) d->qfrc_damper[da] = -damp * d->qvel[da];
    }
  }
  /* passive.py:183-252: tendon spring (dead band between lengthspring[0] and [1]) and damper */
  for (int t = 0; t < m->ntendon; t++) {
    const real k = m->tendon_stiffness[t], b = m->tendon_damping[t];
    const int has_s = k != 0 && !dsbl_spring, has_d = b != 0 && !dsbl_damper;
    if (!has_s && !has_d) continue;
    const real L = d->ten_length[t], lo = m->tendon_lengthspring[2 * t], hi = m->tendon_lengthspring[2 * t + 1];
    const real fs = L > hi ? k * (hi - L) : (L < lo ? k * (lo - L) : 0);
    const real fd = -b * d->ten_velocity[t];
    for (int q = 0; q < m->ten_J_rownnz[t]; q++) {
      const int e = m->ten_J_rowadr[t] + q, i = m->ten_J_colind[e];
      if (has_s) d->qfrc_spring[i] += d->ten_J[e] * fs;
      if (has_d) d->qfrc_damper[i] += d->ten_J[e] * fd;
    }
  }
  if (!dsbl_spring) flex_passive(m, d);
  const int gc = m->ngravcomp && !(m->opt_disableflags & DSBL_GRAVITY);
  if (gc || m->has_fluid) {
    real* ft = (real*)malloc(6 * m->nbody * sizeof(real));
    if (gc) gravcomp(m, d, ft);
    if (m->has_fluid) fluid(m, d, ft);
    free(ft);
  }
  for (int i = 0; i < nv; i++) {
    d->qfrc_passive[i] = d->qfrc_spring[i] + d->qfrc_damper[i];
    if (gc && !m->jnt_actgravcomp[m->dof_jntid[i]]) d->qfrc_passive[i] += d->qfrc_gravcomp[i];
    if (m->has_fluid) d->qfrc_passive[i] += d->qfrc_fluid[i];
  }
}

/* =============================================================================================
 * collision (collision_driver.py, collision_core.py, collision_primitive*.py)
 * ============================================================================================= */
typedef struct {
  real dist[2];
  real pos[2][3];
  real frame[2][9];
  int n;
} contacts2;

/* collision_driver.py:90-103 */
static int plane_filter(real size1, real size2, real margin1, real margin2, const real* xpos1, const real* xpos2,
                        const real* xmat1, const real* xmat2) {
  if (size1 == 0) {
    real dif[3] = {xpos2[0] - xpos1[0], xpos2[1] - xpos1[1], xpos2[2] - xpos1[2]};
    real n[3] = {xmat1[2], xmat1[5], xmat1[8]};
    return dot3(dif, n) <= size2 + margin1 + margin2;
  } else if (size2 == 0) {
    real dif[3] = {xpos1[0] - xpos2[0], xpos1[1] - xpos2[1], xpos1[2] - xpos2[2]};
    real n[3] = {xmat2[2], xmat2[5], xmat2[8]};
    return dot3(dif, n) <= size1 + margin1 + margin2;
  }
  return 1;
}

/* collision_driver.py:106-111 */
static int sphere_filter(real size1, real size2, real margin1, real margin2, const real* xpos1, const real* xpos2) {
  real bound = size1 + size2 + margin1 + margin2;
  real dif[3] = {xpos2[0] - xpos1[0], xpos2[1] - xpos1[1], xpos2[2] - xpos1[2]};
  return dot3(dif, dif) <= bound * bound;
}

static void matvec3(real* r, const real* M, const real* v) {
  real t[3];
  for (int i = 0; i < 3; i++) t[i] = M[3 * i] * v[0] + M[3 * i + 1] * v[1] + M[3 * i + 2] * v[2];
  r[0] = t[0]; r[1] = t[1]; r[2] = t[2];
}

/* collision_driver.py:116-213 */
static int aabb_filter(const real* c1, const real* c2, const real* s1, const real* s2, real m1, real m2, const real* xp1,
                       const real* xp2, const real* xm1, const real* xm2) {
  real cen1[3], cen2[3];
  matvec3(cen1, xm1, c1); matvec3(cen2, xm2, c2);
  for (int i = 0; i < 3; i++) { cen1[i] += xp1[i]; cen2[i] += xp2[i]; }
  real margin = m1 + m2;
  real mx1[3] = {-MAXVAL, -MAXVAL, -MAXVAL}, mn1[3] = {MAXVAL, MAXVAL, MAXVAL};
  real mx2[3] = {-MAXVAL, -MAXVAL, -MAXVAL}, mn2[3] = {MAXVAL, MAXVAL, MAXVAL};
  real sgn[2] = {-1, 1};
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 2; j++)
      for (int k = 0; k < 2; k++) {
        real cr1[3] = {sgn[i] * s1[0], sgn[j] * s1[1], sgn[k] * s1[2]}, p1[3];
        real cr2[3] = {sgn[i] * s2[0], sgn[j] * s2[1], sgn[k] * s2[2]}, p2[3];
        matvec3(p1, xm1, cr1); matvec3(p2, xm2, cr2);
        for (int a = 0; a < 3; a++) {
          if (p1[a] > mx1[a]) mx1[a] = p1[a];
          if (p1[a] < mn1[a]) mn1[a] = p1[a];
          if (p2[a] > mx2[a]) mx2[a] = p2[a];
          if (p2[a] < mn2[a]) mn2[a] = p2[a];
        }
      }
  for (int a = 0; a < 3; a++) {
    if (cen1[a] + mx1[a] + margin < cen2[a] + mn2[a]) return 0;
    if (cen2[a] + mx2[a] + margin < cen1[a] + mn1[a]) return 0;
  }
  return 1;
}

/* collision_driver.py:217-271 */
static int obb_filter(const real* c1, const real* c2, const real* s1, const real* s2, real m1, real m2, const real* xp1,
                      const real* xp2, const real* xm1, const real* xm2) {
  real margin = m1 + m2;
  real xc[2][3], nrm[6][3];
  matvec3(xc[0], xm1, c1); matvec3(xc[1], xm2, c2);
  for (int i = 0; i < 3; i++) { xc[0][i] += xp1[i]; xc[1][i] += xp2[i]; }
  for (int k = 0; k < 3; k++)
    for (int i = 0; i < 3; i++) { nrm[k][i] = xm1[3 * i + k]; nrm[3 + k][i] = xm2[3 * i + k]; }
  for (int j = 0; j < 2; j++)
    for (int k = 0; k < 3; k++) {
      real proj[2], radius[2];
      for (int i = 0; i < 2; i++) {
        proj[i] = dot3(xc[i], nrm[3 * j + k]);
        const real* size = i == 0 ? s1 : s2;
        radius[i] = fabs(size[0] * dot3(nrm[3 * i + 0], nrm[3 * j + k])) + fabs(size[1] * dot3(nrm[3 * i + 1], nrm[3 * j + k])) +
                    fabs(size[2] * dot3(nrm[3 * i + 2], nrm[3 * j + k]));
      }
      if (radius[0] + radius[1] + margin < fabs(proj[1] - proj[0])) return 0;
    }
  return 1;
}

/* collision_driver.py:274-321 */
static int broadphase_filter(const orc_model* m, const orc_data* d, int g1, int g2) {
  int filt = m->opt_broadphase_filter;
  const real *c1 = m->geom_aabb + 6 * g1, *c2 = m->geom_aabb + 6 * g2;
  const real *s1 = c1 + 3, *s2 = c2 + 3;
  real rb1 = m->geom_rbound[g1], rb2 = m->geom_rbound[g2];
  real mg1 = m->geom_margin[g1], mg2 = m->geom_margin[g2];
  const real *xp1 = d->geom_xpos + 3 * g1, *xp2 = d->geom_xpos + 3 * g2;
  const real *xm1 = d->geom_xmat + 9 * g1, *xm2 = d->geom_xmat + 9 * g2;
  if (rb1 == 0 || rb2 == 0) {
    if (filt & FILTER_PLANE) return plane_filter(rb1, rb2, mg1, mg2, xp1, xp2, xm1, xm2);
  } else {
    if (filt & FILTER_SPHERE)
      if (!sphere_filter(rb1, rb2, mg1, mg2, xp1, xp2)) return 0;
    if (filt & FILTER_AABB)
      if (!aabb_filter(c1, c2, s1, s2, mg1, mg2, xp1, xp2, xm1, xm2)) return 0;
    if (filt & FILTER_OBB)
      if (!obb_filter(c1, c2, s1, s2, mg1, mg2, xp1, xp2, xm1, xm2)) return 0;
  }
  return 1;
}

/* collision_primitive_core.py:106-111 */
static real plane_sphere(real* pos, const real* n, const real* ppos, const real* spos, real r) {
  real dif[3] = {spos[0] - ppos[0], spos[1] - ppos[1], spos[2] - ppos[2]};
  real dist = dot3(dif, n) - r;
  for (int i = 0; i < 3; i++) pos[i] = spos[i] - n[i] * (r + (real)0.5 * dist);
  return dist;
}

/* collision_primitive_core.py:114-143 */
static real sphere_sphere(real* pos, real* n, const real* p1, real r1, const real* p2, real r2) {
  real dir[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  real dist = sqrt(dot3(dir, dir));
  if (dist == 0) { n[0] = 1; n[1] = 0; n[2] = 0; }
  else { n[0] = dir[0] / dist; n[1] = dir[1] / dist; n[2] = dir[2] / dist; }
  dist = dist - (r1 + r2);
  for (int i = 0; i < 3; i++) pos[i] = p1[i] + n[i] * (r1 + (real)0.5 * dist);
  return dist;
}

/* collision_primitive_core.py:146-178 */
static real sphere_capsule(real* pos, real* n, const real* spos, real sr, const real* cpos, const real* axis, real cr, real chl) {
  real a[3], b[3], pt[3];
  for (int i = 0; i < 3; i++) { a[i] = cpos[i] - axis[i] * chl; b[i] = cpos[i] + axis[i] * chl; }
  closest_segment_point(pt, a, b, spos);
  return sphere_sphere(pos, n, spos, sr, pt, cr);
}

/* collision_primitive_core.py:181-308 */
static void capsule_capsule(contacts2* out, const real* p1, const real* ax1, real r1, real hl1, const real* p2, const real* ax2,
                            real r2, real hl2, real margin) {
  real axis1[3], axis2[3], dif[3];
  for (int i = 0; i < 3; i++) { axis1[i] = ax1[i] * hl1; axis2[i] = ax2[i] * hl2; dif[i] = p1[i] - p2[i]; }
  real ma = dot3(axis1, axis1), mb = -dot3(axis1, axis2), mc = dot3(axis2, axis2);
  real u = -dot3(axis1, dif), v = dot3(axis2, dif);
  real det = ma * mc - mb * mb;
  out->n = 0;
  out->dist[0] = out->dist[1] = INFINITY;
  real v1[3], v2[3], pos[3], nrm[3];
  if (fabs(det) >= MINVAL) {
    real inv = 1 / det;
    real x1 = (mc * u - mb * v) * inv, x2 = (ma * v - mb * u) * inv;
    if (x1 > 1) { x1 = 1; x2 = (v - mb) / mc; }
    else if (x1 < -1) { x1 = -1; x2 = (v + mb) / mc; }
    if (x2 > 1) { x2 = 1; x1 = clampr((u - mb) / ma, -1, 1); }
    else if (x2 < -1) { x2 = -1; x1 = clampr((u + mb) / ma, -1, 1); }
    for (int i = 0; i < 3; i++) { v1[i] = p1[i] + axis1[i] * x1; v2[i] = p2[i] + axis2[i] * x2; }
    real dist = sphere_sphere(pos, nrm, v1, r1, v2, r2);
    if (dist <= margin) {
      out->dist[0] = dist;
      memcpy(out->pos[0], pos, sizeof(pos));
      make_frame(out->frame[0], nrm);
      out->n = 1;
    }
    return;
  }
  int cnt = 0;
  for (int t = 0; t < 4; t++) {
    if (t >= 2 && cnt >= 2) break;
    real x;
    if (t == 0) { for (int i = 0; i < 3; i++) v1[i] = p1[i] + axis1[i]; x = clampr((v - mb) / mc, -1, 1); for (int i = 0; i < 3; i++) v2[i] = p2[i] + axis2[i] * x; }
    else if (t == 1) { for (int i = 0; i < 3; i++) v1[i] = p1[i] - axis1[i]; x = clampr((v + mb) / mc, -1, 1); for (int i = 0; i < 3; i++) v2[i] = p2[i] + axis2[i] * x; }
    else if (t == 2) { for (int i = 0; i < 3; i++) v2[i] = p2[i] + axis2[i]; x = clampr((u - mb) / ma, -1, 1); for (int i = 0; i < 3; i++) v1[i] = p1[i] + axis1[i] * x; }
    else { for (int i = 0; i < 3; i++) v2[i] = p2[i] - axis2[i]; x = clampr((u + mb) / ma, -1, 1); for (int i = 0; i < 3; i++) v1[i] = p1[i] + axis1[i] * x; }
    real dist = sphere_sphere(pos, nrm, v1, r1, v2, r2);
    if (dist <= margin) {
      out->dist[cnt] = dist;
      memcpy(out->pos[cnt], pos, sizeof(pos));
      make_frame(out->frame[cnt], nrm);
      cnt++;
    }
  }
  out->n = cnt;
}

/* collision_primitive_core.py:311-361 */
static void plane_capsule(contacts2* out, const real* n, const real* ppos, const real* cpos, const real* axis, real r, real hl) {
  real b[3], tmp[3];
  real nd = dot3(n, axis);
  for (int i = 0; i < 3; i++) tmp[i] = axis[i] - n[i] * nd;
  real bn = normalize_with_norm(b, tmp);
  if (bn < 0.5) {
    if (-0.5 < n[1] && n[1] < 0.5) { b[0] = 0; b[1] = 1; b[2] = 0; }
    else { b[0] = 0; b[1] = 0; b[2] = 1; }
  }
  real c[3];
  cross3(c, n, b);
  real frame[9] = {n[0], n[1], n[2], b[0], b[1], b[2], c[0], c[1], c[2]};
  real e1[3], e2[3];
  for (int i = 0; i < 3; i++) { e1[i] = cpos[i] + axis[i] * hl; e2[i] = cpos[i] - axis[i] * hl; }
  out->dist[0] = plane_sphere(out->pos[0], n, ppos, e1, r);
  out->dist[1] = plane_sphere(out->pos[1], n, ppos, e2, r);
  memcpy(out->frame[0], frame, sizeof(frame));
  memcpy(out->frame[1], frame, sizeof(frame));
  out->n = 2;
}

/* collision_core.py:235-341: an explicit <pair> (pairid > -1) supplies every parameter (:270-277),
   otherwise the two geoms' parameters are mixed */
static void contact_params(const orc_model* m, int g1, int g2, int pairid, real* margin, real* gap, int* condim,
                           real* friction, real* solref, real* solreffriction, real* solimp) {
  if (pairid > -1) {
    *margin = m->pair_margin[pairid];
    *gap = m->pair_gap[pairid];
    *condim = m->pair_dim[pairid];
    for (int i = 0; i < 5; i++) friction[i] = maxr(MINMU, m->pair_friction[5 * pairid + i]);
    for (int i = 0; i < 2; i++) { solref[i] = m->pair_solref[2 * pairid + i]; solreffriction[i] = m->pair_solreffriction[2 * pairid + i]; }
    for (int i = 0; i < 5; i++) solimp[i] = m->pair_solimp[5 * pairid + i];
    return;
  }
  real s1 = m->geom_solmix[g1], s2 = m->geom_solmix[g2];
  int c1 = m->geom_condim[g1], c2 = m->geom_condim[g2];
  int p1 = m->geom_priority[g1], p2 = m->geom_priority[g2];
  real mix, fr[3];
  if (p1 > p2) { mix = 1; *condim = c1; memcpy(fr, m->geom_friction + 3 * g1, sizeof(fr)); }
  else if (p2 > p1) { mix = 0; *condim = c2; memcpy(fr, m->geom_friction + 3 * g2, sizeof(fr)); }
  else {
    mix = safe_div(s1, s1 + s2);
    if (s1 < MINVAL && s2 < MINVAL) mix = 0.5;
    else if (s1 < MINVAL && s2 >= MINVAL) mix = 0;
    else if (s1 >= MINVAL && s2 < MINVAL) mix = 1;
    *condim = c1 > c2 ? c1 : c2;
    for (int i = 0; i < 3; i++) fr[i] = maxr(m->geom_friction[3 * g1 + i], m->geom_friction[3 * g2 + i]);
  }
  friction[0] = fr[0]; friction[1] = fr[0]; friction[2] = fr[1]; friction[3] = fr[2]; friction[4] = fr[2];
  const real *sr1 = m->geom_solref + 2 * g1, *sr2 = m->geom_solref + 2 * g2;
  if (sr1[0] > 0 && sr2[0] > 0) {
    for (int i = 0; i < 2; i++) solref[i] = mix * sr1[i] + (1 - mix) * sr2[i];
  } else {
    for (int i = 0; i < 2; i++) solref[i] = minr(sr1[i], sr2[i]);
  }
  solreffriction[0] = solreffriction[1] = 0;
  for (int i = 0; i < 5; i++) solimp[i] = mix * m->geom_solimp[5 * g1 + i] + (1 - mix) * m->geom_solimp[5 * g2 + i];
  *margin = m->geom_margin[g1] + m->geom_margin[g2];
  *gap = m->geom_gap[g1] + m->geom_gap[g2];
  for (int i = 0; i < 5; i++) friction[i] = maxr(MINMU, friction[i]);
}

/* collision_driver.py:697-789 + collision_primitive.py:1300-1454 (+ write_contact collision_core.py:159-232) */
/* collision_primitive_core.py:395-443: corner k of the box against the plane */
static void plane_box_corner(int k, const real* n, const real* ppos, const real* bpos, const real* brot, const real* bsize,
                             real* dist, real* pos) {
  real dif[3] = {bpos[0] - ppos[0], bpos[1] - ppos[1], bpos[2] - ppos[2]};
  real center_dist = dot3(dif, n);
  real cl[3] = {(k & 1) ? bsize[0] : -bsize[0], (k & 2) ? bsize[1] : -bsize[1], (k & 4) ? bsize[2] : -bsize[2]};
  real corner[3];
  matvec3(corner, brot, cl);
  real cdist = center_dist + dot3(n, corner);
  *dist = cdist;
  for (int i = 0; i < 3; i++) pos[i] = corner[i] + bpos[i] - 0.5 * n[i] * cdist;
}


#include "oracle_ccd.h"

/* a mesh geom's vertices and polygon data (mesh_poly*) for the convex routines; meshid < 0: not a mesh */
static void ccd_geom_mesh(const orc_model* m, int meshid, ccd_geom* g) {
  if (meshid < 0) return;
  const int va = m->mesh_vertadr[meshid], pa = m->mesh_polyadr[meshid];
  g->vert = m->mesh_vert + 3 * va;
  g->nvert = m->mesh_vertnum[meshid];
  if (m->mesh_polynum[meshid] > 0) {
    g->pnormal = m->mesh_polynormal + 3 * pa;
    g->pvadr = m->mesh_polyvertadr + pa;
    g->pvnum = m->mesh_polyvertnum + pa;
    g->pvert = m->mesh_polyvert;
    g->pmapadr = m->mesh_polymapadr + va;
    g->pmapnum = m->mesh_polymapnum + va;
    g->pmap = m->mesh_polymap;
  }
}

/* collision_primitive_core.py:1103-1155 sphere_box */
static real sphere_box(real* pos, real* nrm, const real* spos, real r, const real* bpos, const real* brot, const real* bsize) {
  real dif[3] = {spos[0] - bpos[0], spos[1] - bpos[1], spos[2] - bpos[2]}, center[3], clamped[3], cdir[3], tmp[3];
  for (int i = 0; i < 3; i++) center[i] = brot[i] * dif[0] + brot[3 + i] * dif[1] + brot[6 + i] * dif[2];
  for (int i = 0; i < 3; i++) { clamped[i] = maxr(-bsize[i], minr(bsize[i], center[i])); tmp[i] = clamped[i] - center[i]; }
  real dist = normalize_with_norm(cdir, tmp);
  real lp[3], dst;
  if (dist <= MINVAL) {
    real closest = 2 * (bsize[0] + bsize[1] + bsize[2]);
    int k = 0;
    for (int i = 0; i < 6; i++) {
      real fd = fabs((i % 2 ? 1.0 : -1.0) * bsize[i / 2] - center[i / 2]);
      if (closest > fd) { closest = fd; k = i; }
    }
    real nearest[3] = {0, 0, 0};
    nearest[k / 2] = (k % 2) ? -1 : 1;
    for (int i = 0; i < 3; i++) lp[i] = center[i] + nearest[i] * (r - closest) / 2;
    matvec3(nrm, brot, nearest);
    dst = -closest - r;
  } else {
    for (int i = 0; i < 3; i++) lp[i] = 0.5 * (clamped[i] + center[i] + cdir[i] * r);
    matvec3(nrm, brot, cdir);
    dst = dist - r;
  }
  real w[3];
  matvec3(w, brot, lp);
  for (int i = 0; i < 3; i++) pos[i] = bpos[i] + w[i];
  return dst;
}

/* collision_primitive_core.py:1158-1480 capsule_box (MuJoCo's mjc_CapsuleBox): up to 2 contacts */
static void capsule_box(contacts2* out, const real* cpos, const real* cax, real cr, real chl, const real* bpos, const real* brot,
                        const real* bsize) {
  real dif[3] = {cpos[0] - bpos[0], cpos[1] - bpos[1], cpos[2] - bpos[2]}, pos[3], axis[3], ha[3];
  for (int i = 0; i < 3; i++) {
    pos[i] = brot[i] * dif[0] + brot[3 + i] * dif[1] + brot[6 + i] * dif[2];
    axis[i] = brot[i] * cax[0] + brot[3 + i] * cax[1] + brot[6 + i] * cax[2];
  }
  for (int i = 0; i < 3; i++) ha[i] = axis[i] * chl;
  int axisdir = (ha[0] > 0) + 2 * (ha[1] > 0) + 4 * (ha[2] > 0);
  real bestdist = 1e32, bestsegmentpos = -12;
  int cltype = -4, clface = -12;
  for (int i = -1; i < 2; i += 2) {
    real tip[3], bp[3];
    for (int k = 0; k < 3; k++) { tip[k] = pos[k] + i * ha[k]; bp[k] = tip[k]; }
    int n_out = 0, ax_out = -1;
    for (int j = 0; j < 3; j++) {
      if (bp[j] < -bsize[j]) { n_out++; ax_out = j; bp[j] = -bsize[j]; }
      else if (bp[j] > bsize[j]) { n_out++; ax_out = j; bp[j] = bsize[j]; }
    }
    if (n_out > 1) continue;
    real dd[3] = {bp[0] - tip[0], bp[1] - tip[1], bp[2] - tip[2]};
    real dist = dot3(dd, dd);
    if (dist < bestdist) { bestdist = dist; bestsegmentpos = i; cltype = -2 + i; clface = ax_out; }
  }
  int clcorner = -123, cledge = -123;
  real bestboxpos = 0;
  for (int i = 0; i < 8; i++) {
    for (int j = 0; j < 3; j++) {
      if (i & (1 << j)) continue;
      real bpt[3] = {(i & 1) ? bsize[0] : -bsize[0], (i & 2) ? bsize[1] : -bsize[1], (i & 4) ? bsize[2] : -bsize[2]};
      bpt[j] = 0;
      real df[3] = {bpt[0] - pos[0], bpt[1] - pos[1], bpt[2] - pos[2]};
      real u = -bsize[j] * df[j], v = dot3(ha, df);
      real ma = bsize[j] * bsize[j], mb = -bsize[j] * ha[j], mc = chl * chl;
      real det = ma * mc - mb * mb;
      if (fabs(det) < MINVAL) continue;
      real idet = 1 / det;
      real x1 = (mc * u - mb * v) * idet, x2 = (ma * v - mb * u) * idet;
      int s1 = 1, s2 = 1;
      if (x1 > 1) { x1 = 1; s1 = 2; x2 = safe_div(v - mb, mc); }
      else if (x1 < -1) { x1 = -1; s1 = 0; x2 = safe_div(v + mb, mc); }
      int x2_over = x2 > 1;
      if (x2_over || x2 < -1) {
        if (x2_over) { x2 = 1; s2 = 2; x1 = safe_div(u - mb, ma); }
        else { x2 = -1; s2 = 0; x1 = safe_div(u + mb, ma); }
        if (x1 > 1) { x1 = 1; s1 = 2; }
        else if (x1 < -1) { x1 = -1; s1 = 0; }
      }
      for (int k = 0; k < 3; k++) df[k] -= ha[k] * x2;
      df[j] += bsize[j] * x1;
      int ct = s1 * 3 + s2;
      real dsq = dot3(df, df);
      if (dsq < bestdist - MINVAL) {
        bestdist = dsq; bestsegmentpos = x2; bestboxpos = x1;
        int c2 = ct / 6;
        clcorner = i + (1 << j) * c2;
        cledge = j;
        cltype = ct;
      }
    }
  }
  real secondpos = -4;
  real uu = ha[0] * bsize[1], vv = ha[1] * bsize[0];
  int w_neg = ha[0] * pos[1] - ha[1] * pos[0] < 0;
  real best = -1;
  int c1 = 0;
  real ee1 = uu - vv, ee2 = uu + vv;
  if (fabs(ee1) > best) { best = fabs(ee1); c1 = ((ee1 < 0) == w_neg) ? 0 : 3; }
  if (fabs(ee2) > best) { best = fabs(ee2); c1 = ((ee2 > 0) == w_neg) ? 1 : 2; }
  out->n = 0;
  if (cltype == -4) return;
  if (cltype >= 0 && cltype / 3 != 1) {
    c1 = axisdir ^ clcorner;
    if (c1 != 0 && c1 != 7) {
      int mul, ax = 0, ax1 = 0, ax2 = 0;
      if (c1 == 1 || c1 == 2 || c1 == 4) mul = 1;
      else { mul = -1; c1 = 7 - c1; }
      if (c1 == 1) { ax = 0; ax1 = 1; ax2 = 2; }
      else if (c1 == 2) { ax = 1; ax1 = 2; ax2 = 0; }
      else if (c1 == 4) { ax = 2; ax1 = 0; ax2 = 1; }
      if (axis[ax] * axis[ax] > 0.5) {
        real mm = 2 * safe_div(bsize[ax], fabs(ha[ax]));
        secondpos = minr(1 - mul * bestsegmentpos, mm);
      } else {
        real mm = 2 * minr(safe_div(bsize[ax1], fabs(ha[ax1])), safe_div(bsize[ax2], fabs(ha[ax2])));
        secondpos = -minr(1 + mul * bestsegmentpos, mm);
      }
      secondpos *= mul;
    }
  } else if (cltype >= 0 && cltype / 3 == 1) {
    c1 = axisdir ^ clcorner;
    c1 &= 7 - (1 << cledge);
    if (c1 == 1 || c1 == 2 || c1 == 4) {
      int ax1 = 0, ax2 = 0, ax = cledge, mul;
      if (cledge == 0) { ax1 = 1; ax2 = 2; }
      if (cledge == 1) { ax1 = 2; ax2 = 0; }
      if (cledge == 2) { ax1 = 0; ax2 = 1; }
      if (fabs(axis[ax1]) > fabs(axis[ax2])) ax1 = ax2;
      ax2 = 3 - ax - ax1;
      if (c1 & (1 << ax2)) { mul = 1; secondpos = 1 - bestsegmentpos; }
      else { mul = -1; secondpos = 1 + bestsegmentpos; }
      real e1 = 2 * safe_div(bsize[ax2], fabs(ha[ax2]));
      secondpos = minr(e1, secondpos);
      real e2;
      if (((axisdir & (1 << ax)) != 0) == ((c1 & (1 << ax2)) != 0)) e2 = 1 - bestboxpos;
      else e2 = 1 + bestboxpos;
      e1 = bsize[ax] * safe_div(e2, fabs(ha[ax]));
      secondpos = minr(e1, secondpos);
      secondpos *= mul;
    }
  } else if (cltype < 0) {
    if (clface != -1) {
      int mul = cltype == -3 ? 1 : -1;
      secondpos = 2;
      real tmp1[3] = {pos[0] - ha[0] * mul, pos[1] - ha[1] * mul, pos[2] - ha[2] * mul};
      for (int i = 0; i < 3; i++) {
        if (i != clface) {
          real ha_r = safe_div((real)mul, ha[i]);
          real e1 = (bsize[i] - tmp1[i]) * ha_r;
          if (0 < e1 && e1 < secondpos) secondpos = e1;
          e1 = (-bsize[i] - tmp1[i]) * ha_r;
          if (0 < e1 && e1 < secondpos) secondpos = e1;
        }
      }
      secondpos *= mul;
    }
  }
  real l1[3], g1[3];
  for (int i = 0; i < 3; i++) l1[i] = pos[i] + ha[i] * bestsegmentpos;
  matvec3(g1, brot, l1);
  for (int i = 0; i < 3; i++) g1[i] += bpos[i];
  real nrm[3];
  out->dist[0] = sphere_box(out->pos[0], nrm, g1, cr, bpos, brot, bsize);
  make_frame(out->frame[0], nrm);
  out->n = 1;
  if (secondpos > -3) {
    real l2[3], g2[3];
    for (int i = 0; i < 3; i++) l2[i] = pos[i] + ha[i] * (secondpos + bestsegmentpos);
    matvec3(g2, brot, l2);
    for (int i = 0; i < 3; i++) g2[i] += bpos[i];
    out->dist[1] = sphere_box(out->pos[1], nrm, g2, cr, bpos, brot, bsize);
    make_frame(out->frame[1], nrm);
    out->n = 2;
  }
}

static void flex_collision(const orc_model* m, orc_data* d);

/* collision_primitive_core.py:519-613 plane_cylinder: candidate k of 4 (both cap rims nearest the plane,
 * then two points of a triangle on the nearer cap) */
static void plane_cylinder_k(int k, const real* n, const real* ppos, const real* cc, const real* cax, real r, real hh, real* dist,
                             real* pos) {
  real axis[3] = {cax[0], cax[1], cax[2]};
  real prjaxis = dot3(n, axis);
  if (prjaxis > 0) { for (int i = 0; i < 3; i++) axis[i] = -axis[i]; prjaxis = -prjaxis; }
  real df[3] = {cc[0] - ppos[0], cc[1] - ppos[1], cc[2] - ppos[2]};
  real dist0 = dot3(df, n);
  real vec[3];
  for (int i = 0; i < 3; i++) vec[i] = axis[i] * prjaxis - n[i];
  real len2 = dot3(vec, vec);
  if (len2 >= 1e-12) { real sc = safe_div(r, sqrt(len2)); for (int i = 0; i < 3; i++) vec[i] *= sc; }
  else { vec[0] = r; vec[1] = 0; vec[2] = 0; }
  real prjvec = dot3(vec, n);
  for (int i = 0; i < 3; i++) axis[i] *= hh;
  prjaxis *= hh;
  if (k == 0) {
    *dist = dist0 + prjaxis + prjvec;
    for (int i = 0; i < 3; i++) pos[i] = cc[i] + vec[i] + axis[i] - n[i] * (*dist * (real)0.5);
  } else if (k == 1) {
    *dist = dist0 - prjaxis + prjvec;
    for (int i = 0; i < 3; i++) pos[i] = cc[i] + vec[i] - axis[i] - n[i] * (*dist * (real)0.5);
  } else {
    real prjvec1 = -prjvec * (real)0.5;
    *dist = dist0 + prjaxis + prjvec1;
    real v1[3];
    cross3(v1, vec, axis);
    normalize3(v1);
    real sc = r * sqrt((real)3) * (real)0.5, sg = k == 2 ? 1 : -1;
    for (int i = 0; i < 3; i++) pos[i] = cc[i] + sg * v1[i] * sc + axis[i] - vec[i] * (real)0.5 - n[i] * (*dist * (real)0.5);
  }
}

/* collision_primitive.py:52-139, 257-277 plane_convex, exhaustive-search branch: the deepest vertex a,
 * then among the vertices within 1e-3 of its depth the one farthest from a (b), farthest from line ab
 * (c), and from the triangle's other edges (d); each distinct vertex is a contact at its own depth. */
static int plane_mesh(const real* nw, const real* ppos, const real* gpos, const real* R, const real* mv, int nvert, real* dist,
                      real pos[4][3]) {
  const real HUGE_ = 1e6;
  real d0[3] = {ppos[0] - gpos[0], ppos[1] - gpos[1], ppos[2] - gpos[2]}, pl[3], n[3];
  for (int i = 0; i < 3; i++) {
    pl[i] = R[i] * d0[0] + R[3 + i] * d0[1] + R[6 + i] * d0[2];
    n[i] = R[i] * nw[0] + R[3 + i] * nw[1] + R[6 + i] * nw[2];
  }
#define PM_SUP(v) ((pl[0] - (v)[0]) * n[0] + (pl[1] - (v)[1]) * n[1] + (pl[2] - (v)[2]) * n[2])
  int idx[4] = {-1, -1, -1, -1};
  real maxs = -HUGE_, a[3] = {0, 0, 0}, b[3] = {0, 0, 0}, c[3] = {0, 0, 0};
  for (int i = 0; i < nvert; i++) {
    real s = PM_SUP(mv + 3 * i);
    if (s > maxs) { maxs = s; idx[0] = i; memcpy(a, mv + 3 * i, sizeof(a)); }
  }
  if (maxs < 0) return 0;
  real thr = maxs - (real)1e-3, best = -HUGE_;
  for (int i = 0; i < nvert; i++) {
    const real* v = mv + 3 * i;
    real mask = PM_SUP(v) > thr ? 0 : -HUGE_;
    real dv[3] = {a[0] - v[0], a[1] - v[1], a[2] - v[2]};
    real dd = dot3(dv, dv) + mask;
    if (dd > best) { idx[1] = i; best = dd; memcpy(b, v, sizeof(b)); }
  }
  real ab[3], t[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
  cross3(ab, n, t);
  best = -HUGE_;
  for (int i = 0; i < nvert; i++) {
    const real* v = mv + 3 * i;
    real mask = PM_SUP(v) > thr ? 0 : -HUGE_;
    real ap[3] = {a[0] - v[0], a[1] - v[1], a[2] - v[2]};
    real dd = fabs(dot3(ap, ab)) + mask;
    if (dd > best) { idx[2] = i; best = dd; memcpy(c, v, sizeof(c)); }
  }
  real ac[3], bc[3], t1[3] = {a[0] - c[0], a[1] - c[1], a[2] - c[2]}, t2[3] = {b[0] - c[0], b[1] - c[1], b[2] - c[2]};
  cross3(ac, n, t1);
  cross3(bc, n, t2);
  best = -HUGE_;
  for (int i = 0; i < nvert; i++) {
    const real* v = mv + 3 * i;
    real mask = PM_SUP(v) > thr ? 0 : -HUGE_;
    real ap[3] = {a[0] - v[0], a[1] - v[1], a[2] - v[2]}, bp[3] = {b[0] - v[0], b[1] - v[1], b[2] - v[2]};
    real dd = (fabs(dot3(ap, ac)) + mask) + (fabs(dot3(bp, bc)) + mask);
    if (dd > best) { idx[3] = i; best = dd; }
  }
  int cnt = 0;
  for (int i = 3; i >= 0; i--) {
    int count = 0;
    for (int j = 0; j <= i; j++) count += idx[j] == idx[i];
    if (count != 1) continue;
    const real* v = mv + 3 * idx[i];
    real dd = -PM_SUP(v);
    for (int k = 0; k < 3; k++) pos[cnt][k] = gpos[k] + R[3 * k] * v[0] + R[3 * k + 1] * v[1] + R[3 * k + 2] * v[2] - (real)0.5 * dd * nw[k];
    dist[cnt] = dd;
    cnt++;
  }
#undef PM_SUP
  return cnt;
}

/* collision_primitive_core.py:364-392 plane_ellipsoid */
static real plane_ellipsoid(real* pos, const real* n, const real* ppos, const real* epos, const real* R, const real* size) {
  real l[3], w[3];
  for (int i = 0; i < 3; i++) l[i] = (R[i] * n[0] + R[3 + i] * n[1] + R[6 + i] * n[2]) * size[i];
  normalize3(l);
  for (int i = 0; i < 3; i++) l[i] = -l[i] * size[i];
  for (int i = 0; i < 3; i++) w[i] = R[3 * i] * l[0] + R[3 * i + 1] * l[1] + R[3 * i + 2] * l[2];
  for (int i = 0; i < 3; i++) pos[i] = epos[i] + w[i];
  real df[3] = {pos[0] - ppos[0], pos[1] - ppos[1], pos[2] - ppos[2]};
  real dist = dot3(n, df);
  for (int i = 0; i < 3; i++) pos[i] -= n[i] * dist * (real)0.5;
  return dist;
}

/* collision_primitive_core.py:446-515 sphere_cylinder */
static real sphere_cylinder(real* pos, real* nrm, const real* sp, real sr, const real* cp, const real* ax, real cr, real hh) {
  real v[3] = {sp[0] - cp[0], sp[1] - cp[1], sp[2] - cp[2]};
  real x = dot3(v, ax);
  real ap[3] = {ax[0] * x, ax[1] * x, ax[2] * x}, pp[3] = {v[0] - ap[0], v[1] - ap[1], v[2] - ap[2]};
  real p2 = dot3(pp, pp);
  int side = fabs(x) < hh, cap = p2 < cr * cr;
  if (side && cap) {
    if (hh - fabs(x) < cr - sqrt(p2)) side = 0;
    else cap = 0;
  }
  if (side) {
    real t[3] = {cp[0] + ap[0], cp[1] + ap[1], cp[2] + ap[2]};
    return sphere_sphere(pos, nrm, sp, sr, t, cr);
  }
  if (cap) {
    real sg = x > 0 ? 1 : -1;
    real pc[3] = {cp[0] + sg * ax[0] * hh, cp[1] + sg * ax[1] * hh, cp[2] + sg * ax[2] * hh}, pn[3] = {sg * ax[0], sg * ax[1], sg * ax[2]};
    real dist = plane_sphere(pos, pn, pc, sp, sr);
    for (int i = 0; i < 3; i++) nrm[i] = -pn[i];
    return dist;
  }
  real inv = safe_div(1, sqrt(p2)), sg = x < 0 ? -1 : 1;
  real c[3];
  for (int i = 0; i < 3; i++) c[i] = cp[i] + ax[i] * sg * hh + pp[i] * cr * inv;
  return sphere_sphere(pos, nrm, sp, sr, c, 0);
}

/* collision_driver.py:43-77 CONVEX entries (heightfields excluded), type-sorted */
static int convex_pair(int t1, int t2) {
  if (t1 == GEOM_PLANE || t1 == GEOM_HFIELD || t2 == GEOM_HFIELD) return 0;
  if (t2 == GEOM_MESH || t2 == GEOM_ELLIPSOID) return 1;
  if (t1 == GEOM_ELLIPSOID) return 1;
  if (t2 == GEOM_CYLINDER) return t1 == GEOM_CAPSULE || t1 == GEOM_CYLINDER;
  if (t1 == GEOM_CYLINDER && t2 == GEOM_BOX) return 1;
  return t1 == GEOM_BOX && t2 == GEOM_BOX;
}

static void collision(const orc_model* m, orc_data* d) {
  *d->ncon = 0;
  *d->ncollision = 0;
  if (m->opt_disableflags & (DSBL_CONSTRAINT | DSBL_CONTACT)) return;
  for (int p = 0; p < m->nxn; p++) {
    int g1 = m->nxn_geom_pair[2 * p], g2 = m->nxn_geom_pair[2 * p + 1];
    int pairid0 = m->nxn_pairid[2 * p], pairid1 = m->nxn_pairid[2 * p + 1];
    if (!(broadphase_filter(m, d, g1, g2) || pairid1 >= 0)) continue;
    (*d->ncollision)++;
    if (m->geom_type[g1] > m->geom_type[g2]) { int t = g1; g1 = g2; g2 = t; }
    real margin, gap, friction[5], solref[2], solreffriction[2], solimp[5];
    int condim;
    contact_params(m, g1, g2, pairid0, &margin, &gap, &condim, friction, solref, solreffriction, solimp);
    int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
    const real *p1 = d->geom_xpos + 3 * g1, *p2 = d->geom_xpos + 3 * g2;
    const real *r1 = d->geom_xmat + 9 * g1, *r2 = d->geom_xmat + 9 * g2;
    const real *s1 = m->geom_size + 3 * g1, *s2 = m->geom_size + 3 * g2;
    real n1[3] = {r1[2], r1[5], r1[8]}, n2[3] = {r2[2], r2[5], r2[8]};
    contacts2 c;
    c.n = 0;
    if (t1 == GEOM_PLANE && t2 == GEOM_SPHERE) {
      c.dist[0] = plane_sphere(c.pos[0], n1, p1, p2, s2[0]);
      make_frame(c.frame[0], n1);
      c.n = 1;
    } else if (t1 == GEOM_PLANE && t2 == GEOM_CAPSULE) {
      plane_capsule(&c, n1, p1, p2, n2, s2[0], s2[1]);
    } else if (t1 == GEOM_SPHERE && t2 == GEOM_SPHERE) {
      real nrm[3];
      c.dist[0] = sphere_sphere(c.pos[0], nrm, p1, s1[0], p2, s2[0]);
      make_frame(c.frame[0], nrm);
      c.n = 1;
    } else if (t1 == GEOM_SPHERE && t2 == GEOM_CAPSULE) {
      real nrm[3];
      c.dist[0] = sphere_capsule(c.pos[0], nrm, p1, s1[0], p2, n2, s2[0], s2[1]);
      make_frame(c.frame[0], nrm);
      c.n = 1;
    } else if (t1 == GEOM_CAPSULE && t2 == GEOM_CAPSULE) {
      capsule_capsule(&c, p1, n1, s1[0], s1[1], p2, n2, s2[0], s2[1], margin);
    } else if (t1 == GEOM_SPHERE && t2 == GEOM_BOX) { /* collision_primitive.py:1047-1114 */
      real nrm[3];
      c.dist[0] = sphere_box(c.pos[0], nrm, p1, s1[0], p2, r2, s2);
      make_frame(c.frame[0], nrm);
      c.n = 1;
    } else if (t1 == GEOM_CAPSULE && t2 == GEOM_BOX) { /* collision_primitive.py:1117-1199 */
      capsule_box(&c, p1, n1, s1[0], s1[1], p2, r2, s2);
    } else if (t1 == GEOM_PLANE && t2 == GEOM_ELLIPSOID) { /* collision_primitive.py:665-733 */
      c.dist[0] = plane_ellipsoid(c.pos[0], n1, p1, p2, r2, s2);
      make_frame(c.frame[0], n1);
      c.n = 1;
    } else if (t1 == GEOM_SPHERE && t2 == GEOM_CYLINDER) { /* collision_primitive.py:882-960 */
      real nrm[3];
      c.dist[0] = sphere_cylinder(c.pos[0], nrm, p1, s1[0], p2, n2, s2[0], s2[1]);
      make_frame(c.frame[0], nrm);
      c.n = 1;
    } else if (t1 == GEOM_PLANE && t2 == GEOM_MESH) { /* collision_primitive.py:52-277, 810-870 plane_convex */
      real pd[4], pp[4][3], fr[9];
      int md = m->geom_dataid[g2];
      int n = plane_mesh(n1, p1, p2, r2, m->mesh_vert + 3 * m->mesh_vertadr[md], m->mesh_vertnum[md], pd, pp);
      make_frame(fr, n1);
      for (int k = 0; k < n; k++) {
        if (!(pd[k] < margin) || pairid0 < -1) continue;
        int cid = *d->ncon;
        if (cid >= d->nconmax) { (*d->ncon)++; continue; }
        d->con_dist[cid] = pd[k];
        memcpy(d->con_pos + 3 * cid, pp[k], 3 * sizeof(real));
        memcpy(d->con_frame + 9 * cid, fr, 9 * sizeof(real));
        d->con_includemargin[cid] = margin - gap;
        memcpy(d->con_friction + 5 * cid, friction, 5 * sizeof(real));
        memcpy(d->con_solref + 2 * cid, solref, 2 * sizeof(real));
        memcpy(d->con_solreffriction + 2 * cid, solreffriction, 2 * sizeof(real));
        memcpy(d->con_solimp + 5 * cid, solimp, 5 * sizeof(real));
        d->con_dim[cid] = condim;
        d->con_geom[2 * cid] = g1;
        d->con_geom[2 * cid + 1] = g2;
        d->con_flex[2 * cid] = d->con_flex[2 * cid + 1] = d->con_vert[2 * cid] = d->con_vert[2 * cid + 1] = -1;
        for (int i = 0; i < 10; i++) d->con_efc_address[10 * cid + i] = -1;
        (*d->ncon)++;
      }
      continue;
    } else if (t1 == GEOM_HFIELD) {
      /* heightfield-convex pair, collision_convex.py:158-697: up to 4 points, each with its own normal */
      ccd_geom cg2;
      memset(&cg2, 0, sizeof(cg2));
      cg2.type = t2;
      memcpy(cg2.pos, p2, sizeof(cg2.pos)); memcpy(cg2.rot, r2, sizeof(cg2.rot)); memcpy(cg2.size, s2, sizeof(cg2.size));
      cg2.vert = t2 == GEOM_MESH ? m->mesh_vert + 3 * m->mesh_vertadr[m->geom_dataid[g2]] : NULL;
      cg2.nvert = t2 == GEOM_MESH ? m->mesh_vertnum[m->geom_dataid[g2]] : 0;
      int hid = m->geom_dataid[g1];
      real hd[4], hp[4][3], hn[4][3], fr[9];
      int n = hfield_pair(p1, r1, m->hfield_size + 4 * hid, m->hfield_nrow[hid], m->hfield_ncol[hid], m->hfield_data + m->hfield_adr[hid],
                          &cg2, m->geom_rbound[g2], m->geom_margin[g1] + m->geom_margin[g2], margin, m->opt_ccd_tolerance,
                          m->opt_ccd_iterations, m->ccd_epa_iterations, hd, hp, hn);
      for (int k = 0; k < n; k++) {
        if (!(hd[k] < margin) || pairid0 < -1) continue;
        int cid = *d->ncon;
        if (cid >= d->nconmax) { (*d->ncon)++; continue; }
        make_frame(fr, hn[k]);
        d->con_dist[cid] = hd[k];
        memcpy(d->con_pos + 3 * cid, hp[k], 3 * sizeof(real));
        memcpy(d->con_frame + 9 * cid, fr, 9 * sizeof(real));
        d->con_includemargin[cid] = margin - gap;
        memcpy(d->con_friction + 5 * cid, friction, 5 * sizeof(real));
        memcpy(d->con_solref + 2 * cid, solref, 2 * sizeof(real));
        memcpy(d->con_solreffriction + 2 * cid, solreffriction, 2 * sizeof(real));
        memcpy(d->con_solimp + 5 * cid, solimp, 5 * sizeof(real));
        d->con_dim[cid] = condim;
        d->con_geom[2 * cid] = g1;
        d->con_geom[2 * cid + 1] = g2;
        d->con_flex[2 * cid] = d->con_flex[2 * cid + 1] = d->con_vert[2 * cid] = d->con_vert[2 * cid + 1] = -1;
        for (int i = 0; i < 10; i++) d->con_efc_address[10 * cid + i] = -1;
        (*d->ncon)++;
      }
      continue;
    } else if (convex_pair(t1, t2)) {
      /* convex (GJK/EPA) pair, collision_convex.py:701-890 */
      ccd_geom cg1, cg2;
      memset(&cg1, 0, sizeof(cg1));
      memset(&cg2, 0, sizeof(cg2));
      cg1.type = t1; cg2.type = t2;
      memcpy(cg1.pos, p1, sizeof(cg1.pos)); memcpy(cg1.rot, r1, sizeof(cg1.rot)); memcpy(cg1.size, s1, sizeof(cg1.size));
      memcpy(cg2.pos, p2, sizeof(cg2.pos)); memcpy(cg2.rot, r2, sizeof(cg2.rot)); memcpy(cg2.size, s2, sizeof(cg2.size));
      if (t1 == GEOM_MESH) ccd_geom_mesh(m, m->geom_dataid[g1], &cg1);
      if (t2 == GEOM_MESH) ccd_geom_mesh(m, m->geom_dataid[g2], &cg2);
      real cdist, cnrm[3], cpts[4][3], cframe[9];
      ccd_multiccd = (m->opt_enableflags & ENBL_MULTICCD) != 0;
      int nc = ccd_pair(&cg1, &cg2, m->opt_ccd_tolerance, m->opt_ccd_iterations, m->ccd_epa_iterations, margin, &cdist, cnrm, cpts);
      make_frame(cframe, cnrm);
      for (int k = 0; k < nc; k++) {
        if (!(cdist < margin) || pairid0 < -1) continue;
        int cid = *d->ncon;
        if (cid >= d->nconmax) { (*d->ncon)++; continue; }
        d->con_dist[cid] = cdist;
        memcpy(d->con_pos + 3 * cid, cpts[k], 3 * sizeof(real));
        memcpy(d->con_frame + 9 * cid, cframe, 9 * sizeof(real));
        d->con_includemargin[cid] = margin - gap;
        memcpy(d->con_friction + 5 * cid, friction, 5 * sizeof(real));
        memcpy(d->con_solref + 2 * cid, solref, 2 * sizeof(real));
        memcpy(d->con_solreffriction + 2 * cid, solreffriction, 2 * sizeof(real));
        memcpy(d->con_solimp + 5 * cid, solimp, 5 * sizeof(real));
        d->con_dim[cid] = condim;
        d->con_geom[2 * cid] = g1;
        d->con_geom[2 * cid + 1] = g2;
      d->con_flex[2 * cid] = d->con_flex[2 * cid + 1] = d->con_vert[2 * cid] = d->con_vert[2 * cid + 1] = -1;
        for (int i = 0; i < 10; i++) d->con_efc_address[10 * cid + i] = -1;
        (*d->ncon)++;
      }
      continue;
    } else if (t1 == GEOM_PLANE && t2 == GEOM_BOX) {
      c.n = 8; /* all 8 corners are candidates (collision_primitive.py:737-790) */
    } else if (t1 == GEOM_PLANE && t2 == GEOM_CYLINDER) {
      c.n = 4; /* collision_primitive.py:964-1040 */
    } else {
      continue; /* pair type not supported by the oracle (not on the benchmark path) */
    }
    for (int k = 0; k < c.n; k++) {
      if (t1 == GEOM_PLANE && t2 == GEOM_BOX) {
        plane_box_corner(k, n1, p1, p2, r2, s2, &c.dist[0], c.pos[0]);
        make_frame(c.frame[0], n1);
      }
      if (t1 == GEOM_PLANE && t2 == GEOM_CYLINDER) {
        plane_cylinder_k(k, n1, p1, p2, n2, s2[0], s2[1], &c.dist[0], c.pos[0]);
        make_frame(c.frame[0], n1);
      }
      int kk = (t1 == GEOM_PLANE && (t2 == GEOM_BOX || t2 == GEOM_CYLINDER)) ? 0 : k;
      real dist = c.dist[kk];
      int active = dist < margin;
      if ((pairid0 == -2 || !active) && pairid1 == -1) continue;
      if (!(pairid0 >= -1 && active)) continue; /* sensor-only contacts are not produced here */
      int cid = *d->ncon;
      if (cid >= d->nconmax) { (*d->ncon)++; continue; }
      d->con_dist[cid] = dist;
      memcpy(d->con_pos + 3 * cid, c.pos[kk], 3 * sizeof(real));
      memcpy(d->con_frame + 9 * cid, c.frame[kk], 9 * sizeof(real));
      d->con_includemargin[cid] = margin - gap;
      memcpy(d->con_friction + 5 * cid, friction, 5 * sizeof(real));
      memcpy(d->con_solref + 2 * cid, solref, 2 * sizeof(real));
      memcpy(d->con_solreffriction + 2 * cid, solreffriction, 2 * sizeof(real));
      memcpy(d->con_solimp + 5 * cid, solimp, 5 * sizeof(real));
      d->con_dim[cid] = condim;
      d->con_geom[2 * cid] = g1;
      d->con_geom[2 * cid + 1] = g2;
      d->con_flex[2 * cid] = d->con_flex[2 * cid + 1] = d->con_vert[2 * cid] = d->con_vert[2 * cid + 1] = -1;
      for (int i = 0; i < 10; i++) d->con_efc_address[10 * cid + i] = -1;
      (*d->ncon)++;
    }
  }
  flex_collision(m, d);
}

/* ---- flex collision (collision_flex.py) ----------------------------------------------------- */

/* collision_primitive_core.py:1495-1515 */
static real tri_area_sign(const real* p1, const real* p2, const real* p3) {
  real a = (p1[0] - p3[0]) * (p2[1] - p3[1]) - (p2[0] - p3[0]) * (p1[1] - p3[1]);
  return (real)((a > 0) - (a < 0));
}

static void tri_point_segment(real* r, const real* p, const real* u, const real* v) {
  real uv[2] = {v[0] - u[0], v[1] - u[1]}, up[2] = {p[0] - u[0], p[1] - u[1]};
  real a = (uv[0] * up[0] + uv[1] * up[1]) / maxr(MINVAL, uv[0] * uv[0] + uv[1] * uv[1]);
  if (a <= 0) { r[0] = u[0]; r[1] = u[1]; }
  else if (a >= 1) { r[0] = v[0]; r[1] = v[1]; }
  else { r[0] = u[0] + a * uv[0]; r[1] = u[1] + a * uv[1]; }
}

/* collision_primitive_core.py:1518-1597 sphere_triangle (mjraw_SphereTriangle) */
static real sphere_triangle(real* pos, real* nrm, const real* sp, real sr, const real* t1, const real* t2, const real* t3,
                            real tr) {
  real S[3], A[3], B[3], N[3], P[3], V1[3], V2[3], X[3];
  for (int i = 0; i < 3; i++) { S[i] = sp[i] - t1[i]; A[i] = t2[i] - t1[i]; B[i] = t3[i] - t1[i]; }
  cross3(N, A, B);
  normalize3(N);
  real dstS = dot3(N, S);
  for (int i = 0; i < 3; i++) P[i] = S[i] - dstS * N[i];
  real lenA = sqrt(dot3(A, A));
  for (int i = 0; i < 3; i++) V1[i] = A[i];
  normalize3(V1);
  cross3(V2, N, A);
  normalize3(V2);
  real o[2] = {0, 0}, a[2] = {lenA, 0}, b[2] = {dot3(V1, B), dot3(V2, B)}, p[2] = {dot3(V1, P), dot3(V2, P)};
  real s1 = tri_area_sign(p, o, a), s2 = tri_area_sign(p, a, b), s3 = tri_area_sign(p, b, o);
  if (s1 == s2 && s2 == s3) {
    for (int i = 0; i < 3; i++) X[i] = P[i];
  } else {
    real x0[2], x1[2], x2[2];
    tri_point_segment(x0, p, o, a);
    tri_point_segment(x1, p, a, b);
    tri_point_segment(x2, p, b, o);
    real d0 = hypot(p[0] - x0[0], p[1] - x0[1]), d1 = hypot(p[0] - x1[0], p[1] - x1[1]), d2 = hypot(p[0] - x2[0], p[1] - x2[1]);
    const real* xs = (d0 < d1 && d0 < d2) ? x0 : (d1 < d2 ? x1 : x2);
    for (int i = 0; i < 3; i++) X[i] = xs[0] * V1[i] + xs[1] * V2[i];
  }
  for (int i = 0; i < 3; i++) nrm[i] = X[i] - S[i];
  real dst = sqrt(dot3(nrm, nrm));
  if (dst > MINVAL) for (int i = 0; i < 3; i++) nrm[i] /= dst;
  else for (int i = 0; i < 3; i++) nrm[i] = N[i];
  real dist = dst - sr - tr;
  for (int i = 0; i < 3; i++) pos[i] = sp[i] + nrm[i] * (sr + (real)0.5 * dist);
  return dist;
}

static void put2(contacts2* c, real dist, const real* pos, const real* nrm) {
  c->dist[c->n] = dist;
  memcpy(c->pos[c->n], pos, 3 * sizeof(real));
  memcpy(c->frame[c->n], nrm, 3 * sizeof(real)); /* normal only; the frame is made by the writer */
  c->n++;
}

/* collision_primitive_core.py:1600-1714 box_triangle */
static void box_triangle(contacts2* c, const real* bp, const real* br, const real* bs, const real* const* t, real tr) {
  for (int vi = 0; vi < 3; vi++) {
    real diff[3], loc[3];
    for (int i = 0; i < 3; i++) diff[i] = t[vi][i] - bp[i];
    for (int i = 0; i < 3; i++) loc[i] = br[i] * diff[0] + br[3 + i] * diff[1] + br[6 + i] * diff[2];
    int maxaxis = 0;
    real maxval = fabs(loc[0]) - bs[0];
    for (int j = 1; j < 3; j++) { real v = fabs(loc[j]) - bs[j]; if (v > maxval) { maxval = v; maxaxis = j; } }
    int inside = 1;
    for (int j = 0; j < 3; j++) if (fabs(loc[j]) > bs[j] + tr) inside = 0;
    if (inside && c->n < 2) {
      real nl[3] = {0, 0, 0}, ng[3], p[3];
      nl[maxaxis] = (real)((loc[maxaxis] > 0) - (loc[maxaxis] < 0));
      matvec3(ng, br, nl);
      real dd = maxval - tr, off = tr + dd * (real)0.5;
      for (int i = 0; i < 3; i++) p[i] = t[vi][i] - ng[i] * off;
      put2(c, dd, p, ng);
    }
  }
  for (int i = 0; i < 8 && c->n < 2; i++) {
    real vec[3] = {(i & 1) ? bs[0] : -bs[0], (i & 2) ? bs[1] : -bs[1], (i & 4) ? bs[2] : -bs[2]}, corner[3], p[3], n[3];
    matvec3(corner, br, vec);
    for (int k = 0; k < 3; k++) corner[k] += bp[k];
    real dd = sphere_triangle(p, n, corner, 0, t[0], t[1], t[2], tr);
    if (dd < MAXVAL) put2(c, dd, p, n);
  }
}

/* collision_primitive_core.py:1717-1819 capsule_triangle */
static void capsule_triangle(contacts2* c, const real* cp, const real* ax, real cr, real hl, const real* const* t, real tr) {
  real p1[3], p2[3], ab[3], p[3], n[3];
  for (int i = 0; i < 3; i++) { p1[i] = cp[i] - ax[i] * hl; p2[i] = cp[i] + ax[i] * hl; ab[i] = p2[i] - p1[i]; }
  real dd = sphere_triangle(p, n, p1, cr, t[0], t[1], t[2], tr);
  if (dd < MAXVAL) put2(c, dd, p, n);
  dd = sphere_triangle(p, n, p2, cr, t[0], t[1], t[2], tr);
  if (dd < MAXVAL && c->n < 2) put2(c, dd, p, n);
  real ab2 = 4 * hl * hl;
  for (int vi = 0; vi < 3 && c->n < 2; vi++) {
    real vec[3], cl[3], df[3];
    for (int i = 0; i < 3; i++) vec[i] = t[vi][i] - p1[i];
    real tp = dot3(vec, ab) / maxr(MINVAL, ab2);
    if (tp > MINVAL && tp < 1 - MINVAL) {
      for (int i = 0; i < 3; i++) { cl[i] = p1[i] + ab[i] * tp; df[i] = t[vi][i] - cl[i]; }
      real draw = sqrt(dot3(df, df));
      if (draw > MINVAL) {
        for (int i = 0; i < 3; i++) { n[i] = df[i] / draw; p[i] = (cl[i] + t[vi][i] + n[i] * (cr - tr)) * (real)0.5; }
        put2(c, draw - cr - tr, p, n);
      }
    }
  }
}

/* collision_primitive_core.py:1822-1990 cylinder_triangle */
static void cylinder_triangle(contacts2* c, const real* cp, const real* ax, real cr, real hh, const real* const* t, real tr) {
  real p1[3], p2[3], ab[3];
  for (int i = 0; i < 3; i++) { p1[i] = cp[i] - ax[i] * hh; p2[i] = cp[i] + ax[i] * hh; ab[i] = p2[i] - p1[i]; }
  real ab2 = 4 * hh * hh;
  for (int vi = 0; vi < 3 && c->n < 2; vi++) {
    const real* vert = t[vi];
    real vec[3], p[3], n[3], dd;
    for (int i = 0; i < 3; i++) vec[i] = vert[i] - p1[i];
    real tp = dot3(vec, ab) / maxr(MINVAL, ab2);
    if (tp > MINVAL && tp < 1 - MINVAL) {
      real cl[3], df[3];
      for (int i = 0; i < 3; i++) { cl[i] = p1[i] + ab[i] * tp; df[i] = vert[i] - cl[i]; }
      real draw = sqrt(dot3(df, df));
      if (draw < cr + tr) {
        if (draw > MINVAL) {
          for (int i = 0; i < 3; i++) { n[i] = df[i] / draw; p[i] = (cl[i] + vert[i] + n[i] * (cr - tr)) * (real)0.5; }
          dd = draw - cr - tr;
        } else {
          real L = sqrt(ab2), d2 = (1 - tp) * L, d1 = tp * L;
          if (d2 < cr && d2 < d1) {
            for (int i = 0; i < 3; i++) { n[i] = ax[i]; p[i] = vert[i]; }
            dd = -d2 - tr;
          } else if (d1 < cr) {
            for (int i = 0; i < 3; i++) { n[i] = -ax[i]; p[i] = vert[i]; }
            dd = -d1 - tr;
          } else {
            real e1[3], e2[3];
            for (int i = 0; i < 3; i++) { e1[i] = t[1][i] - t[0][i]; e2[i] = t[2][i] - t[0][i]; }
            cross3(n, e1, e2);
            normalize3(n);
            for (int i = 0; i < 3; i++) p[i] = cl[i];
            dd = -cr - tr;
          }
        }
        put2(c, dd, p, n);
      }
    } else {
      const real* pe = tp <= MINVAL ? p1 : p2;
      real sgn = tp <= MINVAL ? -1 : 1;
      real df[3], perp[3];
      for (int i = 0; i < 3; i++) df[i] = vert[i] - pe[i];
      real sd = dot3(df, ax);
      for (int i = 0; i < 3; i++) perp[i] = df[i] - ax[i] * sd;
      real pl = sqrt(dot3(perp, perp));
      if (pl < cr) {
        dd = sgn * sd - tr;
        for (int i = 0; i < 3; i++) { n[i] = sgn * ax[i]; p[i] = vert[i] - n[i] * (tr + dd * (real)0.5); }
        put2(c, dd, p, n);
      } else if (pl < cr + tr) {
        real ep[3], de[3];
        for (int i = 0; i < 3; i++) { ep[i] = pe[i] + perp[i] / pl * cr; de[i] = vert[i] - ep[i]; }
        real draw = sqrt(dot3(de, de));
        if (draw > MINVAL) {
          dd = draw - tr;
          for (int i = 0; i < 3; i++) { n[i] = de[i] / draw; p[i] = vert[i] - n[i] * (tr + dd * (real)0.5); }
          put2(c, dd, p, n);
        }
      }
    }
  }
}

/* collision_flex.py:32-88 _write_flex_contact: geom[0] = geom, flex[1] / vert[1] = the flex vertex */
static void write_flex_contact(const orc_model* m, orc_data* d, real dist, const real* pos, const real* nrm, real margin,
                               int condim, const real* friction, const real* solref, const real* solimp, int g, int f, int vert) {
  if (dist >= margin || dist >= MAXVAL) return;
  int cid = *d->ncon;
  if (cid >= d->nconmax) { (*d->ncon)++; return; }
  d->con_dist[cid] = dist;
  memcpy(d->con_pos + 3 * cid, pos, 3 * sizeof(real));
  make_frame(d->con_frame + 9 * cid, nrm);
  d->con_includemargin[cid] = margin;
  memcpy(d->con_friction + 5 * cid, friction, 5 * sizeof(real));
  memcpy(d->con_solref + 2 * cid, solref, 2 * sizeof(real));
  d->con_solreffriction[2 * cid] = d->con_solreffriction[2 * cid + 1] = 0;
  memcpy(d->con_solimp + 5 * cid, solimp, 5 * sizeof(real));
  d->con_dim[cid] = condim;
  d->con_geom[2 * cid] = g;
  d->con_geom[2 * cid + 1] = -1;
  d->con_flex[2 * cid] = -1;
  d->con_flex[2 * cid + 1] = f;
  d->con_vert[2 * cid] = -1;
  d->con_vert[2 * cid + 1] = vert;
  for (int i = 0; i < 10; i++) d->con_efc_address[10 * cid + i] = -1;
  (*d->ncon)++;
  (void)m;
}

/* collision_flex.py:381-529 (dim-2 elements and, :531-683, dim-3 shell triangles vs sphere / capsule /
 * box / cylinder, every geom tested -- the reference has no flex broadphase) and :261-378 (vertices of
 * every flex vs planes) */
static void flex_collision(const orc_model* m, orc_data* d) {
  for (int f = 0; f < m->nflex; f++) {
    /* dim 2: the elements; dim 3: the boundary (shell) triangles, collision_flex.py:531-683 */
    if (m->flex_dim[f] != 2 && m->flex_dim[f] != 3) continue;
    const int shell = m->flex_dim[f] == 3;
    real tr = m->flex_radius[f], tm = m->flex_margin[f];
    const int ntri = shell ? m->flex_shellnum[f] : m->flex_elemnum[f];
    for (int el = 0; el < ntri; el++) {
      const int* ev = shell ? m->flex_shell + m->flex_shelldataadr[f] + 3 * el : m->flex_elem + m->flex_elemdataadr[f] + 3 * el;
      const real* t[3];
      for (int k = 0; k < 3; k++) t[k] = d->flexvert_xpos + 3 * (m->flex_vertadr[f] + ev[k]);
      for (int g = 0; g < m->ngeom; g++) {
        int gt = m->geom_type[g];
        if (gt != GEOM_SPHERE && gt != GEOM_CAPSULE && gt != GEOM_BOX && gt != GEOM_CYLINDER) continue;
        if (!((m->geom_contype[g] & m->flex_conaffinity[f]) || (m->flex_contype[f] & m->geom_conaffinity[g]))) continue;
        real margin = m->geom_margin[g] + tm;
        const real *gp = d->geom_xpos + 3 * g, *gr = d->geom_xmat + 9 * g, *gs = m->geom_size + 3 * g;
        const real* gf = m->geom_friction + 3 * g;
        real fr[5] = {maxr(MINMU, gf[0]), maxr(MINMU, gf[0]), maxr(MINMU, gf[1]), maxr(MINMU, gf[2]), maxr(MINMU, gf[2])};
        real ax[3] = {gr[2], gr[5], gr[8]};
        contacts2 c;
        c.n = 0;
        if (gt == GEOM_SPHERE) {
          real p[3], n[3];
          real dd = sphere_triangle(p, n, gp, gs[0], t[0], t[1], t[2], tr);
          put2(&c, dd, p, n);
        } else if (gt == GEOM_CAPSULE) {
          capsule_triangle(&c, gp, ax, gs[0], gs[1], t, tr);
        } else if (gt == GEOM_BOX) {
          box_triangle(&c, gp, gr, gs, t, tr);
        } else {
          cylinder_triangle(&c, gp, ax, gs[0], gs[1], t, tr);
        }
        for (int k = 0; k < c.n; k++)
          if (c.dist[k] < margin)
            write_flex_contact(m, d, c.dist[k], c.pos[k], c.frame[k], margin, m->geom_condim[g], fr, m->geom_solref + 2 * g,
                               m->geom_solimp + 5 * g, g, f, ev[0]);
      }
    }
  }
  for (int v = 0; v < m->nflexvert; v++) {
    int f = m->flex_vertflexid[v];
    const real* x = d->flexvert_xpos + 3 * v;
    for (int g = 0; g < m->ngeom; g++) {
      if (m->geom_type[g] != GEOM_PLANE) continue;
      const real *pp = d->geom_xpos + 3 * g, *pr = d->geom_xmat + 9 * g;
      real n[3] = {pr[2], pr[5], pr[8]}, df[3] = {x[0] - pp[0], x[1] - pp[1], x[2] - pp[2]};
      real margin = m->geom_margin[g] + m->flex_margin[f];
      real dist = dot3(df, n) - m->flex_radius[f];
      if (!(dist < margin)) continue;
      const real *gf = m->geom_friction + 3 * g, *ff = m->flex_friction + 3 * f;
      real f0 = maxr(gf[0], ff[0]), f1 = maxr(gf[1], ff[1]), f2 = maxr(gf[2], ff[2]);
      real fr[5] = {maxr(MINMU, f0), maxr(MINMU, f0), maxr(MINMU, f1), maxr(MINMU, f2), maxr(MINMU, f2)};
      real p[3];
      for (int i = 0; i < 3; i++) p[i] = x[i] - n[i] * (dist * (real)0.5 + m->flex_radius[f]);
      int condim = m->geom_condim[g] > m->flex_condim[f] ? m->geom_condim[g] : m->flex_condim[f];
      write_flex_contact(m, d, dist, p, n, margin, condim, fr, m->geom_solref + 2 * g, m->geom_solimp + 5 * g, g, f,
                         v - m->flex_vertadr[f]);
    }
  }
}

/* =============================================================================================
 * constraint.py
 * ============================================================================================= */

/* constraint.py:52-121: D and aref of one row from its impedance / reference inputs */
static void efc_params(int disableflags, real timestep, real pos_aref, real pos_imp, real invweight, const real* solref,
                       const real* solimp, real vel, real* D, real* aref) {
  real timeconst = solref[0], dampratio = solref[1];
  real dmin = solimp[0], dmax = solimp[1], width = solimp[2], mid = solimp[3], power = solimp[4];
  if (!(disableflags & DSBL_REFSAFE)) timeconst = maxr(timeconst, 2 * timestep);
  dmin = clampr(dmin, MINIMP, MAXIMP);
  dmax = clampr(dmax, MINIMP, MAXIMP);
  width = maxr(MINVAL, width);
  mid = clampr(mid, MINIMP, MAXIMP);
  power = maxr(1, power);
  real dmax_sq = dmax * dmax;
  real k = 1 / (dmax_sq * timeconst * timeconst * dampratio * dampratio);
  real b = 2 / (dmax * timeconst);
  if (solref[0] <= 0) k = -solref[0] / dmax_sq;
  if (solref[1] <= 0) b = -solref[1] / dmax;
  real imp_x = fabs(pos_imp) / width;
  real imp_a = (1 / pow(mid, power - 1)) * pow(imp_x, power);
  real imp_b = 1 - (1 / pow(1 - mid, power - 1)) * pow(1 - imp_x, power);
  real imp_y = imp_x < mid ? imp_a : imp_b;
  real imp = dmin + imp_y * (dmax - dmin);
  imp = clampr(imp, dmin, dmax);
  if (imp_x > 1) imp = dmax;
  *D = 1 / maxr(invweight * (1 - imp) / imp, MINVAL);
  *aref = -k * imp * pos_aref - b * vel;
}

void orc_kat_efc_row(int disableflags, real timestep, real pos_aref, real pos_imp, real invweight, const real* solref,
                     const real* solimp, real vel, real* out) {
  efc_params(disableflags, timestep, pos_aref, pos_imp, invweight, solref, solimp, vel, out, out + 1);
}

static void efc_row(const orc_model* m, orc_data* d, int efcid, real pos_aref, real pos_imp, real invweight, const real* solref,
                    const real* solimp, real margin, real vel, real frictionloss, int type, int id) {
  efc_params(m->opt_disableflags, m->opt_timestep, pos_aref, pos_imp, invweight, solref, solimp, vel, d->efc_D + efcid,
             d->efc_aref + efcid);
  d->efc_vel[efcid] = vel;
  d->efc_pos[efcid] = pos_aref + margin;
  d->efc_margin[efcid] = margin;
  d->efc_frictionloss[efcid] = frictionloss;
  d->efc_type[efcid] = type;
  d->efc_id[efcid] = id;
  real* prm = d->efc_prm + 9 * efcid;
  prm[0] = pos_imp;
  prm[1] = invweight;
  prm[2] = solref[0];
  prm[3] = solref[1];
  for (int i = 0; i < 5; i++) prm[4 + i] = solimp[i];
}

/* support.py:396-432 */
static int jac_dof(const orc_model* m, const orc_data* d, const real* point, int bodyid, int dofid, real* jacp, real* jacr) {
  int db = m->dof_bodyid[dofid];
  int in_tree = db == 0;
  int p = bodyid;
  while (p != 0) {
    if (p == db) { in_tree = 1; break; }
    p = m->body_parentid[p];
  }
  if (!in_tree) { jacp[0] = jacp[1] = jacp[2] = jacr[0] = jacr[1] = jacr[2] = 0; return 0; }
  real off[3];
  for (int i = 0; i < 3; i++) off[i] = point[i] - d->subtree_com[3 * m->body_rootid[bodyid] + i];
  const real* cd = d->cdof + 6 * dofid;
  real c[3];
  cross3(c, cd, off);
  for (int i = 0; i < 3; i++) { jacp[i] = cd[3 + i] + c[i]; jacr[i] = cd[i]; }
  return 1;
}

/* constraint.py:124-365 _equality_connect / :792-1110 _equality_weld, rows efcid .. efcid+2 (+5) */
static void eq_connect_weld(const orc_model* m, orc_data* d, int e, int efcid, int weld) {
  int nv = m->nv;
  const real* data = m->eq_data + 11 * e;
  int o1 = m->eq_obj1id[e], o2 = m->eq_obj2id[e], b1, b2;
  real p1[3], p2[3], q[4] = {1, 0, 0, 0}, q1[4] = {1, 0, 0, 0};
  if (m->eq_objtype[e] == OBJ_SITE && m->nsite > 0) {
    b1 = m->site_bodyid[o1];
    b2 = m->site_bodyid[o2];
    memcpy(p1, d->site_xpos + 3 * o1, sizeof(p1));
    memcpy(p2, d->site_xpos + 3 * o2, sizeof(p2));
    if (weld) {
      real t[4];
      mul_quat(q, d->xquat + 4 * b1, m->site_quat + 4 * o1);
      mul_quat(t, d->xquat + 4 * b2, m->site_quat + 4 * o2);
      q1[0] = t[0]; q1[1] = -t[1]; q1[2] = -t[2]; q1[3] = -t[3];
    }
  } else {
    b1 = o1;
    b2 = o2;
    const real* a1 = weld ? data + 3 : data; /* the weld reads its anchors swapped (:855-856) */
    const real* a2 = weld ? data : data + 3;
    matvec3(p1, d->xmat + 9 * b1, a1);
    matvec3(p2, d->xmat + 9 * b2, a2);
    for (int k = 0; k < 3; k++) { p1[k] += d->xpos[3 * b1 + k]; p2[k] += d->xpos[3 * b2 + k]; }
    if (weld) {
      mul_quat(q, d->xquat + 4 * b1, data + 6);
      const real* x2 = d->xquat + 4 * b2;
      q1[0] = x2[0]; q1[1] = -x2[1]; q1[2] = -x2[2]; q1[3] = -x2[3];
    }
  }
  real ts = data[10], jq[6] = {0, 0, 0, 0, 0, 0};
  int nrow = weld ? 6 : 3;
  for (int i = 0; i < nv; i++) {
    real j1p[3], j1r[3], j2p[3], j2r[3], v[6];
    jac_dof(m, d, p1, b1, i, j1p, j1r);
    jac_dof(m, d, p2, b2, i, j2p, j2r);
    for (int k = 0; k < 3; k++) v[k] = j1p[k] - j2p[k];
    if (weld) {
      real dr[3], t[4], u[4];
      for (int k = 0; k < 3; k++) dr[k] = (j1r[k] - j2r[k]) * ts;
      t[0] = -q1[1] * dr[0] - q1[2] * dr[1] - q1[3] * dr[2]; /* math.py:33-41 quat_mul_axis */
      t[1] = q1[0] * dr[0] + q1[2] * dr[2] - q1[3] * dr[1];
      t[2] = q1[0] * dr[1] + q1[3] * dr[0] - q1[1] * dr[2];
      t[3] = q1[0] * dr[2] + q1[1] * dr[1] - q1[2] * dr[0];
      mul_quat(u, t, q);
      for (int k = 0; k < 3; k++) v[3 + k] = 0.5 * u[1 + k];
    }
    for (int k = 0; k < nrow; k++) {
      d->efc_J[(size_t)(efcid + k) * nv + i] = v[k];
      jq[k] += v[k] * d->qvel[i];
    }
  }
  real cpos[6], pos_imp;
  for (int k = 0; k < 3; k++) cpos[k] = p1[k] - p2[k];
  if (weld) {
    real cq[4];
    mul_quat(cq, q1, q);
    for (int k = 0; k < 3; k++) cpos[3 + k] = cq[1 + k] * ts;
    pos_imp = sqrt(dot3(cpos, cpos) + dot3(cpos + 3, cpos + 3));
  } else {
    pos_imp = sqrt(dot3(cpos, cpos));
  }
  for (int k = 0; k < nrow; k++) {
    int c = k < 3 ? 0 : 1;
    real iw = m->body_invweight0[2 * b1 + c] + m->body_invweight0[2 * b2 + c];
    efc_row(m, d, efcid + k, cpos[k], pos_imp, iw, m->eq_solref + 2 * e, m->eq_solimp + 5 * e, 0, jq[k], 0, CNSTR_EQUALITY, e);
  }
}

/* constraint.py:2209-2779 (equality / friction / limit / contact, in that order) */
static void make_constraint(const orc_model* m, orc_data* d) {
  int nv = m->nv, njmax = d->njmax;
  *d->ne = *d->nf = *d->nl = *d->nefc = 0;
  if (m->opt_disableflags & DSBL_CONSTRAINT) return;
  /* connect, then weld (constraint.py:2221-2330 launch order), each in equality index order */
  if (!(m->opt_disableflags & DSBL_EQUALITY)) {
    for (int weld = 0; weld < 2; weld++) {
      for (int e = 0; e < m->neq; e++) {
        if (m->eq_type[e] != (weld ? EQ_WELD : EQ_CONNECT) || !d->eq_active[e]) continue;
        int nrow = weld ? 6 : 3;
        int efcid = *d->nefc;
        *d->ne += nrow;
        *d->nefc += nrow;
        if (efcid + nrow <= njmax) eq_connect_weld(m, d, e, efcid, weld);
      }
    }
  }
  /* equality joint constraint.py:367-495 (rows in equality index order) */
  if (!(m->opt_disableflags & DSBL_EQUALITY)) {
    for (int e = 0; e < m->neq; e++) {
      if (m->eq_type[e] != EQ_JOINT || !d->eq_active[e]) continue;
      (*d->ne)++;
      int efcid = (*d->nefc)++;
      if (efcid >= njmax) continue;
      int j1 = m->eq_obj1id[e], j2 = m->eq_obj2id[e];
      const real* data = m->eq_data + 11 * e;
      int da1 = m->jnt_dofadr[j1], qa1 = m->jnt_qposadr[j1];
      real* J = d->efc_J + (size_t)efcid * nv;
      memset(J, 0, nv * sizeof(real));
      J[da1] = 1;
      real pos, Jqvel, invweight;
      if (j2 > -1) {
        int qa2 = m->jnt_qposadr[j2], da2 = m->jnt_dofadr[j2];
        real dif = d->qpos[qa2] - m->qpos0[qa2];
        real rhs = data[0] + dif * (data[1] + dif * (data[2] + dif * (data[3] + dif * data[4])));
        real deriv_2 = data[1] + dif * (2 * data[2] + dif * (3 * data[3] + dif * 4 * data[4]));
        pos = d->qpos[qa1] - m->qpos0[qa1] - rhs;
        Jqvel = d->qvel[da1] - d->qvel[da2] * deriv_2;
        invweight = m->dof_invweight0[da1] + m->dof_invweight0[da2];
        J[da2] = -deriv_2;
      } else {
        pos = d->qpos[qa1] - m->qpos0[qa1] - data[0];
        Jqvel = d->qvel[da1];
        invweight = m->dof_invweight0[da1];
      }
      efc_row(m, d, efcid, pos, pos, invweight, m->eq_solref + 2 * e, m->eq_solimp + 5 * e, 0, Jqvel, 0, CNSTR_EQUALITY, e);
    }
  }
  /* equality tendon constraint.py:498-674: L1 - L1_0 = poly(L2 - L2_0), J = J1 - poly'(L2 - L2_0) J2 */
  if (!(m->opt_disableflags & DSBL_EQUALITY)) {
    for (int e = 0; e < m->neq; e++) {
      if (m->eq_type[e] != EQ_TENDON || !d->eq_active[e]) continue;
      (*d->ne)++;
      int efcid = (*d->nefc)++;
      if (efcid >= njmax) continue;
      const int t1 = m->eq_obj1id[e], t2 = m->eq_obj2id[e];
      const real* data = m->eq_data + 11 * e;
      real pos1 = d->ten_length[t1] - m->tendon_length0[t1], pos, deriv = 0, invweight = m->tendon_invweight0[t1];
      if (t2 > -1) {
        invweight += m->tendon_invweight0[t2];
        const real dif = d->ten_length[t2] - m->tendon_length0[t2];
        pos = pos1 - (data[0] + data[1] * dif + data[2] * dif * dif + data[3] * dif * dif * dif + data[4] * dif * dif * dif * dif);
        deriv = data[1] + 2 * data[2] * dif + 3 * data[3] * dif * dif + 4 * data[4] * dif * dif * dif;
      } else {
        pos = pos1 - data[0];
      }
      real* J = d->efc_J + (size_t)efcid * nv;
      ten_J_dense(m, d, t1, J);
      if (deriv != 0) {
        real* J2 = (real*)malloc(nv * sizeof(real));
        ten_J_dense(m, d, t2, J2);
        for (int i = 0; i < nv; i++) J[i] += J2[i] * -deriv;
        free(J2);
      }
      real Jqvel = 0;
      for (int i = 0; i < nv; i++) Jqvel += J[i] * d->qvel[i];
      efc_row(m, d, efcid, pos, pos, invweight, m->eq_solref + 2 * e, m->eq_solimp + 5 * e, 0, Jqvel, 0, CNSTR_EQUALITY, e);
    }
  }
  /* equality flex constraint.py:677-790: one row per edge of each flex with an active FLEX equality */
  if (!(m->opt_disableflags & DSBL_EQUALITY)) {
    for (int e = 0; e < m->neq; e++) {
      if (m->eq_type[e] != EQ_FLEX || !d->eq_active[e]) continue;
      int f = m->eq_obj1id[e];
      for (int ed = m->flex_edgeadr[f]; ed < m->flex_edgeadr[f] + m->flex_edgenum[f]; ed++) {
        (*d->ne)++;
        int efcid = (*d->nefc)++;
        if (efcid >= njmax) continue;
        real* J = d->efc_J + (size_t)efcid * nv;
        memset(J, 0, nv * sizeof(real));
        int v[2] = {m->flex_vertadr[f] + m->flex_edge[2 * ed], m->flex_vertadr[f] + m->flex_edge[2 * ed + 1]};
        int slot = 0;
        real Jqvel = 0;
        for (int s2 = 0; s2 < 2; s2++) {
          int b = m->flex_vertbodyid[v[s2]];
          for (int k = 0; k < m->body_dofnum[b]; k++) {
            int dof = m->body_dofadr[b] + k;
            J[dof] += d->flexedge_J[6 * ed + slot];
            Jqvel += d->flexedge_J[6 * ed + slot] * d->qvel[dof];
            slot++;
          }
        }
        real pos = d->flexedge_length[ed] - m->flexedge_length0[ed];
        efc_row(m, d, efcid, pos, pos, m->flexedge_invweight0[ed], m->eq_solref + 2 * e, m->eq_solimp + 5 * e, 0, Jqvel, 0,
                CNSTR_EQUALITY, e);
      }
    }
  }
  /* friction dof constraint.py:1113-1190 */
  if (!(m->opt_disableflags & DSBL_FRICTIONLOSS)) {
    for (int i = 0; i < nv; i++) {
      real fl = m->dof_frictionloss[i];
      if (fl <= 0) continue;
      (*d->nf)++;
      int efcid = (*d->nefc)++;
      if (efcid >= njmax) continue;
      real* J = d->efc_J + (size_t)efcid * nv;
      memset(J, 0, nv * sizeof(real));
      J[i] = 1;
      efc_row(m, d, efcid, 0, 0, m->dof_invweight0[i], m->dof_solref + 2 * i, m->dof_solimp + 5 * i, 0, d->qvel[i], fl,
              CNSTR_FRICTION_DOF, i);
    }
    /* friction tendon constraint.py:1204-1313 */
    for (int t = 0; t < m->ntendon; t++) {
      real fl = m->tendon_frictionloss[t];
      if (fl <= 0) continue;
      (*d->nf)++;
      int efcid = (*d->nefc)++;
      if (efcid >= njmax) continue;
      real* J = d->efc_J + (size_t)efcid * nv;
      ten_J_dense(m, d, t, J);
      real Jqvel = 0;
      for (int i = 0; i < nv; i++) Jqvel += J[i] * d->qvel[i];
      efc_row(m, d, efcid, 0, 0, m->tendon_invweight0[t], m->tendon_solref_fri + 2 * t, m->tendon_solimp_fri + 5 * t, 0, Jqvel, fl,
              CNSTR_FRICTION_TENDON, t);
    }
  }
  /* limit ball constraint.py:1421-1543 */
  if (!(m->opt_disableflags & DSBL_LIMIT)) {
    for (int j = 0; j < m->njnt; j++) {
      if (!m->jnt_limited[j] || m->jnt_type[j] != JNT_BALL) continue;
      real q[4], aa[3], axis[3];
      memcpy(q, d->qpos + m->jnt_qposadr[j], sizeof(q));
      normalize4(q);
      quat_to_vel(aa, q);
      real angle = sqrt(dot3(aa, aa));
      for (int k = 0; k < 3; k++) axis[k] = angle == 0 ? aa[k] : aa[k] / angle;
      const real* rng = m->jnt_range + 2 * j;
      real pos = maxr(rng[0], rng[1]) - angle - m->jnt_margin[j];
      if (!(pos < 0)) continue;
      (*d->nl)++;
      int efcid = (*d->nefc)++;
      if (efcid >= njmax) continue;
      int da = m->jnt_dofadr[j];
      real* J = d->efc_J + (size_t)efcid * nv;
      memset(J, 0, nv * sizeof(real));
      real Jqvel = 0;
      for (int k = 0; k < 3; k++) { J[da + k] = -axis[k]; Jqvel -= axis[k] * d->qvel[da + k]; }
      efc_row(m, d, efcid, pos, pos, m->dof_invweight0[da], m->jnt_solref + 2 * j, m->jnt_solimp + 5 * j, m->jnt_margin[j], Jqvel, 0,
              CNSTR_LIMIT_JOINT, j);
    }
  }
  /* limit slide/hinge constraint.py:1316-1418 */
  if (!(m->opt_disableflags & DSBL_LIMIT)) {
    for (int j = 0; j < m->njnt; j++) {
      int jt = m->jnt_type[j];
      if (!m->jnt_limited[j] || !(jt == JNT_SLIDE || jt == JNT_HINGE)) continue;
      const real* rng = m->jnt_range + 2 * j;
      real q = d->qpos[m->jnt_qposadr[j]];
      real dmn = q - rng[0], dmx = rng[1] - q;
      real pos = minr(dmn, dmx) - m->jnt_margin[j];
      if (!(pos < 0)) continue;
      (*d->nl)++;
      int efcid = (*d->nefc)++;
      if (efcid >= njmax) continue;
      int da = m->jnt_dofadr[j];
      real Jv = (real)(dmn < dmx) * 2 - 1;
      real* J = d->efc_J + (size_t)efcid * nv;
      memset(J, 0, nv * sizeof(real));
      J[da] = Jv;
      efc_row(m, d, efcid, pos, pos, m->dof_invweight0[da], m->jnt_solref + 2 * j, m->jnt_solimp + 5 * j, m->jnt_margin[j],
              Jv * d->qvel[da], 0, CNSTR_LIMIT_JOINT, j);
    }
    /* limit tendon constraint.py:1547-1665 */
    for (int t = 0; t < m->ntendon; t++) {
      if (!m->tendon_limited[t]) continue;
      const real* rng = m->tendon_range + 2 * t;
      real L = d->ten_length[t], dmn = L - rng[0], dmx = rng[1] - L;
      real pos = minr(dmn, dmx) - m->tendon_margin[t];
      if (!(pos < 0)) continue;
      (*d->nl)++;
      int efcid = (*d->nefc)++;
      if (efcid >= njmax) continue;
      real scl = (real)(dmn < dmx) * 2 - 1;
      real* J = d->efc_J + (size_t)efcid * nv;
      ten_J_dense(m, d, t, J);
      real Jqvel = 0;
      for (int i = 0; i < nv; i++) { J[i] *= scl; Jqvel += J[i] * d->qvel[i]; }
      efc_row(m, d, efcid, pos, pos, m->tendon_invweight0[t], m->tendon_solref_lim + 2 * t, m->tendon_solimp_lim + 5 * t,
              m->tendon_margin[t], Jqvel, 0, CNSTR_LIMIT_TENDON, t);
    }
  }
  /* contact pyramidal constraint.py:1668-1936, elliptic :1940-2200 */
  if (!(m->opt_disableflags & DSBL_CONTACT)) {
    int ncon = *d->ncon < d->nconmax ? *d->ncon : d->nconmax;
    for (int c = 0; c < ncon; c++) {
      int condim = d->con_dim[c];
      int elliptic = m->opt_cone == CONE_ELLIPTIC && condim > 1;
      int nrow = condim == 1 ? 1 : (elliptic ? condim : 2 * (condim - 1));
      real includemargin = d->con_includemargin[c];
      real pos = d->con_dist[c] - includemargin;
      if (!(pos < 0)) continue;
      int g1 = d->con_geom[2 * c], g2 = d->con_geom[2 * c + 1];
      /* constraint.py:1758-1771: a flex side resolves to its vertex body */
      int body1 = g1 >= 0 ? m->geom_bodyid[g1] : m->flex_vertbodyid[m->flex_vertadr[d->con_flex[2 * c]] + d->con_vert[2 * c]];
      int body2 = g2 >= 0 ? m->geom_bodyid[g2] : m->flex_vertbodyid[m->flex_vertadr[d->con_flex[2 * c + 1]] + d->con_vert[2 * c + 1]];
      real iw_base = m->body_invweight0[2 * body1] + m->body_invweight0[2 * body2];
      int w1 = m->body_weldid[body1], w2 = m->body_weldid[body2];
      const real* frame = d->con_frame + 9 * c;
      const real* cpos = d->con_pos + 3 * c;
      for (int dimid = 0; dimid < nrow; dimid++) {
        int efcid = (*d->nefc)++;
        if (efcid >= njmax) { d->con_efc_address[10 * c + dimid] = -1; continue; }
        d->con_efc_address[10 * c + dimid] = efcid;
        if (elliptic) {
          /* constraint.py:2107-2195: row dimid projects the relative jacobian on frame row dimid
           * (translational for dimid < 3, rotational after); friction rows scale invweight by
           * impratio^-1 and (fri0 / frii)^2, use solreffriction when set, and have no position term */
          real invw = iw_base, pos_aref = pos;
          const real* sr = d->con_solref + 2 * c;
          if (dimid > 0) {
            const real* srf = d->con_solreffriction + 2 * c;
            if (srf[0] != 0 || srf[1] != 0) sr = srf;
            invw = invw * m->opt_impratio_invsqrt * m->opt_impratio_invsqrt;
            if (dimid > 1) {
              real fri0 = d->con_friction[5 * c], frii = d->con_friction[5 * c + dimid - 1];
              invw *= fri0 * fri0 / (frii * frii);
            }
            pos_aref = 0;
          }
          real* J = d->efc_J + (size_t)efcid * nv;
          real Jqvel = 0;
          for (int i = nv - 1; i >= 0; i--) {
            real j1p[3], j1r[3], j2p[3], j2r[3];
            jac_dof(m, d, cpos, w1, i, j1p, j1r);
            jac_dof(m, d, cpos, w2, i, j2p, j2r);
            real Jval = 0;
            for (int x = 0; x < 3; x++)
              Jval += dimid < 3 ? frame[3 * dimid + x] * (j2p[x] - j1p[x]) : frame[3 * (dimid - 3) + x] * (j2r[x] - j1r[x]);
            J[i] = Jval;
            Jqvel += Jval * d->qvel[i];
          }
          efc_row(m, d, efcid, pos_aref, pos, invw, sr, d->con_solimp + 5 * c, includemargin, Jqvel, 0, CNSTR_CONTACT_ELLIPTIC, c);
          continue;
        }
        real invweight = iw_base;
        real frii = 0;
        int dimid2 = dimid / 2 + 1;
        if (condim > 1) {
          real fri0 = d->con_friction[5 * c];
          frii = d->con_friction[5 * c + dimid2 - 1];
          invweight = invweight + fri0 * fri0 * invweight;
          invweight = invweight * 2 * fri0 * fri0 * m->opt_impratio_invsqrt * m->opt_impratio_invsqrt;
        }
        real* J = d->efc_J + (size_t)efcid * nv;
        real Jqvel = 0;
        for (int i = nv - 1; i >= 0; i--) {
          real j1p[3], j1r[3], j2p[3], j2r[3];
          jac_dof(m, d, cpos, w1, i, j1p, j1r);
          jac_dof(m, d, cpos, w2, i, j2p, j2r);
          real Jval = 0, Ji = 0;
          for (int x = 0; x < 3; x++) {
            real jd = j2p[x] - j1p[x];
            Jval += frame[x] * jd;
            if (condim > 1) {
              if (dimid2 < 3) Ji += frame[3 * dimid2 + x] * jd;
              else Ji += frame[3 * (dimid2 - 3) + x] * (j2r[x] - j1r[x]);
            }
          }
          if (condim > 1) {
            if (dimid % 2 == 0) Jval += Ji * frii;
            else Jval -= Ji * frii;
          }
          J[i] = Jval;
          Jqvel += Jval * d->qvel[i];
        }
        int type = condim == 1 ? CNSTR_CONTACT_FRICTIONLESS : CNSTR_CONTACT_PYRAMIDAL;
        efc_row(m, d, efcid, pos, pos, invweight, d->con_solref + 2 * c, d->con_solimp + 5 * c, includemargin, Jqvel, 0, type, c);
      }
    }
  }
}

/* =============================================================================================
 * forward.py stages
 * ============================================================================================= */

/* forward.py:513-537 (factorize=False) */
static void fwd_position(const orc_model* m, orc_data* d) {
  kinematics(m, d);
  com_pos(m, d);
  camlight(m, d);
  flex_kinematics(m, d);
  tendon(m, d);
  crb(m, d);
  tendon_armature(m, d);
  collision(m, d);
  make_constraint(m, d);
  transmission(m, d);
}

/* forward.py:540-613 */
static void fwd_velocity(const orc_model* m, orc_data* d) {
  for (int a = 0; a < m->nu; a++) {
    real v = 0;
    for (int i = 0; i < m->nv; i++) v += d->actuator_moment[(size_t)a * m->nv + i] * d->qvel[i];
    d->actuator_velocity[a] = v;
  }
  /* forward.py:604-609 _tendon_velocity */
  for (int t = 0; t < m->ntendon; t++) {
    real v = 0;
    for (int q = 0; q < m->ten_J_rownnz[t]; q++) v += d->ten_J[m->ten_J_rowadr[t] + q] * d->qvel[m->ten_J_colind[m->ten_J_rowadr[t] + q]];
    d->ten_velocity[t] = v;
  }
  com_vel(m, d);
  passive(m, d);
  rne(m, d);
  tendon_bias(m, d, d->qfrc_bias); /* smooth.py:1878-1932; zero for fixed tendons */
}

/* support.py:38-64 next_act */
static real next_act(const orc_model* m, int a, real act, real act_dot, real scale, int clamp) {
  real dt = m->opt_timestep, r;
  int dyn = m->actuator_dyntype[a];
  if (dyn == DYN_FILTEREXACT) {
    real tau = maxr(MINVAL, m->actuator_dynprm[10 * a]);
    r = act + scale * act_dot * tau * (1 - exp(-dt / tau));
  } else if (dyn == DYN_USER) {
    return act;
  } else {
    r = act + scale * act_dot * dt;
  }
  return clamp ? clampr(r, m->actuator_actrange[2 * a], m->actuator_actrange[2 * a + 1]) : r;
}

/* util_misc.py:454-600: muscle length / velocity curves, passive force and activation dynamics;
   prm = (range[2], force, scale, lmin, lmax, vmax, fpmax, fvmax), dynprm = (tau_act, tau_deact, tausmooth) */
static real muscle_gain_length(real L, real lmin, real lmax) {
  if (lmin > L || L > lmax) return 0;
  real a = 0.5 * (lmin + 1), b = 0.5 * (1 + lmax), x;
  if (L <= a) { x = (L - lmin) / maxr(MINVAL, a - lmin); return 0.5 * x * x; }
  if (L <= 1) { x = (1 - L) / maxr(MINVAL, 1 - a); return 1 - 0.5 * x * x; }
  if (L <= b) { x = (L - 1) / maxr(MINVAL, b - 1); return 1 - 0.5 * x * x; }
  x = (lmax - L) / maxr(MINVAL, lmax - b);
  return 0.5 * x * x;
}

static real muscle_force_scale(const real* prm, real acc0) { return prm[2] < 0 ? prm[3] / maxr(MINVAL, acc0) : prm[2]; }

static real muscle_gain(real len, real vel, const real* lr, real acc0, const real* prm) {
  real force = muscle_force_scale(prm, acc0);
  real L0 = (lr[1] - lr[0]) / maxr(MINVAL, prm[1] - prm[0]);
  real L = prm[0] + (len - lr[0]) / maxr(MINVAL, L0), V = vel / maxr(MINVAL, L0 * prm[6]);
  real FL = muscle_gain_length(L, prm[4], prm[5]), fvmax = prm[8], y = fvmax - 1, FV;
  if (V <= -1) FV = 0;
  else if (V <= 0) FV = (V + 1) * (V + 1);
  else if (V <= y) FV = fvmax - (y - V) * (y - V) / maxr(MINVAL, y);
  else FV = fvmax;
  return -force * FL * FV;
}

static real muscle_bias(real len, const real* lr, real acc0, const real* prm) {
  real force = muscle_force_scale(prm, acc0);
  real L0 = (lr[1] - lr[0]) / maxr(MINVAL, prm[1] - prm[0]);
  real L = prm[0] + (len - lr[0]) / maxr(MINVAL, L0), b = 0.5 * (1 + prm[5]), x;
  if (L <= 1) return 0;
  if (L <= b) { x = (L - 1) / maxr(MINVAL, b - 1); return -force * prm[7] * 0.5 * x * x; }
  x = (L - b) / maxr(MINVAL, b - 1);
  return -force * prm[7] * (0.5 + x);
}

static real muscle_dynamics(real ctrl, real act, const real* prm) {
  real cc = clampr(ctrl, 0, 1), ac = clampr(act, 0, 1);
  real tau_act = prm[0] * (0.5 + 1.5 * ac), tau_deact = prm[1] / (0.5 + 1.5 * ac), dctrl = cc - act, tau;
  if (prm[2] < MINVAL) {
    tau = dctrl > 0 ? tau_act : tau_deact;
  } else {
    real x = dctrl / prm[2] + 0.5;
    real sig = x <= 0 ? 0 : (x >= 1 ? 1 : x * x * x * (3 * x * (2 * x - 5) + 10));
    tau = tau_deact + (tau_act - tau_deact) * sig;
  }
  return dctrl / maxr(MINVAL, tau);
}

/* forward.py:616-927: activation dynamics (integrator / filter / filterexact), actearly, gain/bias */
static void fwd_actuation(const orc_model* m, orc_data* d) {
  int nv = m->nv;
  if (!m->nu || (m->opt_disableflags & DSBL_ACTUATION)) {
    memset(d->qfrc_actuator, 0, nv * sizeof(real));
    if (m->na) memset(d->act_dot, 0, m->na * sizeof(real));
    return;
  }
  for (int a = 0; a < m->nu; a++) {
    real ctrl = d->ctrl[a];
    if (m->actuator_ctrllimited[a] && !(m->opt_disableflags & DSBL_CLAMPCTRL))
      ctrl = clampr(ctrl, m->actuator_ctrlrange[2 * a], m->actuator_ctrlrange[2 * a + 1]);
    real ctrl_act = ctrl;
    int act_first = m->actuator_actadr[a];
    if (m->na && act_first >= 0) {
      int last = act_first + m->actuator_actnum[a] - 1, dyn = m->actuator_dyntype[a];
      real act = d->act[last], act_dot = 0;
      if (dyn == DYN_INTEGRATOR) act_dot = ctrl;
      else if (dyn == DYN_FILTER || dyn == DYN_FILTEREXACT) act_dot = (ctrl - act) / maxr(m->actuator_dynprm[10 * a], MINVAL);
      else if (dyn == DYN_MUSCLE) act_dot = muscle_dynamics(ctrl, act, m->actuator_dynprm + 10 * a);  /* forward.py:671-674 */
      d->act_dot[last] = act_dot;
      ctrl_act = m->actuator_actearly[a] ? next_act(m, a, act, act_dot, 1, m->actuator_actlimited[a]) : act;
    }
    real len = d->actuator_length[a], vel = d->actuator_velocity[a];
    const real* gp = m->actuator_gainprm + 10 * a;
    const real* bp = m->actuator_biasprm + 10 * a;
    real gain = 0, bias = 0;
    if (m->actuator_gaintype[a] == GAIN_FIXED) gain = gp[0];
    else if (m->actuator_gaintype[a] == GAIN_AFFINE) gain = gp[0] + gp[1] * len + gp[2] * vel;
    if (m->actuator_biastype[a] == BIAS_AFFINE) bias = bp[0] + bp[1] * len + bp[2] * vel;
    if (m->actuator_gaintype[a] == GAIN_MUSCLE) gain = muscle_gain(len, vel, m->actuator_lengthrange + 2 * a, m->actuator_acc0[a], gp);
    if (m->actuator_biastype[a] == BIAS_MUSCLE) bias = muscle_bias(len, m->actuator_lengthrange + 2 * a, m->actuator_acc0[a], bp);
    real force = gain * ctrl_act + bias;
    if (m->actuator_forcelimited[a]) force = clampr(force, m->actuator_forcerange[2 * a], m->actuator_forcerange[2 * a + 1]);
    d->actuator_force[a] = force;
  }
  /* forward.py:739-779: total actuator force per tendon clamped to its actuatorfrcrange by scaling */
  for (int t = 0; t < m->ntendon; t++) {
    if (!m->tendon_actfrclimited[t]) continue;
    real tot = 0;
    for (int a = 0; a < m->nu; a++)
      if (m->actuator_trntype[a] == TRN_TENDON && m->actuator_trnid[2 * a] == t) tot += d->actuator_force[a];
    const real lo = m->tendon_actfrcrange[2 * t], hi = m->tendon_actfrcrange[2 * t + 1];
    for (int a = 0; a < m->nu; a++) {
      if (m->actuator_trntype[a] != TRN_TENDON || m->actuator_trnid[2 * a] != t) continue;
      if (tot < lo) d->actuator_force[a] *= lo / tot;
      else if (tot > hi) d->actuator_force[a] *= hi / tot;
    }
  }
  memset(d->qfrc_actuator, 0, nv * sizeof(real));
  for (int a = 0; a < m->nu; a++)
    for (int i = 0; i < nv; i++) d->qfrc_actuator[i] += d->actuator_moment[(size_t)a * nv + i] * d->actuator_force[a];
  for (int i = 0; i < nv; i++) {
    int j = m->dof_jntid[i];
    if (m->ngravcomp && m->jnt_actgravcomp[j]) d->qfrc_actuator[i] += d->qfrc_gravcomp[i];  /* forward.py:824-826 */
    if (m->jnt_actfrclimited[j]) d->qfrc_actuator[i] = clampr(d->qfrc_actuator[i], m->jnt_actfrcrange[2 * j], m->jnt_actfrcrange[2 * j + 1]);
  }
}

/* support.py:174-237 (apply_ft, flg_add) */
static void xfrc_accumulate(const orc_model* m, orc_data* d, real* qfrc) {
  for (int i = 0; i < m->nv; i++) {
    const real* cd = d->cdof + 6 * i;
    int db = m->dof_bodyid[i];
    real acc = 0;
    for (int b = db; b < m->nbody; b++) {
      const real* ft = d->xfrc_applied + 6 * b;
      if (ft[0] == 0 && ft[1] == 0 && ft[2] == 0 && ft[3] == 0 && ft[4] == 0 && ft[5] == 0) continue;
      int p = b;
      while (p != 0 && p != db) p = m->body_parentid[p];
      if (p == 0) continue;
      real off[3], c[3];
      for (int k = 0; k < 3; k++) off[k] = d->xipos[3 * b + k] - d->subtree_com[3 * m->body_rootid[b] + k];
      cross3(c, cd, off);
      acc += cd[3] * ft[0] + cd[4] * ft[1] + cd[5] * ft[2] + cd[0] * ft[3] + cd[1] * ft[4] + cd[2] * ft[5] + dot3(c, ft);
    }
    qfrc[i] += acc;
  }
}

/* forward.py:930-969 (factorize = True) */
static void fwd_acceleration(const orc_model* m, orc_data* d) {
  int nv = m->nv;
  for (int i = 0; i < nv; i++)
    d->qfrc_smooth[i] = d->qfrc_passive[i] - d->qfrc_bias[i] + d->qfrc_actuator[i] + d->qfrc_applied[i];
  xfrc_accumulate(m, d, d->qfrc_smooth);
  factor_m(m, nv, d->qM, d->qLD);
  solve_m(m, nv, d->qLD, d->qfrc_smooth, d->qacc_smooth);
}

/* =============================================================================================
 * solver.py (primal CG / Newton, pyramidal cones, iterative linesearch)
 * ============================================================================================= */
typedef struct {
  real* Jaref; real* jv;
  real* quad;  /* 9 per row: the elliptic primary row's quad, quad1, quad2 (solver.py:1550-1611) */
  real* grad; real* Mgrad; real* search; real* mv; real* prev_grad; real* prev_Mgrad;
  real* H; real* HL;
  real cost, prev_cost, gauss, search_dot, grad_dot;
  int done;
} solver_ctx;

static void matvec(int n, const real* M, const real* x, real* y) {
  for (int i = 0; i < n; i++) {
    real s = 0;
    for (int j = 0; j < n; j++) s += M[i * n + j] * x[j];
    y[i] = s;
  }
}

/* solver.py:2154-2219 + 1805-1951 (non-elliptic) + 1987-2051 */
static void update_constraint(const orc_model* m, orc_data* d, solver_ctx* c) {
  int nv = m->nv, nefc = *d->nefc < d->njmax ? *d->nefc : d->njmax;
  int ne = *d->ne, nf = *d->nf;
  c->gauss = 0;
  c->prev_cost = c->cost;
  c->cost = 0;
  for (int r = 0; r < nefc; r++) {
    real D = d->efc_D[r], Jaref = c->Jaref[r];
    int state;
    if (r < ne) {
      d->efc_force[r] = -D * Jaref; state = STATE_QUADRATIC; c->cost += (real)0.5 * D * Jaref * Jaref;
    } else if (r < ne + nf) {
      real f = d->efc_frictionloss[r], rf = safe_div(f, D);
      if (Jaref <= -rf) { d->efc_force[r] = f; state = STATE_LINEARNEG; c->cost += -f * ((real)0.5 * rf + Jaref); }
      else if (Jaref >= rf) { d->efc_force[r] = -f; state = STATE_LINEARPOS; c->cost += -f * ((real)0.5 * rf - Jaref); }
      else { d->efc_force[r] = -D * Jaref; state = STATE_QUADRATIC; c->cost += (real)0.5 * D * Jaref * Jaref; }
    } else if (d->efc_type[r] != CNSTR_CONTACT_ELLIPTIC) {
      if (Jaref >= 0) { d->efc_force[r] = 0; state = STATE_SATISFIED; }
      else { d->efc_force[r] = -D * Jaref; state = STATE_QUADRATIC; c->cost += (real)0.5 * D * Jaref * Jaref; }
    } else {
      /* elliptic friction cone, solver.py:1886-1942 */
      int con = d->efc_id[r], dim = d->con_dim[con];
      const real* fr = d->con_friction + 5 * con;
      real mu = fr[0] * m->opt_impratio_invsqrt;
      int r0 = d->con_efc_address[10 * con];
      real N = c->Jaref[r0] * mu, uf = 0, TT = 0;
      int cut = r0 < 0;
      for (int j = 1; j < dim && !cut; j++) {
        int rj = d->con_efc_address[10 * con + j];
        if (rj < 0) { cut = 1; break; }  /* rows past njmax: the reference leaves the row untouched */
        real uj = c->Jaref[rj] * fr[j - 1];
        TT += uj * uj;
        if (rj == r) uf = uj * fr[j - 1];
      }
      if (cut) { d->efc_force[r] = 0; d->efc_state[r] = STATE_SATISFIED; continue; }
      real T = TT <= 0 ? 0 : sqrt(TT);
      if (N >= mu * T || (T <= 0 && N >= 0)) {
        d->efc_force[r] = 0; state = STATE_SATISFIED;
      } else if (mu * N + T <= 0 || (T <= 0 && N < 0)) {
        d->efc_force[r] = -D * Jaref; state = STATE_QUADRATIC; c->cost += (real)0.5 * D * Jaref * Jaref;
      } else {
        real dm = safe_div(d->efc_D[r0], mu * mu * (1 + mu * mu));
        real nmt = N - mu * T;
        real force = -dm * nmt * mu;
        if (r == r0) { d->efc_force[r] = force; c->cost += (real)0.5 * dm * nmt * nmt; }
        else d->efc_force[r] = -safe_div(force, T) * uf;
        state = STATE_CONE;
      }
    }
    d->efc_state[r] = state;
  }
  for (int i = 0; i < nv; i++) {
    real s = 0;
    for (int r = 0; r < nefc; r++) s += d->efc_J[(size_t)r * nv + i] * d->efc_force[r];
    d->qfrc_constraint[i] = s;
  }
  real g = 0;
  for (int i = 0; i < nv; i++) g += (d->efc_Ma[i] - d->qfrc_smooth[i]) * (d->qacc[i] - d->qacc_smooth[i]);
  c->gauss += (real)0.5 * g;
  c->cost += (real)0.5 * g;
}

/* solver.py:2879-3008 (CG: Mgrad = M^-1 grad; Newton: H = M + J' D_active J, Cholesky) */
static void update_gradient(const orc_model* m, orc_data* d, solver_ctx* c) {
  int nv = m->nv, nefc = *d->nefc < d->njmax ? *d->nefc : d->njmax;
  c->grad_dot = 0;
  for (int i = 0; i < nv; i++) {
    real g = d->efc_Ma[i] - d->qfrc_smooth[i] - d->qfrc_constraint[i];
    c->grad[i] = g;
    c->grad_dot += g * g;
  }
  if (m->opt_solver == SOLVER_CG) {
    solve_m(m, nv, d->qLD, c->grad, c->Mgrad);
  } else {
    memcpy(c->H, d->qM, (size_t)nv * nv * sizeof(real));
    for (int r = 0; r < nefc; r++) {
      if (d->efc_state[r] != STATE_QUADRATIC) continue;
      real D = d->efc_D[r];
      const real* J = d->efc_J + (size_t)r * nv;
      for (int i = 0; i < nv; i++) {
        if (J[i] == 0) continue;
        for (int j = 0; j < nv; j++) c->H[i * nv + j] += D * J[i] * J[j];
      }
    }
    /* elliptic cones in the CONE state: H += J_c' C J_c with the cone Hessian C of the contact
     * (update_gradient_JTCJ, solver.py:2430-2585) */
    for (int r0 = 0; r0 < nefc; r0++) {
      if (d->efc_type[r0] != CNSTR_CONTACT_ELLIPTIC || d->efc_state[r0] != STATE_CONE) continue;
      int con = d->efc_id[r0];
      if (d->con_efc_address[10 * con] != r0) continue;
      int dim = d->con_dim[con];
      const real* fr = d->con_friction + 5 * con;
      real mu = fr[0] * m->opt_impratio_invsqrt, mu2 = mu * mu;
      real dm = safe_div(d->efc_D[r0], mu2 * (1 + mu2));
      if (dm == 0) continue;
      real u[6], fri[6];
      int rows[6];
      u[0] = c->Jaref[r0] * mu;
      fri[0] = mu;
      rows[0] = r0;
      real tt = 0;
      int cut = 0;
      for (int j = 1; j < dim; j++) {
        rows[j] = d->con_efc_address[10 * con + j];
        if (rows[j] < 0) { cut = 1; break; }
        u[j] = c->Jaref[rows[j]] * fr[j - 1];
        fri[j] = fr[j - 1];
        tt += u[j] * u[j];
      }
      if (cut) continue;
      real t = tt <= 0 ? 0 : sqrt(tt);
      t = maxr(t, MINVAL);
      real ttt = maxr(t * t * t, MINVAL);
      real mu_over_t = safe_div(mu, t), mu_n_over_ttt = mu * safe_div(u[0], ttt), diag = mu2 - mu * safe_div(u[0], t);
      for (int a = 0; a < dim; a++) {
        for (int b = 0; b < dim; b++) {
          real h;
          if (a == 0 && b == 0) h = 1;
          else if (a == 0) h = -mu_over_t * u[b];
          else if (b == 0) h = -mu_over_t * u[a];
          else h = mu_n_over_ttt * u[a] * u[b] + (a == b ? diag : 0);
          h *= dm * fri[a] * fri[b];
          if (h == 0) continue;
          const real* Ja = d->efc_J + (size_t)rows[a] * nv;
          const real* Jb = d->efc_J + (size_t)rows[b] * nv;
          for (int i = 0; i < nv; i++) {
            if (Ja[i] == 0) continue;
            for (int j = 0; j < nv; j++) c->H[i * nv + j] += h * Ja[i] * Jb[j];
          }
        }
      }
    }
    cholesky(nv, c->H, c->HL);
    cholesky_solve(nv, c->HL, c->grad, c->Mgrad);
  }
}

/* elliptic cone (cost, grad, hess) of one contact at alpha, solver.py:263-323 (_eval_elliptic) */
static void eval_elliptic(real mu, const real* quad, const real* quad1, const real* quad2, real alpha, real* out) {
  real u0 = quad1[0], v0 = quad1[1], uu = quad1[2], uv = quad2[0], vv = quad2[1], dm = quad2[2];
  real N = u0 + alpha * v0;
  real Tsqr = uu + alpha * (2 * uv + alpha * vv);
  int bottom = 0;
  if (Tsqr <= 0) {
    if (N < 0) bottom = 1;
    else return;
  } else {
    real T = sqrt(Tsqr);
    if (N >= mu * T) return;
    if (mu * N + T <= 0) bottom = 1;
    else {
      real N1 = v0, T1 = (uv + alpha * vv) / T;
      real T2 = vv / T - (uv + alpha * vv) * T1 / (T * T);
      out[0] += (real)0.5 * dm * (N - mu * T) * (N - mu * T);
      out[1] += dm * (N - mu * T) * (N1 - mu * T1);
      out[2] += dm * ((N1 - mu * T1) * (N1 - mu * T1) + (N - mu * T) * (-mu * T2));
      return;
    }
  }
  if (bottom) {
    real aq2 = alpha * quad[2];
    out[0] += alpha * aq2 + alpha * quad[1] + quad[0];
    out[1] += 2 * aq2 + quad[1];
    out[2] += 2 * quad[2];
  }
}

/* per-row (cost, grad, hess), solver.py:570-640; an elliptic contact is evaluated once, at its first
 * row, from the quad coefficients linesearch() prepared */
static void eval_row(const orc_model* m, const orc_data* d, const solver_ctx* c, int r, int ne, int nf, real alpha, real* out) {
  real D = d->efc_D[r], jaref = c->Jaref[r], jv = c->jv[r];
  real x = jaref + alpha * jv;
  if (r >= ne + nf && d->efc_type[r] == CNSTR_CONTACT_ELLIPTIC) {
    int con = d->efc_id[r];
    if (d->con_efc_address[10 * con] != r) return;
    const real* q = c->quad + 9 * (size_t)r;
    eval_elliptic(d->con_friction[5 * con] * m->opt_impratio_invsqrt, q, q + 3, q + 6, alpha, out);
    return;
  }
  if (r >= ne + nf) {
    if (x < 0) { real jvD = jv * D; out[0] += (real)0.5 * D * x * x; out[1] += jvD * x; out[2] += jv * jvD; }
    return;
  }
  if (r >= ne) {
    real f = d->efc_frictionloss[r], rf = safe_div(f, D);
    if ((-rf < x) && (x < rf)) { real jvD = jv * D; out[0] += (real)0.5 * D * x * x; out[1] += jvD * x; out[2] += jv * jvD; }
    else if (x <= -rf) { out[0] += f * (-(real)0.5 * rf - x); out[1] += -f * jv; }
    else { out[0] += f * (-(real)0.5 * rf + x); out[1] += f * jv; }
    return;
  }
  real jvD = jv * D;
  out[0] += (real)0.5 * D * x * x; out[1] += jvD * x; out[2] += jv * jvD;
}

static int in_bracket(const real* x, const real* y) { return (x[1] < y[1] && y[1] < 0) || (x[1] > y[1] && y[1] > 0); }

/* solver.py:886-1341 (linesearch_iterative) + :1662-1703 */
static void linesearch(const orc_model* m, orc_data* d, solver_ctx* c) {
  int nv = m->nv, ne = *d->ne, nf = *d->nf;
  int nefc = *d->nefc < d->njmax ? *d->nefc : d->njmax;
  matvec(nv, d->qM, c->search, c->mv);
  for (int r = 0; r < nefc; r++) {
    real s = 0;
    const real* J = d->efc_J + (size_t)r * nv;
    for (int i = 0; i < nv; i++) s += J[i] * c->search[i];
    c->jv[r] = s;
  }
  /* elliptic contacts: quad / quad1 / quad2 at the first row (solver.py:1550-1611) */
  if (m->opt_cone == CONE_ELLIPTIC) {
    for (int r = ne + nf; r < nefc; r++) {
      if (d->efc_type[r] != CNSTR_CONTACT_ELLIPTIC) continue;
      int con = d->efc_id[r];
      if (d->con_efc_address[10 * con] != r) continue;
      int dim = d->con_dim[con];
      const real* fr = d->con_friction + 5 * con;
      real mu = fr[0] * m->opt_impratio_invsqrt;
      real Jaref = c->Jaref[r], jv = c->jv[r], D = d->efc_D[r];
      real* q = c->quad + 9 * (size_t)r;
      q[0] = (real)0.5 * Jaref * Jaref * D; q[1] = jv * Jaref * D; q[2] = (real)0.5 * jv * jv * D;
      real uu = 0, uv = 0, vv = 0;
      int cut = 0;
      for (int j = 1; j < dim; j++) {
        int rj = d->con_efc_address[10 * con + j];
        if (rj < 0) { cut = 1; break; }
        real jvj = c->jv[rj], jarefj = c->Jaref[rj], dj = d->efc_D[rj], DJj = dj * jarefj;
        q[0] += (real)0.5 * jarefj * DJj; q[1] += jvj * DJj; q[2] += (real)0.5 * jvj * dj * jvj;
        real uj = jarefj * fr[j - 1], vj = jvj * fr[j - 1];
        uu += uj * uj; uv += uj * vj; vv += vj * vj;
      }
      q[3] = Jaref * mu; q[4] = jv * mu; q[5] = uu;
      q[6] = uv; q[7] = vv; q[8] = D / (mu * mu * (1 + mu * mu));
      if (cut) memset(q, 0, 9 * sizeof(real));  /* a contact cut by njmax contributes nothing */
    }
  }
  real snorm = sqrt(c->search_dot);
  real scale = m->stat_meaninertia * (real)nv;
  real gtol = maxr(m->opt_tolerance * m->opt_ls_tolerance * snorm * scale, (real)1e-6);
  real p0s[3] = {0, 0, 0};
  for (int r = 0; r < nefc; r++) eval_row(m, d, c, r, ne, nf, 0, p0s);
  real qg1 = 0, qg2 = 0;
  for (int i = 0; i < nv; i++) {
    qg1 += c->search[i] * (d->efc_Ma[i] - d->qfrc_smooth[i]);
    qg2 += (real)0.5 * c->search[i] * c->mv[i];
  }
  real qg[3] = {c->gauss, qg1, qg2};
  real p0[3] = {qg[0] + p0s[0], qg[1] + p0s[1], 2 * qg[2] + p0s[2]};
#define EVAL_GAUSS(out, a) { out[0] = (a) * (a) * qg[2] + (a) * qg[1] + qg[0]; out[1] = 2 * (a) * qg[2] + qg[1]; out[2] = 2 * qg[2]; }
  real alpha;
  real lo_alpha_in = 0, lo_in[3] = {0, 0, 0};
  int initial_converged;
  if (m->opt_ls_parallel) {
    /* solver.py:325-478 linesearch_parallel: the cheapest of ls_iterations step sizes log-spaced over
       [ls_parallel_min_step, 1] (_log_scale :325-327), the first on ties */
    int n = m->opt_ls_iterations;
    real step = (log((real)1) - log(m->opt_ls_parallel_min_step)) / maxr(1, (real)(n - 1)), best = (real)1e10;
    alpha = 0;
    for (int i = 0; i < n; i++) {
      real al = exp(log(m->opt_ls_parallel_min_step) + (real)i * step), v[3];
      EVAL_GAUSS(v, al);
      for (int r = 0; r < nefc; r++) eval_row(m, d, c, r, ne, nf, al, v);
      if (v[0] < best) { best = v[0]; alpha = al; }
    }
    lo_alpha_in = alpha;
    initial_converged = 1;
  } else {
    lo_alpha_in = -safe_div(p0[1], p0[2]);
    EVAL_GAUSS(lo_in, lo_alpha_in);
    for (int r = 0; r < nefc; r++) eval_row(m, d, c, r, ne, nf, lo_alpha_in, lo_in);
    initial_converged = fabs(lo_in[1]) < gtol && lo_in[0] < p0[0];
  }
  if (!initial_converged) {
    alpha = 0;
    int lo_less = lo_in[1] < p0[1];
    real lo[3], hi[3], lo_alpha, hi_alpha;
    if (lo_less) { memcpy(lo, lo_in, sizeof(lo)); lo_alpha = lo_alpha_in; memcpy(hi, p0, sizeof(hi)); hi_alpha = 0; }
    else { memcpy(lo, p0, sizeof(lo)); lo_alpha = 0; memcpy(hi, lo_in, sizeof(hi)); hi_alpha = lo_alpha_in; }
    for (int it = 0; it < m->opt_ls_iterations; it++) {
      real lo_next_alpha = lo_alpha - safe_div(lo[1], lo[2]);
      real hi_next_alpha = hi_alpha - safe_div(hi[1], hi[2]);
      real mid_alpha = (real)0.5 * (lo_alpha + hi_alpha);
      real lo_next[3], hi_next[3], mid[3];
      EVAL_GAUSS(lo_next, lo_next_alpha);
      EVAL_GAUSS(hi_next, hi_next_alpha);
      EVAL_GAUSS(mid, mid_alpha);
      for (int r = 0; r < nefc; r++) {
        eval_row(m, d, c, r, ne, nf, lo_next_alpha, lo_next);
        eval_row(m, d, c, r, ne, nf, hi_next_alpha, hi_next);
        eval_row(m, d, c, r, ne, nf, mid_alpha, mid);
      }
      int s1 = in_bracket(lo, lo_next);
      if (s1) { memcpy(lo, lo_next, sizeof(lo)); lo_alpha = lo_next_alpha; }
      int s2 = in_bracket(lo, mid);
      if (s2) { memcpy(lo, mid, sizeof(lo)); lo_alpha = mid_alpha; }
      int s3 = in_bracket(lo, hi_next);
      if (s3) { memcpy(lo, hi_next, sizeof(lo)); lo_alpha = hi_next_alpha; }
      int swap_lo = s1 || s2 || s3;
      int h1 = in_bracket(hi, hi_next);
      if (h1) { memcpy(hi, hi_next, sizeof(hi)); hi_alpha = hi_next_alpha; }
      int h2 = in_bracket(hi, mid);
      if (h2) { memcpy(hi, mid, sizeof(hi)); hi_alpha = mid_alpha; }
      int h3 = in_bracket(hi, lo_next);
      if (h3) { memcpy(hi, lo_next, sizeof(hi)); hi_alpha = lo_next_alpha; }
      int swap_hi = h1 || h2 || h3;
      int ls_done = (!swap_lo && !swap_hi) || (lo[1] < 0 && lo[1] > -gtol) || (hi[1] > 0 && hi[1] < gtol);
      int improved = lo[0] < p0[0] || hi[0] < p0[0];
      int lo_better = lo[0] < hi[0];
      if (improved && lo_better) alpha = lo_alpha;
      if (improved && !lo_better) alpha = hi_alpha;
      if (ls_done) break;
    }
  } else {
    alpha = lo_alpha_in;
  }
#undef EVAL_GAUSS
  for (int i = 0; i < nv; i++) { d->qacc[i] += alpha * c->search[i]; d->efc_Ma[i] += alpha * c->mv[i]; }
  for (int r = 0; r < nefc; r++) c->Jaref[r] += alpha * c->jv[r];
}

/* solver.py:3296-3343 (+ init_context :3257-3293, iteration :3187-3254) */
static void solve(const orc_model* m, orc_data* d) {
  int nv = m->nv, njmax = d->njmax;
  if (njmax == 0 || nv == 0) {
    memcpy(d->qacc, d->qacc_smooth, nv * sizeof(real));
    *d->solver_niter = 0;
    return;
  }
  real* buf = (real*)calloc((size_t)11 * njmax + 8 * (size_t)nv + 2 * (size_t)nv * nv, sizeof(real));
  solver_ctx c;
  c.Jaref = buf; c.jv = buf + njmax; c.quad = buf + 2 * (size_t)nv * nv + 8 * (size_t)nv + 2 * njmax;
  c.grad = buf + 2 * njmax; c.Mgrad = c.grad + nv; c.search = c.Mgrad + nv; c.mv = c.search + nv;
  c.prev_grad = c.mv + nv; c.prev_Mgrad = c.prev_grad + nv; c.H = c.prev_Mgrad + 2 * nv; c.HL = c.H + nv * nv;
  if (!(m->opt_disableflags & DSBL_WARMSTART)) memcpy(d->qacc, d->qacc_warmstart, nv * sizeof(real));
  else memcpy(d->qacc, d->qacc_smooth, nv * sizeof(real));
  int nefc = *d->nefc < njmax ? *d->nefc : njmax;
  *d->solver_niter = 0;
  c.search_dot = 0;
  c.cost = MAXVAL;
  c.done = 0;
  for (int r = 0; r < nefc; r++) {
    real s = 0;
    for (int i = 0; i < nv; i++) s += d->efc_J[(size_t)r * nv + i] * d->qacc[i];
    c.Jaref[r] = s - d->efc_aref[r];
  }
  matvec(nv, d->qM, d->qacc, d->efc_Ma);
  update_constraint(m, d, &c);
  update_gradient(m, d, &c);
  for (int i = 0; i < nv; i++) { c.search[i] = -c.Mgrad[i]; c.search_dot += c.search[i] * c.search[i]; }
  real scale = 1 / (m->stat_meaninertia * (real)nv);
  if (m->opt_iterations != 0) {
    while (!c.done) {
      linesearch(m, d, &c);
      if (m->opt_solver == SOLVER_CG) {
        memcpy(c.prev_grad, c.grad, nv * sizeof(real));
        memcpy(c.prev_Mgrad, c.Mgrad, nv * sizeof(real));
      }
      update_constraint(m, d, &c);
      update_gradient(m, d, &c);
      real beta = 0;
      if (m->opt_solver == SOLVER_CG) {
        real num = 0, den = 0;
        for (int i = 0; i < nv; i++) {
          num += c.grad[i] * (c.Mgrad[i] - c.prev_Mgrad[i]);
          den += c.prev_grad[i] * c.prev_Mgrad[i];
        }
        beta = maxr(0, num / maxr(MINVAL, den));
      }
      c.search_dot = 0;
      for (int i = 0; i < nv; i++) {
        real s = -c.Mgrad[i];
        if (m->opt_solver == SOLVER_CG) s += beta * c.search[i];
        c.search[i] = s;
        c.search_dot += s * s;
      }
      (*d->solver_niter)++;
      real improvement = (c.prev_cost - c.cost) * scale;
      real gradient = sqrt(c.grad_dot) * scale;
      int done = (improvement < m->opt_tolerance) || (gradient < m->opt_tolerance);
      if (done || *d->solver_niter == m->opt_iterations) c.done = 1;
    }
  }
  *d->solver_cost = c.cost;
  free(buf);
}

/* forward.py:51-354 (_advance + euler with optional implicit damping) */
/* forward.py:213-274 _advance */
static void euler_advance(const orc_model* m, orc_data* d, const real* qacc_adv) {
  int nv = m->nv;
  real dt = m->opt_timestep;
  /* _next_activation: na-sized, skipped when na == 0 */
  for (int a = 0; a < m->nu; a++) {
    int adr = m->actuator_actadr[a];
    for (int j = adr; j >= 0 && j < adr + m->actuator_actnum[a]; j++) {
      d->act[j] = next_act(m, a, d->act[j], d->act_dot[j], 1, m->actuator_actlimited[a]);
    }
  }
  for (int i = 0; i < nv; i++) d->qvel[i] = d->qvel[i] + qacc_adv[i] * dt;
  for (int j = 0; j < m->njnt; j++) {
    int qa = m->jnt_qposadr[j], da = m->jnt_dofadr[j], jt = m->jnt_type[j];
    if (jt == JNT_FREE) {
      for (int i = 0; i < 3; i++) d->qpos[qa + i] = d->qpos[qa + i] + dt * d->qvel[da + i];
      real qn[4];
      quat_integrate(qn, d->qpos + qa + 3, d->qvel + da + 3, dt);
      memcpy(d->qpos + qa + 3, qn, sizeof(qn));
    } else if (jt == JNT_BALL) {
      real qn[4];
      quat_integrate(qn, d->qpos + qa, d->qvel + da, dt);
      memcpy(d->qpos + qa, qn, sizeof(qn));
    } else {
      d->qpos[qa] = d->qpos[qa] + dt * d->qvel[da];
    }
  }
  d->time[0] += dt;
  memcpy(d->qacc_warmstart, d->qacc, nv * sizeof(real));
}

/* forward.py:326-354 euler (implicit damping when EULERDAMP is enabled) */
static void euler(const orc_model* m, orc_data* d) {
  int nv = m->nv;
  real dt = m->opt_timestep;
  if (m->opt_disableflags & (DSBL_EULERDAMP | DSBL_DAMPER)) {
    euler_advance(m, d, d->qacc);
    return;
  }
  real* tmp = (real*)malloc(((size_t)2 * nv * nv + nv) * sizeof(real));
  real* Mi = tmp;
  real* L = tmp + (size_t)nv * nv;
  real* q = L + (size_t)nv * nv;
  memcpy(Mi, d->qM, (size_t)nv * nv * sizeof(real));
  for (int i = 0; i < nv; i++) Mi[i * nv + i] += dt * m->dof_damping[i];
  factor_m(m, nv, Mi, L);
  solve_m(m, nv, L, d->efc_Ma, q);
  euler_advance(m, d, q);
  free(tmp);
}

static void implicit(const orc_model* m, orc_data* d);

/* forward.py:1003-1018: the integrator selected by the model */
static void integrate(const orc_model* m, orc_data* d) {
  if (m->opt_integrator == INTEGRATOR_IMPLICITFAST) implicit(m, d);
  else euler(m, d);
}

/* derivative.py:36-107 _qderiv_actuator_passive_vel: d(actuator force)/d(velocity) scale */
static real actuator_vel_deriv(const orc_model* m, const orc_data* d, int a) {
  real gain = m->actuator_gaintype[a] == GAIN_AFFINE ? m->actuator_gainprm[10 * a + 2] : 0;
  real bias = m->actuator_biastype[a] == BIAS_AFFINE ? m->actuator_biasprm[10 * a + 2] : 0;
  if (bias == 0 && gain == 0) return 0;
  if (m->actuator_forcelimited[a]) {
    real f = d->actuator_force[a];
    if (f <= m->actuator_forcerange[2 * a] || f >= m->actuator_forcerange[2 * a + 1]) return 0;
  }
  real vel = bias;
  if (m->actuator_dyntype[a] != DYN_NONE) {
    if (gain != 0) {
      int adr = m->actuator_actadr[a] + m->actuator_actnum[a] - 1;
      vel += gain * (m->actuator_actearly[a] ? next_act(m, a, d->act[adr], d->act_dot[adr], 1, m->actuator_actlimited[a]) : d->act[adr]);
    }
  } else if (gain != 0) {
    vel += gain * d->ctrl[a];
  }
  return vel;
}

/* forward.py:494-510 implicit() + derivative.py:320-416 deriv_smooth_vel (implicitfast):
 * (qM - dt * qDeriv) qacc = Ma with qDeriv = sum_a vel_a m_a m_a' - diag(damping) on the tree pattern */
static void implicit(const orc_model* m, orc_data* d) {
  int nv = m->nv;
  real dt = m->opt_timestep;
  int flags = m->opt_disableflags;
  if ((flags & (DSBL_ACTUATION | DSBL_SPRING | DSBL_DAMPER)) == (DSBL_ACTUATION | DSBL_SPRING | DSBL_DAMPER)) {
    euler_advance(m, d, d->qacc);
    return;
  }
  real* A = (real*)malloc(((size_t)2 * nv * nv + nv + m->nu) * sizeof(real));
  real* L = A + (size_t)nv * nv;
  real* q = L + (size_t)nv * nv;
  real* vel = q + nv;
  for (int a = 0; a < m->nu; a++) vel[a] = (flags & DSBL_ACTUATION) ? 0 : actuator_vel_deriv(m, d, a);
  for (int i = 0; i < nv; i++)
    for (int j = 0; j < nv; j++) A[i * nv + j] = 0;
  for (int i = 0; i < nv; i++) {
    for (int j = i; j > -1; j = m->dof_parentid[j]) { /* qM_fullm pattern (io.py:601-607) */
      real qd = 0;
      for (int a = 0; a < m->nu; a++)
        if (vel[a] != 0) qd += d->actuator_moment[a * nv + i] * d->actuator_moment[a * nv + j] * vel[a];
      if (!(flags & DSBL_DAMPER) && i == j) qd -= m->dof_damping[i];
      /* derivative.py:267-320 _qderiv_tendon_damping: - sum_t damping_t J_ti J_tj on the qM pattern */
      if (!(flags & DSBL_DAMPER)) {
        for (int t = 0; t < m->ntendon; t++) {
          if (m->tendon_damping[t] == 0) continue;
          real Ji = 0, Jj = 0;
          for (int k = 0; k < m->ten_J_rownnz[t]; k++) {
            const int e = m->ten_J_rowadr[t] + k;
            if (m->ten_J_colind[e] == i) Ji = d->ten_J[e];
            if (m->ten_J_colind[e] == j) Jj = d->ten_J[e];
          }
          qd -= Ji * Jj * m->tendon_damping[t];
        }
      }
      qd *= dt;
      A[i * nv + j] = d->qM[i * nv + j] - qd;
      A[j * nv + i] = A[i * nv + j];
    }
  }
  factor_m(m, nv, A, L);
  solve_m(m, nv, L, d->efc_Ma, q);
  euler_advance(m, d, q);
  free(A);
}


/* =============================================================================================
 * sensor.py (position / velocity / acceleration sensors) + smooth.py rne_postconstraint
 * ============================================================================================= */
enum { DATATYPE_REAL = 0, DATATYPE_POSITIVE = 1 };
enum { STAGE_POS = 1, STAGE_VEL = 2, STAGE_ACC = 3 };
enum {
  SENS_ACCELEROMETER = 1, SENS_VELOCIMETER = 2, SENS_GYRO = 3, SENS_FORCE = 4, SENS_TORQUE = 5, SENS_MAGNETOMETER = 6,
  SENS_JOINTPOS = 9, SENS_JOINTVEL = 10, SENS_ACTUATORPOS = 13, SENS_ACTUATORVEL = 14, SENS_ACTUATORFRC = 15,
  SENS_JOINTACTFRC = 16, SENS_BALLQUAT = 18, SENS_BALLANGVEL = 19, SENS_FRAMEPOS = 26, SENS_FRAMEQUAT = 27,
  SENS_FRAMEXAXIS = 28, SENS_FRAMEYAXIS = 29, SENS_FRAMEZAXIS = 30, SENS_FRAMELINVEL = 31, SENS_FRAMEANGVEL = 32,
  SENS_FRAMELINACC = 33, SENS_FRAMEANGACC = 34, SENS_SUBTREECOM = 35, SENS_CLOCK = 45, SENS_CAMPROJECTION = 8
};

/* sensor.py:54-110 _write_scalar / _write_vector: cutoff clamps REAL, caps POSITIVE */
static void sensor_write(const orc_model* m, orc_data* d, int s, const real* v, int dim) {
  real cutoff = m->sensor_cutoff[s];
  int dt = m->sensor_datatype[s];
  real* out = d->sensordata + m->sensor_adr[s];
  for (int i = 0; i < dim; i++) {
    real x = v[i];
    int clip = cutoff > 0 && m->sensor_type[s] != 41; /* sensor.py:69, 98: never GEOMFROMTO */
    if (clip && dt == DATATYPE_REAL) x = clampr(x, -cutoff, cutoff);
    else if (clip && dt == DATATYPE_POSITIVE) x = minr(x, cutoff);
    out[i] = x;
  }
}

/* object frame position / rotation / body (sensor.py:282-340, :1011-1050) */
static void obj_frame(const orc_model* m, const orc_data* d, int type, int id, const real** pos, const real** mat, int* body) {
  static const real zero[3] = {0, 0, 0};
  static const real eye[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  *pos = zero; *mat = eye; *body = 0;
  if (type == OBJ_BODY) { *pos = d->xipos + 3 * id; *mat = d->ximat + 9 * id; *body = id; }
  else if (type == OBJ_XBODY) { *pos = d->xpos + 3 * id; *mat = d->xmat + 9 * id; *body = id; }
  else if (type == OBJ_GEOM) { *pos = d->geom_xpos + 3 * id; *mat = d->geom_xmat + 9 * id; *body = m->geom_bodyid[id]; }
  else if (type == OBJ_SITE) { *pos = d->site_xpos + 3 * id; *mat = d->site_xmat + 9 * id; *body = m->site_bodyid[id]; }
  else if (type == OBJ_CAMERA) { *pos = d->cam_xpos + 3 * id; *mat = d->cam_xmat + 9 * id; *body = m->cam_bodyid[id]; }
}

/* r = M^T v */
static void mat_t_vec(real* r, const real* M, const real* v) {
  for (int i = 0; i < 3; i++) r[i] = M[i] * v[0] + M[3 + i] * v[1] + M[6 + i] * v[2];
}

/* sensor.py:394-446 _frame_quat */
static void frame_quat(const orc_model* m, const orc_data* d, int type, int id, real* q) {
  q[0] = 1; q[1] = q[2] = q[3] = 0;
  if (type == OBJ_BODY) mul_quat(q, d->xquat + 4 * id, m->body_iquat + 4 * id);
  else if (type == OBJ_XBODY) memcpy(q, d->xquat + 4 * id, 4 * sizeof(real));
  else if (type == OBJ_GEOM) mul_quat(q, d->xquat + 4 * m->geom_bodyid[id], m->geom_quat + 4 * id);
  else if (type == OBJ_SITE) mul_quat(q, d->xquat + 4 * m->site_bodyid[id], m->site_quat + 4 * id);
  else if (type == OBJ_CAMERA) mul_quat(q, d->xquat + 4 * m->cam_bodyid[id], m->cam_quat + 4 * id);
}

#include "oracle_sensor.h"

/* sensor.py:459-706 (_sensor_pos, supported types) */
static void sensor_pos(const orc_model* m, orc_data* d) {
  sensor_extra(m, d, STAGE_POS);
  for (int s = 0; s < m->nsensor; s++) {
    if (m->sensor_needstage[s] != STAGE_POS) continue;
    int t = m->sensor_type[s], id = m->sensor_objid[s], ot = m->sensor_objtype[s];
    int rid = m->sensor_refid[s], rt = m->sensor_reftype[s];
    real v[4] = {0, 0, 0, 0};
    if (t == SENS_MAGNETOMETER) {
      mat_t_vec(v, d->site_xmat + 9 * id, m->opt_magnetic);
      sensor_write(m, d, s, v, 3);
    } else if (t == SENS_JOINTPOS) {
      v[0] = d->qpos[m->jnt_qposadr[id]];
      sensor_write(m, d, s, v, 1);
    } else if (t == SENS_ACTUATORPOS) {
      v[0] = d->actuator_length[id];
      sensor_write(m, d, s, v, 1);
    } else if (t == SENS_BALLQUAT) {
      memcpy(v, d->qpos + m->jnt_qposadr[id], 4 * sizeof(real));
      normalize4(v);
      sensor_write(m, d, s, v, 4);
    } else if (t == SENS_FRAMEPOS) {
      const real *p, *R; int b;
      obj_frame(m, d, ot, id, &p, &R, &b);
      if (rid == -1) { memcpy(v, p, 3 * sizeof(real)); }
      else {
        /* reference branch order (sensor.py:323-336): the XBODY test reads objtype */
        const real *pr, *Rr; int br;
        if (rt == OBJ_BODY) obj_frame(m, d, OBJ_BODY, rid, &pr, &Rr, &br);
        else if (ot == OBJ_XBODY) obj_frame(m, d, OBJ_XBODY, rid, &pr, &Rr, &br);
        else if (rt == OBJ_GEOM || rt == OBJ_SITE || rt == OBJ_CAMERA) obj_frame(m, d, rt, rid, &pr, &Rr, &br);
        else obj_frame(m, d, OBJ_UNKNOWN, rid, &pr, &Rr, &br);
        real dif[3] = {p[0] - pr[0], p[1] - pr[1], p[2] - pr[2]};
        mat_t_vec(v, Rr, dif);
      }
      sensor_write(m, d, s, v, 3);
    } else if (t == SENS_FRAMEXAXIS || t == SENS_FRAMEYAXIS || t == SENS_FRAMEZAXIS) {
      int ax = t - SENS_FRAMEXAXIS;
      const real *p, *R; int b;
      obj_frame(m, d, ot, id, &p, &R, &b);
      real a[3] = {R[ax], R[3 + ax], R[6 + ax]};
      if (rid == -1) memcpy(v, a, 3 * sizeof(real));
      else {
        const real *pr, *Rr; int br;
        obj_frame(m, d, rt, rid, &pr, &Rr, &br);
        mat_t_vec(v, Rr, a);
      }
      sensor_write(m, d, s, v, 3);
    } else if (t == SENS_FRAMEQUAT) {
      real q[4];
      frame_quat(m, d, ot, id, q);
      if (rid == -1) memcpy(v, q, sizeof(q));
      else {
        real qr[4], qi[4];
        frame_quat(m, d, rt, rid, qr);
        qi[0] = qr[0]; qi[1] = -qr[1]; qi[2] = -qr[2]; qi[3] = -qr[3];
        mul_quat(v, qi, q);
      }
      sensor_write(m, d, s, v, 4);
    } else if (t == SENS_CAMPROJECTION) {
      /* sensor.py:128-190: proj = image @ focal @ rotation @ translation applied to [site_xpos; 1] */
      const real* sp = d->site_xpos + 3 * id;
      const real* cp = d->cam_xpos + 3 * rid;
      const real* R = d->cam_xmat + 9 * rid;
      real T[16] = {1, 0, 0, -cp[0], 0, 1, 0, -cp[1], 0, 0, 1, -cp[2], 0, 0, 0, 1};
      real Rot[16] = {R[0], R[3], R[6], 0, R[1], R[4], R[7], 0, R[2], R[5], R[8], 0, 0, 0, 0, 1};
      int rx = m->cam_resolution[2 * rid], ry = m->cam_resolution[2 * rid + 1];
      const real* ss = m->cam_sensorsize + 2 * rid;
      const real* in = m->cam_intrinsic + 4 * rid;
      real fx, fy;
      if (ss[0] != 0 && ss[1] != 0) {
        fx = in[0] / (ss[0] + MINVAL) * (real)rx;
        fy = in[1] / (ss[1] + MINVAL) * (real)ry;
      } else {
        fx = fy = 0.5 / tan(m->cam_fovy[rid] * (3.14159265358979323846 / 360.0)) * (real)ry;
      }
      real Fo[16] = {-fx, 0, 0, 0, 0, fy, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0};
      real Im[16] = {1, 0, 0.5 * rx, 0, 0, 1, 0.5 * ry, 0, 0, 0, 1, 0, 0, 0, 0, 0};
      real A[16], B[16], P[16];
      for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
          A[4 * i + j] = B[4 * i + j] = 0;
          for (int k = 0; k < 4; k++) A[4 * i + j] += Im[4 * i + k] * Fo[4 * k + j];
        }
      for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
          for (int k = 0; k < 4; k++) B[4 * i + j] += A[4 * i + k] * Rot[4 * k + j];
      for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
          P[4 * i + j] = 0;
          for (int k = 0; k < 4; k++) P[4 * i + j] += B[4 * i + k] * T[4 * k + j];
        }
      real ph[3];
      for (int i = 0; i < 3; i++) ph[i] = P[4 * i] * sp[0] + P[4 * i + 1] * sp[1] + P[4 * i + 2] * sp[2] + P[4 * i + 3];
      real den = ph[2];
      if (fabs(den) < MINVAL) den = clampr(den, -MINVAL, MINVAL);
      v[0] = ph[0] / den;
      v[1] = ph[1] / den;
      sensor_write(m, d, s, v, 2);
    } else if (t == SENS_SUBTREECOM) {
      memcpy(v, d->subtree_com + 3 * id, 3 * sizeof(real));
      sensor_write(m, d, s, v, 3);
    } else if (t == SENS_CLOCK) {
      v[0] = d->time[0];
      sensor_write(m, d, s, v, 1);
    }
  }
}

/* sensor.py:1011-1050 _cvel_offset */
static void cvel_offset(const orc_model* m, const orc_data* d, int type, int id, const real** cvel, real* off) {
  const real *p, *R; int b;
  obj_frame(m, d, type, id, &p, &R, &b);
  *cvel = d->cvel + 6 * b;
  const real* com = d->subtree_com + 3 * m->body_rootid[b];
  for (int i = 0; i < 3; i++) off[i] = p[i] - com[i];
}

/* sensor.py:1251-1373 (_sensor_vel, supported types) */
static void sensor_vel(const orc_model* m, orc_data* d) {
  sensor_extra(m, d, STAGE_VEL);
  for (int s = 0; s < m->nsensor; s++) {
    if (m->sensor_needstage[s] != STAGE_VEL) continue;
    int t = m->sensor_type[s], id = m->sensor_objid[s], ot = m->sensor_objtype[s];
    int rid = m->sensor_refid[s], rt = m->sensor_reftype[s];
    real v[3] = {0, 0, 0};
    if (t == SENS_VELOCIMETER || t == SENS_GYRO) {
      int b = m->site_bodyid[id];
      const real* cv = d->cvel + 6 * b;
      const real* R = d->site_xmat + 9 * id;
      if (t == SENS_GYRO) mat_t_vec(v, R, cv);
      else { /* sensor.py:909-931 */
        const real* com = d->subtree_com + 3 * m->body_rootid[b];
        real dif[3], c[3], lin[3];
        for (int i = 0; i < 3; i++) dif[i] = d->site_xpos[3 * id + i] - com[i];
        cross3(c, dif, cv);
        for (int i = 0; i < 3; i++) lin[i] = cv[3 + i] - c[i];
        mat_t_vec(v, R, lin);
      }
      sensor_write(m, d, s, v, 3);
    } else if (t == SENS_JOINTVEL) {
      v[0] = d->qvel[m->jnt_dofadr[id]];
      sensor_write(m, d, s, v, 1);
    } else if (t == SENS_ACTUATORVEL) {
      v[0] = d->actuator_velocity[id];
      sensor_write(m, d, s, v, 1);
    } else if (t == SENS_BALLANGVEL) {
      memcpy(v, d->qvel + m->jnt_dofadr[id], 3 * sizeof(real));
      sensor_write(m, d, s, v, 3);
    } else if (t == SENS_FRAMELINVEL) { /* sensor.py:1053-1156 */
      const real *p, *R, *pr, *Rr; int b, br;
      obj_frame(m, d, ot, id, &p, &R, &b);
      obj_frame(m, d, rt, rid, &pr, &Rr, &br);
      const real *cv, *cvr;
      real off[3], offr[3], c[3], xl[3];
      cvel_offset(m, d, ot, id, &cv, off);
      cvel_offset(m, d, rt, rid, &cvr, offr);
      cross3(c, off, cv);
      for (int i = 0; i < 3; i++) xl[i] = cv[3 + i] - c[i];
      if (rid > -1) {
        real cr[3], xlr[3], rvec[3], rc[3], rel[3];
        cross3(cr, offr, cvr);
        for (int i = 0; i < 3; i++) { xlr[i] = cvr[3 + i] - cr[i]; rvec[i] = p[i] - pr[i]; }
        cross3(rc, rvec, cvr);
        for (int i = 0; i < 3; i++) rel[i] = xl[i] - xlr[i] + rc[i];
        mat_t_vec(v, Rr, rel);
      } else memcpy(v, xl, sizeof(xl));
      sensor_write(m, d, s, v, 3);
    } else if (t == SENS_FRAMEANGVEL) { /* sensor.py:1159-1238 */
      const real *cv, *cvr;
      real off[3];
      cvel_offset(m, d, ot, id, &cv, off);
      if (rid > -1) {
        const real *pr, *Rr; int br;
        obj_frame(m, d, rt, rid, &pr, &Rr, &br);
        cvel_offset(m, d, rt, rid, &cvr, off);
        real dw[3] = {cv[0] - cvr[0], cv[1] - cvr[1], cv[2] - cvr[2]};
        mat_t_vec(v, Rr, dw);
      } else memcpy(v, cv, 3 * sizeof(real));
      sensor_write(m, d, s, v, 3);
    }
  }
}

/* support.py:241-308 contact force (pyramidal decode or the elliptic rows directly, to world frame) */
static void contact_force_world(const orc_model* m, const orc_data* d, int c, real* f6) {
  real f[6] = {0, 0, 0, 0, 0, 0};
  int condim = d->con_dim[c];
  int adr = d->con_efc_address[10 * c];
  if (adr >= 0) {
    if (m->opt_cone == CONE_ELLIPTIC) {
      for (int i = 0; i < condim; i++) {
        int a = d->con_efc_address[10 * c + i];
        if (a >= 0 && a < d->njmax) f[i] = d->efc_force[a];
      }
    } else if (condim == 1) f[0] = d->efc_force[adr];
    else {
      for (int i = 0; i < condim - 1; i++) {
        int a = 2 * i + adr;
        real d1 = a < d->njmax ? d->efc_force[a] : 0, d2 = a + 1 < d->njmax ? d->efc_force[a + 1] : 0;
        f[0] += d1 + d2;
        f[i + 1] = (d1 - d2) * d->con_friction[5 * c + i];
      }
    }
  }
  const real* F = d->con_frame + 9 * c;
  for (int i = 0; i < 3; i++) {
    f6[i] = f[0] * F[i] + f[1] * F[3 + i] + f[2] * F[6 + i];
    f6[3 + i] = f[3] * F[i] + f[4] * F[3 + i] + f[5] * F[6 + i];
  }
}

/* smooth.py:1276-1499 rne_postconstraint: cfrc_ext (xfrc_applied + contacts), cacc with qacc, cfrc_int */
static void rne_postconstraint(const orc_model* m, orc_data* d) {
  int nb = m->nbody;
  memset(d->cfrc_ext, 0, 6 * sizeof(real));
  for (int b = 1; b < nb; b++) { /* smooth.py:1278-1295 */
    const real* xf = d->xfrc_applied + 6 * b;
    const real* com = d->subtree_com + 3 * m->body_rootid[b];
    real off[3], c[3];
    for (int i = 0; i < 3; i++) off[i] = com[i] - d->xipos[3 * b + i];
    cross3(c, off, xf);
    for (int i = 0; i < 3; i++) { d->cfrc_ext[6 * b + i] = xf[3 + i] - c[i]; d->cfrc_ext[6 * b + 3 + i] = xf[i]; }
  }
  /* connect / weld forces, smooth.py:1296-1430 (rows lead the efc block: connects, then welds) */
  int ne = *d->ne < *d->nefc ? *d->ne : *d->nefc;
  if (ne > d->njmax) ne = d->njmax;
  for (int r = 0; r < ne;) {
    int id = d->efc_id[r], et = m->eq_type[id];
    if (et != EQ_CONNECT && et != EQ_WELD) break;
    int weld = et == EQ_WELD, body_sem = m->eq_objtype[id] == OBJ_BODY;
    real frc[3], trq[3] = {0, 0, 0};
    for (int i = 0; i < 3; i++) frc[i] = d->efc_force[r + i];
    if (weld)
      for (int i = 0; i < 3; i++) trq[i] = d->efc_force[r + 3 + i];
    int o[2] = {m->eq_obj1id[id], m->eq_obj2id[id]};
    const real* data = m->eq_data + 11 * id;
    for (int k = 0; k < 2; k++) {
      int b = body_sem ? o[k] : m->site_bodyid[o[k]];
      if (!b) continue;
      const real* off = body_sem ? data + (((k == 0) != weld) ? 0 : 3) : m->site_pos + 3 * o[k];
      real pos[3], dif[3], c[3];
      matvec3(pos, d->xmat + 9 * b, off);
      for (int i = 0; i < 3; i++) dif[i] = d->subtree_com[3 * m->body_rootid[b] + i] - (pos[i] + d->xpos[3 * b + i]);
      cross3(c, dif, frc);
      real sg = k == 0 ? 1 : -1;
      for (int i = 0; i < 3; i++) {
        d->cfrc_ext[6 * b + i] += sg * (trq[i] - c[i]);
        d->cfrc_ext[6 * b + 3 + i] += sg * frc[i];
      }
    }
    r += weld ? 6 : 3;
  }
  int ncon = *d->ncon < d->nconmax ? *d->ncon : d->nconmax;
  for (int c = 0; c < ncon; c++) { /* smooth.py:1447-1495 */
    int id1 = m->geom_bodyid[d->con_geom[2 * c]], id2 = m->geom_bodyid[d->con_geom[2 * c + 1]];
    if (id1 == 0 && id2 == 0) continue;
    real f6[6];
    contact_force_world(m, d, c, f6);
    const real* pos = d->con_pos + 3 * c;
    for (int k = 0; k < 2; k++) {
      int b = k == 0 ? id1 : id2;
      if (!b) continue;
      const real* com = d->subtree_com + 3 * m->body_rootid[b];
      real off[3], cr[3];
      for (int i = 0; i < 3; i++) off[i] = com[i] - pos[i];
      cross3(cr, off, f6);
      real sg = k == 0 ? -1 : 1;
      for (int i = 0; i < 3; i++) {
        d->cfrc_ext[6 * b + i] += sg * (f6[3 + i] - cr[i]);
        d->cfrc_ext[6 * b + 3 + i] += sg * f6[i];
      }
    }
  }
  real* cacc = d->cacc;
  memset(cacc, 0, 6 * sizeof(real));
  if (!(m->opt_disableflags & DSBL_GRAVITY))
    for (int i = 0; i < 3; i++) cacc[3 + i] = -m->opt_gravity[i];
  for (int b = 1; b < nb; b++) {
    int p = m->body_parentid[b];
    real acc[6];
    memcpy(acc, cacc + 6 * p, sizeof(acc));
    for (int k = 0; k < m->body_dofnum[b]; k++) {
      int dof = m->body_dofadr[b] + k;
      for (int i = 0; i < 6; i++) acc[i] += d->cdof_dot[6 * dof + i] * d->qvel[dof] + d->cdof[6 * dof + i] * d->qacc[dof];
    }
    memcpy(cacc + 6 * b, acc, sizeof(acc));
  }
  real* cfrc = d->cfrc_int;
  memset(cfrc, 0, 6 * sizeof(real));
  for (int b = 1; b < nb; b++) {
    real f1[6], iv[6], f2[6];
    inert_vec(f1, d->cinert + 10 * b, cacc + 6 * b);
    inert_vec(iv, d->cinert + 10 * b, d->cvel + 6 * b);
    motion_cross_force(f2, d->cvel + 6 * b, iv);
    for (int i = 0; i < 6; i++) cfrc[6 * b + i] = f1[i] + f2[i] - d->cfrc_ext[6 * b + i];
  }
  for (int b = nb - 1; b > 0; b--) {
    int p = m->body_parentid[b];
    for (int i = 0; i < 6; i++) cfrc[6 * p + i] += cfrc[6 * b + i];
  }
}

/* sensor.py:2447-2680 (_sensor_acc, supported types) */
static void sensor_acc(const orc_model* m, orc_data* d) {
  int post = 0;
  for (int s = 0; s < m->nsensor; s++) {
    int t = m->sensor_type[s];
    post |= t == SENS_ACCELEROMETER || t == SENS_FORCE || t == SENS_TORQUE || t == SENS_FRAMELINACC || t == SENS_FRAMEANGACC;
  }
  if (post) rne_postconstraint(m, d);
  sensor_extra(m, d, STAGE_ACC);
  for (int s = 0; s < m->nsensor; s++) {
    if (m->sensor_needstage[s] != STAGE_ACC) continue;
    int t = m->sensor_type[s], id = m->sensor_objid[s], ot = m->sensor_objtype[s];
    real v[3] = {0, 0, 0};
    if (t == SENS_ACCELEROMETER || t == SENS_FRAMELINACC) { /* sensor.py:1451-1480, 1619-1667 */
      const real *p, *R; int b;
      if (t == SENS_ACCELEROMETER) obj_frame(m, d, OBJ_SITE, id, &p, &R, &b);
      else obj_frame(m, d, ot, id, &p, &R, &b);
      const real* cv = d->cvel + 6 * b;
      const real* ca = d->cacc + 6 * b;
      const real* com = d->subtree_com + 3 * m->body_rootid[b];
      real dif[3], c1[3], c2[3], lin[3], acc[3], corr[3];
      for (int i = 0; i < 3; i++) dif[i] = p[i] - com[i];
      cross3(c1, dif, cv);
      cross3(c2, dif, ca);
      for (int i = 0; i < 3; i++) { lin[i] = cv[3 + i] - c1[i]; acc[i] = ca[3 + i] - c2[i]; }
      if (t == SENS_ACCELEROMETER) {
        real ang_l[3], lin_l[3], acc_l[3];
        mat_t_vec(ang_l, R, cv);
        mat_t_vec(lin_l, R, lin);
        mat_t_vec(acc_l, R, acc);
        cross3(corr, ang_l, lin_l);
        for (int i = 0; i < 3; i++) v[i] = acc_l[i] + corr[i];
      } else {
        cross3(corr, cv, lin);
        for (int i = 0; i < 3; i++) v[i] = acc[i] + corr[i];
      }
      sensor_write(m, d, s, v, 3);
    } else if (t == SENS_FORCE || t == SENS_TORQUE) { /* sensor.py:1483-1518 */
      int b = m->site_bodyid[id];
      const real* cf = d->cfrc_int + 6 * b;
      const real* R = d->site_xmat + 9 * id;
      if (t == SENS_FORCE) mat_t_vec(v, R, cf + 3);
      else {
        const real* com = d->subtree_com + 3 * m->body_rootid[b];
        real dif[3], c[3], tq[3];
        for (int i = 0; i < 3; i++) dif[i] = d->site_xpos[3 * id + i] - com[i];
        cross3(c, dif, cf + 3);
        for (int i = 0; i < 3; i++) tq[i] = cf[i] - c[i];
        mat_t_vec(v, R, tq);
      }
      sensor_write(m, d, s, v, 3);
    } else if (t == SENS_ACTUATORFRC) {
      v[0] = d->actuator_force[id];
      sensor_write(m, d, s, v, 1);
    } else if (t == SENS_JOINTACTFRC) {
      v[0] = d->qfrc_actuator[m->jnt_dofadr[id]];
      sensor_write(m, d, s, v, 1);
    } else if (t == SENS_FRAMEANGACC) { /* sensor.py:1670-1694 */
      const real *p, *R; int b;
      obj_frame(m, d, ot == OBJ_BODY ? OBJ_XBODY : ot, id, &p, &R, &b);
      memcpy(v, d->cacc + 6 * b, 3 * sizeof(real));
      sensor_write(m, d, s, v, 3);
    }
  }
}

/* forward.py:972-1000 */
static void forward_world(const orc_model* m, orc_data* d) {
  int sensors = m->nsensor > 0 && !(m->opt_disableflags & DSBL_SENSOR);
  fwd_position(m, d);
  if (m->nsensordata) memset(d->sensordata, 0, (size_t)m->nsensordata * sizeof(real));
  if (sensors) sensor_pos(m, d);
  fwd_velocity(m, d);
  if (sensors) sensor_vel(m, d);
  fwd_actuation(m, d);
  fwd_acceleration(m, d);
  solve(m, d);
  if (sensors) sensor_acc(m, d);
}

/* forward.py:51-109 _next_position: out = in (+) dt * scale * qvel (quaternions integrated) */
static void next_position(const orc_model* m, const real* qin, const real* qvel, real scale, real* qout) {
  real dt = m->opt_timestep;
  for (int j = 0; j < m->njnt; j++) {
    int qa = m->jnt_qposadr[j], da = m->jnt_dofadr[j], jt = m->jnt_type[j];
    real w[3], qn[4];
    if (jt == JNT_FREE) {
      for (int i = 0; i < 3; i++) qout[qa + i] = qin[qa + i] + dt * (qvel[da + i] * scale);
      for (int i = 0; i < 3; i++) w[i] = qvel[da + 3 + i] * scale;
      quat_integrate(qn, qin + qa + 3, w, dt);
      memcpy(qout + qa + 3, qn, sizeof(qn));
    } else if (jt == JNT_BALL) {
      for (int i = 0; i < 3; i++) w[i] = qvel[da + i] * scale;
      quat_integrate(qn, qin + qa, w, dt);
      memcpy(qout + qa, qn, sizeof(qn));
    } else {
      qout[qa] = qin[qa] + dt * qvel[da] * scale;
    }
  }
}

/* forward.py:457-491 rungekutta4 (tableau A = diag(1/2, 1/2, 1), B = (1/6, 1/3, 1/3, 1/6)) with
 * _rk_perturb_state :357-399, _rk_accumulate :402-454 and _advance :213-274; after forward_world */
static void rungekutta4(const orc_model* m, orc_data* d) {
  const real A[3] = {0.5, 0.5, 1.0}, B[4] = {1.0 / 6, 1.0 / 3, 1.0 / 3, 1.0 / 6};
  int nq = m->nq, nv = m->nv, na = m->na;
  real dt = m->opt_timestep;
  real* buf = (real*)malloc(((size_t)nq + 3 * nv + 2 * na + 1) * sizeof(real));
  real *qpos0 = buf, *qvel0 = qpos0 + nq, *qvel_rk = qvel0 + nv, *qacc_rk = qvel_rk + nv, *act0 = qacc_rk + nv, *act_dot_rk = act0 + na;
  memcpy(qpos0, d->qpos, nq * sizeof(real));
  memcpy(qvel0, d->qvel, nv * sizeof(real));
  memcpy(act0, d->act, na * sizeof(real));
  for (int i = 0; i < nv; i++) { qvel_rk[i] = B[0] * d->qvel[i]; qacc_rk[i] = B[0] * d->qacc[i]; }
  for (int i = 0; i < na; i++) act_dot_rk[i] = B[0] * d->act_dot[i];
  for (int k = 0; k < 3; k++) {
    next_position(m, qpos0, d->qvel, A[k], d->qpos);
    for (int i = 0; i < nv; i++) d->qvel[i] = qvel0[i] + A[k] * d->qacc[i] * dt;
    for (int a = 0; a < m->nu; a++) {
      int adr = m->actuator_actadr[a];
      for (int j = adr; adr >= 0 && j < adr + m->actuator_actnum[a]; j++) d->act[j] = next_act(m, a, act0[j], d->act_dot[j], A[k], 0);
    }
    forward_world(m, d);
    for (int i = 0; i < nv; i++) { qvel_rk[i] += B[k + 1] * d->qvel[i]; qacc_rk[i] += B[k + 1] * d->qacc[i]; }
    for (int i = 0; i < na; i++) act_dot_rk[i] += B[k + 1] * d->act_dot[i];
  }
  memcpy(d->act, act0, na * sizeof(real));
  memcpy(d->act_dot, act_dot_rk, na * sizeof(real));
  for (int a = 0; a < m->nu; a++) {
    int adr = m->actuator_actadr[a];
    for (int j = adr; adr >= 0 && j < adr + m->actuator_actnum[a]; j++) d->act[j] = next_act(m, a, d->act[j], d->act_dot[j], 1, m->actuator_actlimited[a]);
  }
  for (int i = 0; i < nv; i++) d->qvel[i] = qvel0[i] + qacc_rk[i] * dt;
  next_position(m, qpos0, qvel_rk, 1, d->qpos);
  d->time[0] += dt;
  memcpy(d->qacc_warmstart, d->qacc, nv * sizeof(real));
  free(buf);
}

/* forward.py:1003-1018 */
static void step_world(const orc_model* m, orc_data* d) {
  forward_world(m, d);
  if (m->opt_integrator == INTEGRATOR_RK4) rungekutta4(m, d);
  else integrate(m, d);
}

int orc_real_size(void) { return (int)sizeof(real); }

#define ORC_BATCH(fn, body)                                                                       \
  void fn(const orc_model* m, const orc_data* b, int nworld) {                                   \
    for (int w = 0; w < nworld; w++) { orc_data d; world_view(m, b, w, &d); body(m, &d); }      \
  }
ORC_BATCH(orc_fwd_position, fwd_position)
ORC_BATCH(orc_fwd_velocity, fwd_velocity)
ORC_BATCH(orc_fwd_actuation, fwd_actuation)
ORC_BATCH(orc_fwd_acceleration, fwd_acceleration)
ORC_BATCH(orc_solve, solve)
ORC_BATCH(orc_euler, integrate)

void orc_step(const orc_model* m, const orc_data* b, int nworld, int nthread) {
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthread > 0 ? nthread : 1)
#endif
  for (int w = 0; w < nworld; w++) {
    orc_data d;
    world_view(m, b, w, &d);
    step_world(m, &d);
  }
  (void)nthread;
}

void orc_forward(const orc_model* m, const orc_data* b, int nworld, int nthread) {
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthread > 0 ? nthread : 1)
#endif
  for (int w = 0; w < nworld; w++) {
    orc_data d;
    world_view(m, b, w, &d);
    forward_world(m, &d);
  }
  (void)nthread;
}

/* ---- known-answer entry points: the reference's own collision unit tests, restated as data ----------
 * (tests/golden/make_golden.py extracts their inputs and expected values; tests/test_golden.py runs them) */

/* collision_gjk_test.py:34-265 _geom_dist: ccd(tolerance, cutoff 1e30, iterations, iterations) of two geoms
 * carrying `margin`, then (multiccd) multicontact.  out = dist, x1[3], x2[3]; returns ncon, or -1 for a
 * multi-contact request this build does not restate (mesh polygons). */
/* collision_gjk_test.py:811-880 test_hfield_support: the support point of a heightfield prism
 * (6 x 3 vertices) with margin `margin` along dir */
int orc_kat_hfield_support(const real* prism, const real* dir, real margin, real* out) {
  ccd_geom g;
  memset(&g, 0, sizeof(g));
  g.type = GEOM_HFIELD;
  g.prism = prism;
  g.margin = margin;
  ccd_sp sp = ccd_support(&g, dir);
  memcpy(out, sp.point, 3 * sizeof(real));
  return sp.vertex_index;
}

int orc_kat_ccd(const int* type, const real* pos, const real* mat, const real* size, const real* mesh_vert, const int* vertadr,
                const int* vertnum, real margin, real tolerance, int iterations, int multiccd, real* out) {
  return orc_kat_ccd_model(type, pos, mat, size, mesh_vert, vertadr, vertnum, margin, tolerance, iterations, multiccd, NULL, NULL, out);
}

/* orc_kat_ccd with the meshes' polygon data from model `pm` (meshid[k]: the geom's mesh, -1 for none) */
int orc_kat_ccd_model(const int* type, const real* pos, const real* mat, const real* size, const real* mesh_vert, const int* vertadr,
                      const int* vertnum, real margin, real tolerance, int iterations, int multiccd, const orc_model* pm,
                      const int* meshid, real* out) {
  ccd_geom g[2], h1, h2;
  memset(g, 0, sizeof(g));
  for (int k = 0; k < 2; k++) {
    memcpy(g[k].pos, pos + 3 * k, 3 * sizeof(real));
    memcpy(g[k].rot, mat + 9 * k, 9 * sizeof(real));
    memcpy(g[k].size, size + 3 * k, 3 * sizeof(real));
    g[k].margin = margin;
    g[k].type = type[k];
    g[k].vert = type[k] == GEOM_MESH ? mesh_vert + 3 * vertadr[k] : NULL;
    g[k].nvert = type[k] == GEOM_MESH ? vertnum[k] : 0;
    if (pm && meshid && type[k] == GEOM_MESH) ccd_geom_mesh(pm, meshid[k], &g[k]);
  }
  polytope* pt = ccd_polytope();
  real d, x1[3], x2[3];
  int idx;
  int ncon = ccd_raw(&g[0], &g[1], tolerance, (real)1e30, iterations, iterations, pt, &d, x1, x2, &idx, &h1, &h2);
  if (multiccd && ((type[0] == GEOM_MESH && !g[0].pnormal) || (type[1] == GEOM_MESH && !g[1].pnormal))) return -1;
  if (multiccd && idx > -1) {
    real w1[4][3], w2[4][3];
    ncon = multicontact(pt, idx, x1, x2, &h1, &h2, w1, w2);
  }
  out[0] = d;
  for (int i = 0; i < 3; i++) { out[1 + i] = x1[i]; out[4 + i] = x2[i]; }
  return ncon;
}

/* collision_primitive_core_test.py: sphere_triangle (gt = SPHERE), box_triangle, capsule_triangle and
 * cylinder_triangle (collision_primitive_core.py:1518-1990); capsule / cylinder take their axis from column
 * 2 of `gr`.  out = 2 x (dist, pos[3], normal[3]); returns the number of candidates. */
/* util_misc.py:30-450 known-answer entry: fn 0 is_intersect(a[0:2], a[2:4], a[4:6], a[6:8]) -> out[0];
 * 1 length_circle(a[0:2], a[2:4], ind, radius) -> out[0]; 2 wrap_circle(end a[0:4], side a[4:6], radius);
 * 3 wrap_inside(end a[0:4], radius); 4 wrap(x0 a[0:3], x1 a[3:6], pos a[6:9], mat a[9:18], radius, ind = type,
 * side a[18:21]).  2-4 write (length, point0, point1) to out. */
int orc_kat_wrap(int fn, const real* a, int ind, real radius, real* out) {
  switch (fn) {
    case 0: out[0] = wrap_is_intersect(a, a + 2, a + 4, a + 6); return 0;
    case 1: out[0] = wrap_length_circle(a, a + 2, ind, radius); return 0;
    case 2: out[0] = wrap_circle(a, a + 4, radius, out + 1, out + 3); return 0;
    case 3: out[0] = wrap_inside(a, radius, out + 1, out + 3); return 0;
    case 4: out[0] = wrap_geom(a, a + 3, a + 6, a + 9, radius, ind, a + 18, out + 1, out + 4); return 0;
  }
  return -1;
}

int orc_kat_geom_triangle(int gt, const real* gp, const real* gr, const real* gs, const real* tri, real tr, real* out) {
  const real* t[3] = {tri, tri + 3, tri + 6};
  real ax[3] = {gr[2], gr[5], gr[8]};
  contacts2 c;
  c.n = 0;
  if (gt == GEOM_SPHERE) {
    real p[3], n[3];
    real dd = sphere_triangle(p, n, gp, gs[0], t[0], t[1], t[2], tr);
    put2(&c, dd, p, n);
  } else if (gt == GEOM_CAPSULE) {
    capsule_triangle(&c, gp, ax, gs[0], gs[1], t, tr);
  } else if (gt == GEOM_BOX) {
    box_triangle(&c, gp, gr, gs, t, tr);
  } else if (gt == GEOM_CYLINDER) {
    cylinder_triangle(&c, gp, ax, gs[0], gs[1], t, tr);
  } else {
    return -1;
  }
  for (int k = 0; k < 2; k++) {
    out[7 * k] = k < c.n ? c.dist[k] : MAXVAL;
    for (int i = 0; i < 3; i++) {
      out[7 * k + 1 + i] = k < c.n ? c.pos[k][i] : 0;
      out[7 * k + 4 + i] = k < c.n ? c.frame[k][i] : 0;
    }
  }
  return c.n;
}
