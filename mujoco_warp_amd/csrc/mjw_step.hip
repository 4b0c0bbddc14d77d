// mjw_step.hip -- world-per-wavefront batched MuJoCo step for MI355X (gfx950).
//
// One 64-lane wavefront owns one world for a whole stage group (or the whole
// step): lanes map to bodies / dofs / geom pairs / constraint rows, tree
// recursions run level by level inside the wave, per-world working state lives
// in LDS, and the CG/Newton convergence loop runs per world inside the kernel
// (no batch-wide solver tail, no graph conditionals).  Algorithms restate the
// reference pipeline mujoco_warp/_src/forward.py:1003-1018; each stage cites
// the reference file:line it follows.
//
// Global memory: Model fields are read-only (L2/scalar-cache resident); Data
// fields keep mujoco_warp's world-major shapes (nworld, ...), read once and
// written once per stage group with lane-contiguous (coalesced) accesses.

#include "mjw_common.h"
#include "mjw_ccd.h"
#include "mjw_narrow.h"
#include "mjw_passive.h"
#include "mjw_tendon.h"
#include "mjw_trn.h"
#include "mjw_dense.h"

#include <algorithm>
#include <cstdlib>

namespace mjw {

// words per elliptic contact of the generic solver's line-search coefficients (Ell, mjw_dense.h)
constexpr int EC_WORDS = 10;

// per-world LDS layout (offsets in 4-byte words)
struct Lay {
  int qpos, qvel, xpos, xquat, xmat, xipos, ximat, xanchor, xaxis, gxpos, gxmat;
  int subtree_com, cinert, crb, cdof, cdof_dot, cvel, cacc, cfrc;
  int qM, L, H, nvs;
  int qfrc_smooth, qacc_smooth, qacc, Ma, qfrc_constraint, qfrc_bias, qfrc_passive, qfrc_actuator, vec;
  int J, efc_D, efc_aref, efc_pos, efc_margin, efc_vel, efc_frictionloss, efc_type, efc_id, efc_force, efc_state;
  int Jaref, jv, rowcon;
  int act_len, act_vel, act_force, act_mom, act_momdof, act_nnz, amax;
  int con, cmax, jqvel, plist, scratch, iscratch, ccd;
  int ecoef, econe;  // generic solver, elliptic cones: per-contact line-search coefficients, Newton cone blocks
  int nofactor;
  int total;
};

// nofactor: the kernel stops at qfrc_smooth and the dense kernel does factor/solve/euler,
// so the Cholesky / Newton / solver row scratch is not allocated
__host__ inline Lay make_layout(const mjw_model_t& m, int njmax, bool nofactor = false, bool ccd = false) {
  Lay L;
  int o = 0;
  L.nofactor = nofactor;
  auto take = [&](int n) { int r = o; o += (n + 3) & ~3; return r; };
  auto r4 = [](int n) { return (n + 3) & ~3; };
  int usz = 0;  // size of the direct-mode region U
  int nv = m.nv, nb = m.nbody, nj = m.njnt, ng = m.ngeom, nu = m.nu;
  L.nvs = nv | 1;  // odd row stride: conflict-free row and column access
  L.qpos = take(m.nq); L.qvel = take(nv);
  L.xpos = take(nb * 3); L.xquat = take(nb * 4); L.xmat = take(nb * 9); L.xipos = take(nb * 3);
  L.xanchor = take(nj * 3); L.xaxis = take(nj * 3); L.gxpos = take(ng * 3); L.gxmat = take(ng * 9);
  L.subtree_com = take(nb * 3); L.cinert = take(nb * 10); L.crb = take(nb * 10); L.cdof = take(nv * 6);
  L.cmax = nofactor ? CMAX / 2 : CMAX;
  if (nofactor) {
    // direct mode (the dense path's forward kernel): constraint rows go straight to global memory
    // (the dense kernel reads them from there) and factor / solve / integrate run elsewhere, so the
    // world's LDS holds one region U whose contents follow the stage lifetimes:
    //   kinematics .. com_pos : ximat
    //   crb_qM                : qM (copied out to global)
    //   collision             : contact staging, broadphase survivors, J.qvel per row
    //   velocity .. accel.    : cdof_dot, cvel, cacc, cfrc, passive scratch (vec)
    const int u_pos = r4(nb * 9);
    const int u_qM = r4(nv * L.nvs);
    const int u_col = r4(L.cmax * CREC) + r4(m.nxn) + r4(njmax);
    const int u_vel = r4(nv * 6) + 3 * r4(nb * 6) + r4(2 * nv);
    usz = std::max(std::max(u_pos, u_qM), std::max(u_col, u_vel));
    const int U = take(usz);
    L.ximat = U;
    L.qM = L.L = L.H = U;
    L.con = U; L.plist = U + r4(L.cmax * CREC); L.jqvel = L.plist + r4(m.nxn);
    L.cdof_dot = U; L.cvel = U + r4(nv * 6); L.cacc = L.cvel + r4(nb * 6); L.cfrc = L.cacc + r4(nb * 6); L.vec = L.cfrc + r4(nb * 6);
    L.qfrc_smooth = take(nv); L.qfrc_bias = take(nv); L.qfrc_passive = take(nv); L.qfrc_actuator = take(nv);
    L.qacc_smooth = L.qacc = L.Ma = L.qfrc_constraint = -1;  // produced by the dense kernel
    L.J = L.efc_D = L.efc_aref = L.efc_pos = L.efc_margin = L.efc_vel = L.efc_frictionloss = L.efc_type = L.efc_id = -1;
    L.efc_force = L.efc_state = L.Jaref = L.jv = -1;
  } else {
    L.ximat = take(nb * 9);
    L.cdof_dot = take(nv * 6); L.cvel = take(nb * 6); L.cacc = take(nb * 6); L.cfrc = take(nb * 6);
    L.qM = take(nv * L.nvs);
    L.L = take(nv * L.nvs);
    L.H = (m.opt_solver == SOLVER_NEWTON) ? take(nv * L.nvs) : L.L;
    L.qfrc_smooth = take(nv); L.qacc_smooth = take(nv); L.qacc = take(nv); L.Ma = take(nv); L.qfrc_constraint = take(nv);
    L.qfrc_bias = take(nv); L.qfrc_passive = take(nv); L.qfrc_actuator = take(nv); L.vec = take(2 * nv);
    L.J = take(njmax * L.nvs);
    L.efc_D = take(njmax); L.efc_aref = take(njmax); L.efc_pos = take(njmax); L.efc_margin = take(njmax);
    L.efc_vel = take(njmax); L.efc_frictionloss = take(njmax); L.efc_type = take(njmax); L.efc_id = take(njmax);
    L.efc_force = take(njmax); L.efc_state = take(njmax); L.Jaref = take(njmax); L.jv = take(njmax);
    L.jqvel = take(njmax);
    L.plist = take(m.nxn);
    L.con = take(L.cmax * CREC);
  }
  // elliptic cones in the generic solver (solve below): the rows' unused efc_pos / efc_margin / efc_vel
  // slots hold each row's cone coefficient, contact extent and u = Jaref * coefficient; ecoef the
  // quad / quad1 / quad2 words of a contact's line search at its first row; econe the 6 cone-Hessian
  // coefficients of a row (Newton)
  const bool ell_generic = !nofactor && m.opt_cone == CONE_ELLIPTIC;
  L.ecoef = ell_generic ? take(EC_WORDS * njmax) : -1;
  L.econe = (ell_generic && m.opt_solver == SOLVER_NEWTON) ? take(6 * njmax) : -1;
  L.rowcon = -1;
  // moment slots per actuator: 1 when every transmission has one non-zero (nJmom == nu: hinge / slide
  // joints), else 6 (free / ball joints)
  L.amax = m.nJmom == nu ? 1 : (m.act_maxnnz > 6 ? m.act_maxnnz : 6);
  L.act_len = take(nu); L.act_vel = take(nu); L.act_force = take(nu); L.act_mom = take(nu * L.amax); L.act_momdof = take(nu * L.amax);
  L.act_nnz = take(nu);
  L.scratch = take(64);
  L.iscratch = take(64);
  // convex-collision (GJK/EPA) workspace of the pre-pass kernel, which runs kinematics only: in
  // direct mode the region U (ximat is dead there), else the cdof_dot..cfrc block when it fits;
  // otherwise the workspace gets its own LDS
  L.ccd = -1;
  if (ccd && m.nxn_ccd > 0) {
    const int need = ccd_layout(m.ccd_epa_iterations, m.nhfield > 0, m.nmaxpolygon, m.nmaxmeshdeg).total;
    if (nofactor) L.ccd = (usz >= need) ? L.ximat : take(need);
    else L.ccd = (L.qM - L.cdof_dot >= need) ? L.cdof_dot : take(need);
  }
  L.total = o;
  return L;
}

// -------------------------------------------------------------------------------------------
// wave-level collectives
// -------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) { return dsum(v); }

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// inclusive prefix sum of small non-negative ints across the wave
__device__ __forceinline__ int wave_scan_incl(int v) {
  int lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    int t = __shfl_up(v, off, 64);
    if (lane >= off) v += t;
  }
  return v;
}

#define WSYNC() __syncthreads()

struct WS {
  float* s;  // LDS base of this world
  int* si;   // same, as ints
  int wid;   // world index within the launch
  int lane;
};

// -------------------------------------------------------------------------------------------
// smooth.py: kinematics (smooth.py:44-224, 357-415)
// -------------------------------------------------------------------------------------------
__device__ __forceinline__ void kinematics(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, WS& w) {
  const int wid = w.wid, lane = w.lane;
  float* s = w.s;
  const float* qpos = s + L.qpos;
  const float* body_pos = MR(body_pos);
  const float* body_quat = MR(body_quat);
  const float* jnt_pos = MR(jnt_pos);
  const float* jnt_axis = MR(jnt_axis);
  const float* qpos0 = MR(qpos0);
  float* xpos = s + L.xpos;
  float* xquat = s + L.xquat;
  float* xanc = s + L.xanchor;
  float* xax = s + L.xaxis;
  if (lane == 0) {
    xpos[0] = xpos[1] = xpos[2] = 0.0f;
    xquat[0] = 1.0f; xquat[1] = xquat[2] = xquat[3] = 0.0f;
  }
  // Pass 1 (all bodies in parallel): the body pose relative to its parent frame after its
  // joints, and each joint's anchor / axis in the parent frame.  smooth.py:44-144 composes the
  // same chain in world frame level by level; world = parent o local is the same product.
  // Pass 2 (level by level, LDS only): world pose = parent world pose o local pose.
  for (int b0 = 0; b0 < m.nbody; b0 += LPW) {
    const int b = b0 + lane;
    const bool ok = b > 0 && b < m.nbody;
    int par = 0, lv = 0;
    bool absolute = false;
    float lp[3] = {0.0f, 0.0f, 0.0f}, lq[4] = {1.0f, 0.0f, 0.0f, 0.0f};
    if (ok) {
      par = m.body_parentid[b];
      lv = m.body_level[b];
      const int jntadr = m.body_jntadr[b], jntnum = m.body_jntnum[b];
      if (jntnum == 1 && m.jnt_type[jntadr] == JNT_FREE) {
        // free joints live in top-level bodies: the pose is qpos itself (world frame)
        absolute = true;
        int qa = m.jnt_qposadr[jntadr];
        for (int i = 0; i < 4; i++) lq[i] = qpos[qa + 3 + i];
        normalize4(lq);
        for (int i = 0; i < 3; i++) {
          lp[i] = qpos[qa + i];
          xanc[3 * jntadr + i] = qpos[qa + i];
          xax[3 * jntadr + i] = jnt_axis[3 * jntadr + i];
        }
      } else {
        int mocapid = m.body_mocapid[b];
        if (mocapid >= 0) {
          for (int i = 0; i < 3; i++) lp[i] = d.mocap_pos[(long)wid * m.nmocap * 3 + 3 * mocapid + i];
          for (int i = 0; i < 4; i++) lq[i] = d.mocap_quat[(long)wid * m.nmocap * 4 + 4 * mocapid + i];
        } else {
          for (int i = 0; i < 3; i++) lp[i] = body_pos[3 * b + i];
          for (int i = 0; i < 4; i++) lq[i] = body_quat[4 * b + i];
        }
        for (int k = 0; k < jntnum; k++) {
          const int j = jntadr + k;
          const int qa = m.jnt_qposadr[j], jt = m.jnt_type[j];
          const float* ax = jnt_axis + 3 * j;
          const float* jp = jnt_pos + 3 * j;
          float anc[3], axis[3], t[3];
          rot_vec_quat(t, jp, lq);
          for (int i = 0; i < 3; i++) anc[i] = t[i] + lp[i];
          rot_vec_quat(axis, ax, lq);
          if (jt == JNT_BALL) {
            float ql[4] = {qpos[qa], qpos[qa + 1], qpos[qa + 2], qpos[qa + 3]};
            normalize4(ql);
            mul_quat(lq, lq, ql);
            rot_vec_quat(t, jp, lq);
            for (int i = 0; i < 3; i++) lp[i] = anc[i] - t[i];
          } else if (jt == JNT_SLIDE) {
            float dq = qpos[qa] - qpos0[qa];
            for (int i = 0; i < 3; i++) lp[i] += axis[i] * dq;
          } else if (jt == JNT_HINGE) {
            float ql[4];
            axis_angle_to_quat(ql, ax, qpos[qa] - qpos0[qa]);
            mul_quat(lq, lq, ql);
            rot_vec_quat(t, jp, lq);
            for (int i = 0; i < 3; i++) lp[i] = anc[i] - t[i];
          }
          for (int i = 0; i < 3; i++) {
            xanc[3 * j + i] = anc[i];
            xax[3 * j + i] = axis[i];
          }
        }
      }
    }
    for (int lvl = 1; lvl < m.nlevel; lvl++) {
      if (ok && lv == lvl) {
        float q[4], t[3];
        if (absolute) {
          for (int i = 0; i < 4; i++) q[i] = lq[i];
          for (int i = 0; i < 3; i++) t[i] = lp[i];
        } else {
          float pq[4] = {xquat[4 * par], xquat[4 * par + 1], xquat[4 * par + 2], xquat[4 * par + 3]};
          rot_vec_quat(t, lp, pq);
          for (int i = 0; i < 3; i++) t[i] += xpos[3 * par + i];
          mul_quat(q, pq, lq);
          normalize4(q);
        }
        for (int i = 0; i < 3; i++) xpos[3 * b + i] = t[i];
        for (int i = 0; i < 4; i++) xquat[4 * b + i] = q[i];
      }
      WSYNC();
    }
  }
  // joint anchors / axes to world frame (free joints are already there)
  for (int j = lane; j < m.njnt; j += LPW) {
    long gj = (long)wid * m.njnt + j;
    float anc[3], axis[3];
    for (int i = 0; i < 3; i++) { anc[i] = xanc[3 * j + i]; axis[i] = xax[3 * j + i]; }
    if (m.jnt_type[j] != JNT_FREE) {
      int p = m.body_parentid[m.jnt_bodyid[j]];
      float pq[4] = {xquat[4 * p], xquat[4 * p + 1], xquat[4 * p + 2], xquat[4 * p + 3]}, t[3];
      rot_vec_quat(t, anc, pq);
      for (int i = 0; i < 3; i++) anc[i] = t[i] + xpos[3 * p + i];
      rot_vec_quat(t, axis, pq);
      for (int i = 0; i < 3; i++) axis[i] = t[i];
    }
    for (int i = 0; i < 3; i++) {
      xanc[3 * j + i] = anc[i];
      xax[3 * j + i] = axis[i];
      d.xanchor[gj * 3 + i] = anc[i];
      d.xaxis[gj * 3 + i] = axis[i];
    }
  }
  // body matrices / inertial frames (smooth.py:146-173)
  const float* body_ipos = MR(body_ipos);
  const float* body_iquat = MR(body_iquat);
  for (int b = lane; b < m.nbody; b += LPW) {
    float q[4] = {xquat[4 * b], xquat[4 * b + 1], xquat[4 * b + 2], xquat[4 * b + 3]};
    float mat[9], t[3], qi[4], imat[9];
    quat_to_mat(mat, q);
    rot_vec_quat(t, body_ipos + 3 * b, q);
    float xi[3] = {xpos[3 * b] + t[0], xpos[3 * b + 1] + t[1], xpos[3 * b + 2] + t[2]};
    mul_quat(qi, q, body_iquat + 4 * b);
    quat_to_mat(imat, qi);
    for (int i = 0; i < 9; i++) { s[L.xmat + 9 * b + i] = mat[i]; s[L.ximat + 9 * b + i] = imat[i]; }
    for (int i = 0; i < 3; i++) s[L.xipos + 3 * b + i] = xi[i];
    long gb = (long)wid * m.nbody;
    for (int i = 0; i < 3; i++) { d.xpos[(gb + b) * 3 + i] = xpos[3 * b + i]; d.xipos[(gb + b) * 3 + i] = xi[i]; }
    for (int i = 0; i < 4; i++) d.xquat[(gb + b) * 4 + i] = q[i];
    for (int i = 0; i < 9; i++) { d.xmat[(gb + b) * 9 + i] = mat[i]; d.ximat[(gb + b) * 9 + i] = imat[i]; }
  }
  // geoms (smooth.py:176-203) -- static world geoms evaluate to the same pose
  const float* geom_pos = MR(geom_pos);
  const float* geom_quat = MR(geom_quat);
  for (int g = lane; g < m.ngeom; g += LPW) {
    int b = m.geom_bodyid[g];
    float q[4] = {xquat[4 * b], xquat[4 * b + 1], xquat[4 * b + 2], xquat[4 * b + 3]};
    float t[3], gq[4], gm[9];
    rot_vec_quat(t, geom_pos + 3 * g, q);
    mul_quat(gq, q, geom_quat + 4 * g);
    quat_to_mat(gm, gq);
    long gg = (long)wid * m.ngeom + g;
    for (int i = 0; i < 3; i++) {
      float v = xpos[3 * b + i] + t[i];
      s[L.gxpos + 3 * g + i] = v;
      d.geom_xpos[gg * 3 + i] = v;
    }
    for (int i = 0; i < 9; i++) { s[L.gxmat + 9 * g + i] = gm[i]; d.geom_xmat[gg * 9 + i] = gm[i]; }
  }
  const float* site_pos = MR(site_pos);
  const float* site_quat = MR(site_quat);
  for (int si = lane; si < m.nsite; si += LPW) {
    int b = m.site_bodyid[si];
    float q[4] = {xquat[4 * b], xquat[4 * b + 1], xquat[4 * b + 2], xquat[4 * b + 3]};
    float t[3], sq[4], sm[9];
    rot_vec_quat(t, site_pos + 3 * si, q);
    mul_quat(sq, q, site_quat + 4 * si);
    quat_to_mat(sm, sq);
    long gs = (long)wid * m.nsite + si;
    for (int i = 0; i < 3; i++) d.site_xpos[gs * 3 + i] = xpos[3 * b + i] + t[i];
    for (int i = 0; i < 9; i++) d.site_xmat[gs * 9 + i] = sm[i];
  }
  WSYNC();
}

// smooth.py:463-632: subtree com (contiguous DFS subtree ranges), cinert, cdof
__device__ __forceinline__ void com_pos(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, WS& w) {
  const int wid = w.wid, lane = w.lane;
  float* s = w.s;
  const float* body_mass = MR(body_mass);
  const float* body_subtreemass = MR(body_subtreemass);
  const float* body_inertia = MR(body_inertia);
  // body masses in the (still unused) crb slots, so that the subtree sums below read LDS only
  // instead of one dependent global load of body_mass per subtree body
  float* bm = s + L.crb;
  for (int b = lane; b < m.nbody; b += LPW) bm[b] = body_mass[b];
  WSYNC();
  for (int b = lane; b < m.nbody; b += LPW) {
    float acc[3] = {0.0f, 0.0f, 0.0f};
    int end = m.body_subtree_end[b];
    for (int j = b; j < end; j++) {
      const float ms = bm[j];
      for (int i = 0; i < 3; i++) acc[i] += s[L.xipos + 3 * j + i] * ms;
    }
    float mass = body_subtreemass[b];
    if (mass != 0.0f)
      for (int i = 0; i < 3; i++) acc[i] /= mass;
    long gb = (long)wid * m.nbody + b;
    for (int i = 0; i < 3; i++) { s[L.subtree_com + 3 * b + i] = acc[i]; d.subtree_com[gb * 3 + i] = acc[i]; }
  }
  WSYNC();
  for (int b = lane; b < m.nbody; b += LPW) {
    const float* mat = s + L.ximat + 9 * b;
    const float* inert = body_inertia + 3 * b;
    float mass = body_mass[b];
    int root = m.body_rootid[b];
    float dif[3];
    for (int i = 0; i < 3; i++) dif[i] = s[L.xipos + 3 * b + i] - s[L.subtree_com + 3 * root + i];
    float tmp[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++)
        tmp[3 * i + j] = mat[3 * i] * inert[0] * mat[3 * j] + mat[3 * i + 1] * inert[1] * mat[3 * j + 1] +
                         mat[3 * i + 2] * inert[2] * mat[3 * j + 2];
    float res[10];
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
    long gb = (long)wid * m.nbody + b;
    for (int i = 0; i < 10; i++) { s[L.cinert + 10 * b + i] = res[i]; d.cinert[gb * 10 + i] = res[i]; }
  }
  for (int i = lane; i < m.nv; i += LPW) {
    int j = m.dof_jntid[i];
    int b = m.jnt_bodyid[j], jt = m.jnt_type[j], k = i - m.jnt_dofadr[j];
    int root = m.body_rootid[b];
    float off[3], r[6];
    for (int a = 0; a < 3; a++) off[a] = s[L.subtree_com + 3 * root + a] - s[L.xanchor + 3 * j + a];
    if ((jt == JNT_FREE && k >= 3) || jt == JNT_BALL) {
      int c = jt == JNT_FREE ? k - 3 : k;
      float ax[3] = {s[L.xmat + 9 * b + c], s[L.xmat + 9 * b + 3 + c], s[L.xmat + 9 * b + 6 + c]};
      r[0] = ax[0]; r[1] = ax[1]; r[2] = ax[2];
      cross3(r + 3, ax, off);
    } else if (jt == JNT_FREE) {
      r[0] = r[1] = r[2] = 0.0f;
      r[3] = k == 0 ? 1.0f : 0.0f; r[4] = k == 1 ? 1.0f : 0.0f; r[5] = k == 2 ? 1.0f : 0.0f;
    } else if (jt == JNT_SLIDE) {
      r[0] = r[1] = r[2] = 0.0f;
      for (int a = 0; a < 3; a++) r[3 + a] = s[L.xaxis + 3 * j + a];
    } else {
      float ax[3] = {s[L.xaxis + 3 * j], s[L.xaxis + 3 * j + 1], s[L.xaxis + 3 * j + 2]};
      r[0] = ax[0]; r[1] = ax[1]; r[2] = ax[2];
      cross3(r + 3, ax, off);
    }
    long gd = (long)wid * m.nv + i;
    for (int a = 0; a < 6; a++) { s[L.cdof + 6 * i + a] = r[a]; d.cdof[gd * 6 + a] = r[a]; }
  }
  WSYNC();
}

// smooth.py:635-803
__device__ __forceinline__ void camlight(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, WS& w) {
  const int wid = w.wid, lane = w.lane;
  const float* s = w.s;
  const float* cam_pos = MR(cam_pos);
  const float* cam_quat = MR(cam_quat);
  const float* cam_pos0 = MR(cam_pos0);
  const float* cam_poscom0 = MR(cam_poscom0);
  const float* cam_mat0 = MR(cam_mat0);
  for (int c = lane; c < m.ncam; c += LPW) {
    int mode = m.cam_mode[c], b = m.cam_bodyid[c], tgt = m.cam_targetbodyid[c];
    bool is_target = mode == CAM_TARGETBODY || mode == CAM_TARGETBODYCOM;
    float cx[3], cm[9];
    const float* xq = s + L.xquat + 4 * b;
    const float* xp = s + L.xpos + 3 * b;
    if ((is_target && tgt < 0) || mode == CAM_FIXED) {
      float t[3], q[4];
      rot_vec_quat(t, cam_pos + 3 * c, xq);
      for (int i = 0; i < 3; i++) cx[i] = xp[i] + t[i];
      mul_quat(q, xq, cam_quat + 4 * c);
      quat_to_mat(cm, q);
    } else if (mode == CAM_TRACK) {
      for (int i = 0; i < 9; i++) cm[i] = cam_mat0[9 * c + i];
      for (int i = 0; i < 3; i++) cx[i] = xp[i] + cam_pos0[3 * c + i];
    } else if (mode == CAM_TRACKCOM) {
      for (int i = 0; i < 9; i++) cm[i] = cam_mat0[9 * c + i];
      for (int i = 0; i < 3; i++) cx[i] = s[L.subtree_com + 3 * b + i] + cam_poscom0[3 * c + i];
    } else {
      float t[3], m1[3], m2[3], m3[3];
      rot_vec_quat(t, cam_pos + 3 * c, xq);
      for (int i = 0; i < 3; i++) cx[i] = xp[i] + t[i];
      const float* tp = mode == CAM_TARGETBODYCOM ? s + L.subtree_com + 3 * tgt : s + L.xpos + 3 * tgt;
      for (int i = 0; i < 3; i++) m3[i] = cx[i] - tp[i];
      normalize3(m3);
      float z[3] = {0.0f, 0.0f, 1.0f};
      cross3(m1, z, m3);
      normalize3(m1);
      cross3(m2, m3, m1);
      normalize3(m2);
      for (int i = 0; i < 3; i++) { cm[3 * i] = m1[i]; cm[3 * i + 1] = m2[i]; cm[3 * i + 2] = m3[i]; }
    }
    long gc = (long)wid * m.ncam + c;
    for (int i = 0; i < 3; i++) d.cam_xpos[gc * 3 + i] = cx[i];
    for (int i = 0; i < 9; i++) d.cam_xmat[gc * 9 + i] = cm[i];
  }
  const float* light_pos = MR(light_pos);
  const float* light_dir = MR(light_dir);
  const float* light_pos0 = MR(light_pos0);
  const float* light_poscom0 = MR(light_poscom0);
  const float* light_dir0 = MR(light_dir0);
  for (int l = lane; l < m.nlight; l += LPW) {
    int mode = m.light_mode[l], b = m.light_bodyid[l], tgt = m.light_targetbodyid[l];
    bool is_target = mode == CAM_TARGETBODY || mode == CAM_TARGETBODYCOM;
    float lx[3], ld[3];
    const float* xq = s + L.xquat + 4 * b;
    const float* xp = s + L.xpos + 3 * b;
    bool norm = true;
    if ((is_target && tgt < 0) || mode == CAM_FIXED) {
      float t[3];
      rot_vec_quat(t, light_pos + 3 * l, xq);
      for (int i = 0; i < 3; i++) lx[i] = xp[i] + t[i];
      rot_vec_quat(ld, light_dir + 3 * l, xq);
      norm = !(is_target && tgt < 0);  // smooth.py:732 returns before normalize
    } else if (mode == CAM_TRACK) {
      for (int i = 0; i < 3; i++) { ld[i] = light_dir0[3 * l + i]; lx[i] = xp[i] + light_pos0[3 * l + i]; }
    } else if (mode == CAM_TRACKCOM) {
      for (int i = 0; i < 3; i++) { ld[i] = light_dir0[3 * l + i]; lx[i] = s[L.subtree_com + 3 * b + i] + light_poscom0[3 * l + i]; }
    } else {
      float t[3];
      rot_vec_quat(t, light_pos + 3 * l, xq);
      for (int i = 0; i < 3; i++) lx[i] = xp[i] + t[i];
      const float* tp = mode == CAM_TARGETBODYCOM ? s + L.subtree_com + 3 * tgt : s + L.xpos + 3 * tgt;
      for (int i = 0; i < 3; i++) ld[i] = tp[i] - lx[i];
    }
    if (norm) normalize3(ld);
    long gl = (long)wid * m.nlight + l;
    for (int i = 0; i < 3; i++) { d.light_xpos[gl * 3 + i] = lx[i]; d.light_xdir[gl * 3 + i] = ld[i]; }
  }
}

// smooth.py:806-912: composite inertia (subtree ranges) and dense qM
template <bool TEN>
__device__ __forceinline__ void crb_qM(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, WS& w) {
  const int wid = w.wid, lane = w.lane;
  float* s = w.s;
  const float* dof_armature = MR(dof_armature);
  for (int b = lane; b < m.nbody; b += LPW) {
    float acc[10];
    for (int i = 0; i < 10; i++) acc[i] = s[L.cinert + 10 * b + i];
    if (b > 0) {
      int end = m.body_subtree_end[b];
      for (int j = b + 1; j < end; j++)
        for (int i = 0; i < 10; i++) acc[i] += s[L.cinert + 10 * j + i];
    }
    long gb = (long)wid * m.nbody + b;
    for (int i = 0; i < 10; i++) { s[L.crb + 10 * b + i] = acc[i]; d.crb[gb * 10 + i] = acc[i]; }
  }
  const int nv = m.nv, nvs = L.nvs;
  float* M = s + L.qM;
  for (int e = lane; e < nv * nvs; e += LPW) M[e] = 0.0f;
  // dof parents in LDS (iscratch is free until the collision stage): the ancestor walks below
  // then chain LDS reads instead of dependent global loads
  int* dpar = w.si + L.iscratch;
  const bool dpar_lds = nv <= 64;
  if (dpar_lds)
    for (int i = lane; i < nv; i += LPW) dpar[i] = m.dof_parentid[i];
  WSYNC();
  for (int i = lane; i < nv; i += LPW) {
    int b = m.dof_bodyid[i];
    float buf[6], cd[6];
    for (int a = 0; a < 6; a++) cd[a] = s[L.cdof + 6 * i + a];
    inert_vec(buf, s + L.crb + 10 * b, cd);
    float Mii = dof_armature[i];
    Mii += cd[0] * buf[0] + cd[1] * buf[1] + cd[2] * buf[2] + cd[3] * buf[3] + cd[4] * buf[4] + cd[5] * buf[5];
    M[i * nvs + i] = Mii;
    int j = dpar_lds ? dpar[i] : m.dof_parentid[i];
    while (j >= 0) {
      const float* cj = s + L.cdof + 6 * j;
      float q = cj[0] * buf[0] + cj[1] * buf[1] + cj[2] * buf[2] + cj[3] * buf[3] + cj[4] * buf[4] + cj[5] * buf[5];
      M[i * nvs + j] = q;
      M[j * nvs + i] = q;
      j = dpar_lds ? dpar[j] : m.dof_parentid[j];
    }
  }
  WSYNC();
  if (TEN && m.ntendon) tendon_armature(m, d, M, nvs, wid, lane);  // smooth.py:916-1000
  const int np = m.nv_pad;
  float* gM = d.qM + (long)wid * np * np;
  for (int e = lane; e < np * np; e += LPW) {
    int r = e / np, c = e - r * np;
    gM[e] = (r < nv && c < nv) ? M[r * nvs + c] : 0.0f;
  }
}

// -------------------------------------------------------------------------------------------
// dense Cholesky (wp.tile_cholesky) and solve (wp.tile_cholesky_solve), lane = row
// -------------------------------------------------------------------------------------------
__device__ __forceinline__ void cholesky(float* A, int n, int nvs, int lane) {
  // in place: lower triangle of A becomes L (A = L L^T), upper set to zero
  for (int j = 0; j < n; j++) {
    float ljj = sqrtf(A[j * nvs + j]);
    float inv = 1.0f / ljj;
    WSYNC();
    if (lane < n) {
      if (lane > j) A[lane * nvs + j] *= inv;
      else if (lane == j) A[j * nvs + j] = ljj;
    }
    WSYNC();
    if (lane > j && lane < n) {
      float lij = A[lane * nvs + j];
      for (int k = j + 1; k <= lane; k++) A[lane * nvs + k] -= lij * A[k * nvs + j];
    }
    WSYNC();
  }
  for (int e = lane; e < n * nvs; e += LPW) {
    int r = e / nvs, c = e - r * nvs;
    if (c > r) A[e] = 0.0f;
  }
  WSYNC();
}

// x = (L L^T)^-1 y ; y held per lane (lane = dof), result per lane
__device__ __forceinline__ float cholesky_solve(const float* Lm, int n, int nvs, int lane, float y) {
  for (int j = 0; j < n; j++) {
    float yj = __shfl(y, j, 64) / Lm[j * nvs + j];
    if (lane == j) y = yj;
    else if (lane > j && lane < n) y -= Lm[lane * nvs + j] * yj;
  }
  for (int k = n - 1; k >= 0; k--) {
    float xk = __shfl(y, k, 64) / Lm[k * nvs + k];
    if (lane == k) y = xk;
    else if (lane < k) y -= Lm[k * nvs + lane] * xk;
  }
  return lane < n ? y : 0.0f;
}
// collision primitives, AABB/OBB filters and contact_params: mjw_narrow.h

// collision_driver.py:274-321; gxpos / gxmat: the world's geom frames (LDS in the fused kernels, HBM in the
// stand-alone broadphase entry point)
__device__ __forceinline__ bool broadphase_filter_g(const mjw_model_t& m, const float* gxpos, const float* gxmat, int wid, int g1, int g2) {
  const float* geom_aabb = MR(geom_aabb);
  const float* geom_rbound = MR(geom_rbound);
  const float* geom_margin = MR(geom_margin);
  float rb1 = geom_rbound[g1], rb2 = geom_rbound[g2];
  float mg1 = geom_margin[g1], mg2 = geom_margin[g2];
  const float* xp1 = gxpos + 3 * g1;
  const float* xp2 = gxpos + 3 * g2;
  const float* xm1 = gxmat + 9 * g1;
  const float* xm2 = gxmat + 9 * g2;
  int filt = m.opt_broadphase_filter;
  if (rb1 == 0.0f || rb2 == 0.0f) {
    if (filt & FILTER_PLANE) {
      if (rb1 == 0.0f) {
        float dif[3] = {xp2[0] - xp1[0], xp2[1] - xp1[1], xp2[2] - xp1[2]}, n[3] = {xm1[2], xm1[5], xm1[8]};
        return dot3(dif, n) <= rb2 + mg1 + mg2;
      } else {
        float dif[3] = {xp1[0] - xp2[0], xp1[1] - xp2[1], xp1[2] - xp2[2]}, n[3] = {xm2[2], xm2[5], xm2[8]};
        return dot3(dif, n) <= rb1 + mg1 + mg2;
      }
    }
    return true;
  }
  if (filt & FILTER_SPHERE) {
    float bound = rb1 + rb2 + mg1 + mg2;
    float dif[3] = {xp2[0] - xp1[0], xp2[1] - xp1[1], xp2[2] - xp1[2]};
    if (!(dot3(dif, dif) <= bound * bound)) return false;
  }
  if (filt & FILTER_AABB)
    if (!aabb_filter(geom_aabb + 6 * g1, geom_aabb + 6 * g2, geom_aabb + 6 * g1 + 3, geom_aabb + 6 * g2 + 3, mg1 + mg2, xp1, xp2, xm1, xm2))
      return false;
  if (filt & FILTER_OBB)
    if (!obb_filter(geom_aabb + 6 * g1, geom_aabb + 6 * g2, geom_aabb + 6 * g1 + 3, geom_aabb + 6 * g2 + 3, mg1 + mg2, xp1, xp2, xm1, xm2))
      return false;
  return true;
}
__device__ __forceinline__ bool broadphase_filter(const mjw_model_t& m, const Lay& L, const float* s, int wid, int g1, int g2) {
  return broadphase_filter_g(m, s + L.gxpos, s + L.gxmat, wid, g1, g2);
}

// narrowphase of one pair (collision_primitive.py:280-662); pair is type-sorted on the host
// BOX = false compiles out the pairs with a box (sphere-box, capsule-box; plane-box and box-box are
// handled by the caller): models without boxes then run a kernel with 118 instead of 128+ VGPRs and
// no scratch spills
template <bool BOX>
__device__ __forceinline__ void narrowphase_g(const mjw_model_t& m, const float* gxpos, const float* gxmat, int wid, int g1, int g2, float margin,
                                              Con2& c) {
  const float* geom_size = MR(geom_size);
  int t1 = m.geom_type[g1], t2 = m.geom_type[g2];
  const float* p1 = gxpos + 3 * g1;
  const float* p2 = gxpos + 3 * g2;
  const float* r1 = gxmat + 9 * g1;
  const float* r2 = gxmat + 9 * g2;
  const float* s1 = geom_size + 3 * g1;
  const float* s2 = geom_size + 3 * g2;
  float n1[3] = {r1[2], r1[5], r1[8]}, n2[3] = {r2[2], r2[5], r2[8]};
  c.n = 0;
  if (t1 == GEOM_PLANE && t2 == GEOM_SPHERE) {
    c.dist[0] = plane_sphere(c.pos[0], n1, p1, p2, s2[0]);
    make_frame(c.frame[0], n1);
    c.n = 1;
  } else if (t1 == GEOM_PLANE && t2 == GEOM_CAPSULE) {
    plane_capsule(c, n1, p1, p2, n2, s2[0], s2[1]);
  } else if (t1 == GEOM_SPHERE && t2 == GEOM_SPHERE) {
    float nrm[3];
    c.dist[0] = sphere_sphere(c.pos[0], nrm, p1, s1[0], p2, s2[0]);
    make_frame(c.frame[0], nrm);
    c.n = 1;
  } else if (t1 == GEOM_SPHERE && t2 == GEOM_CAPSULE) {
    float a[3], b[3], pt[3], nrm[3];
    for (int i = 0; i < 3; i++) { a[i] = p2[i] - n2[i] * s2[1]; b[i] = p2[i] + n2[i] * s2[1]; }
    closest_segment_point(pt, a, b, p1);
    c.dist[0] = sphere_sphere(c.pos[0], nrm, p1, s1[0], pt, s2[0]);
    make_frame(c.frame[0], nrm);
    c.n = 1;
  } else if (t1 == GEOM_CAPSULE && t2 == GEOM_CAPSULE) {
    capsule_capsule(c, p1, n1, s1[0], s1[1], p2, n2, s2[0], s2[1], margin);
  } else if (BOX && t1 == GEOM_SPHERE && t2 == GEOM_BOX) {  // collision_primitive.py:1047-1114
    float nrm[3];
    c.dist[0] = sphere_box(c.pos[0], nrm, p1, s1[0], p2, r2, s2);
    make_frame(c.frame[0], nrm);
    c.n = 1;
  } else if (BOX && t1 == GEOM_CAPSULE && t2 == GEOM_BOX) {  // collision_primitive.py:1117-1199
    capsule_box(c, p1, n1, s1[0], s1[1], p2, r2, s2);
  }
}
template <bool BOX>
__device__ __forceinline__ void narrowphase(const mjw_model_t& m, const Lay& L, const float* s, int wid, int g1, int g2, float margin, Con2& c) {
  narrowphase_g<BOX>(m, s + L.gxpos, s + L.gxmat, wid, g1, g2, margin, c);
}


// -------------------------------------------------------------------------------------------
// constraint.py
// -------------------------------------------------------------------------------------------
// constraint.py:52-121 (writes LDS row scalars)
__device__ __forceinline__ void efc_row(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, float* s, int wid, int r, float pos_aref, float pos_imp,
                        float invweight, const float* solref, const float* solimp, float margin, float vel, float frictionloss,
                        int type, int id) {
  float timestep = MR(opt_timestep)[0];
  float timeconst = solref[0], dampratio = solref[1];
  float dmin = solimp[0], dmax = solimp[1], width = solimp[2], mid = solimp[3], power = solimp[4];
  if (!(m.opt_disableflags & DSBL_REFSAFE)) timeconst = fmaxf(timeconst, 2.0f * timestep);
  dmin = clampf(dmin, MJW_MINIMP, MJW_MAXIMP);
  dmax = clampf(dmax, MJW_MINIMP, MJW_MAXIMP);
  width = fmaxf(MJW_MINVAL, width);
  mid = clampf(mid, MJW_MINIMP, MJW_MAXIMP);
  power = fmaxf(1.0f, power);
  float dmax_sq = dmax * dmax;
  float k = 1.0f / (dmax_sq * timeconst * timeconst * dampratio * dampratio);
  float b = 2.0f / (dmax * timeconst);
  if (solref[0] <= 0.0f) k = -solref[0] / dmax_sq;
  if (solref[1] <= 0.0f) b = -solref[1] / dmax;
  float imp_x = fabsf(pos_imp) / width;
  float imp_y = imp_shape(imp_x, mid, power);
  float imp = dmin + imp_y * (dmax - dmin);
  imp = clampf(imp, dmin, dmax);
  if (imp_x > 1.0f) imp = dmax;
  float D = 1.0f / fmaxf(invweight * (1.0f - imp) / imp, MJW_MINVAL);
  float aref = -k * imp * pos_aref - b * vel;
  long gr = (long)wid * d.njmax + r;
  d.efc_D[(long)wid * d.njmax_pad + r] = D;
  d.efc_vel[gr] = vel;
  d.efc_aref[gr] = aref;
  d.efc_pos[gr] = pos_aref + margin;
  d.efc_margin[gr] = margin;
  d.efc_frictionloss[gr] = frictionloss;
  d.efc_type[gr] = type;
  d.efc_id[gr] = id;
  if (L.efc_D >= 0) {  // generic fused solver reads them from LDS
    s[L.efc_D + r] = D;
    s[L.efc_aref + r] = aref;
    s[L.efc_frictionloss + r] = frictionloss;
    reinterpret_cast<int*>(s)[L.efc_type + r] = type;
  }
}

// one entry of constraint Jacobian row r (LDS in the generic layout, else global efc_J)
__device__ __forceinline__ void put_J(const mjw_data_t& d, const Lay& L, float* s, int wid, int np, int r, int k, float v) {
  if (L.J >= 0) s[L.J + r * L.nvs + k] = v;
  else d.efc_J[((long)wid * d.njmax_pad + r) * np + k] = v;
}

// the rows of the ballot `bal` (row nefc + rank for each set lane, in lane order) whose Jacobian has up
// to three non-zeros (columns c0 < c1 < c2 of the source lane, -1 = none): one coalesced row store per
// row with the lanes over columns, instead of kJ scattered stores by each row's own lane
__device__ __forceinline__ void put_J_rows(const mjw_data_t& d, const Lay& L, float* s, int wid, int np, int kJ, int njmax, int lane,
                                           unsigned long long bal, int nefc, int c0, float v0, int c1 = -1, float v1 = 0.0f, int c2 = -1,
                                           float v2 = 0.0f) {
  for (int rr = nefc; bal && rr < njmax; rr++) {
    const int src = __builtin_ctzll(bal);
    bal &= bal - 1;
    const int a0 = __builtin_amdgcn_readlane(c0, src), a1 = __builtin_amdgcn_readlane(c1, src), a2 = __builtin_amdgcn_readlane(c2, src);
    const float w0 = rdlane(v0, src), w1 = rdlane(v1, src), w2 = rdlane(v2, src);
    if (lane < kJ) put_J(d, L, s, wid, np, rr, lane, lane == a0 ? w0 : (lane == a1 ? w1 : (lane == a2 ? w2 : 0.0f)));
  }
}

// support.py:396-432 restricted to one dof; returns jacp, jacr (zero when not in tree).  The
// reference walks bodyid's ancestors looking for the dof's body; with bodies in DFS pre-order that
// is the range test db <= bodyid < subtree_end(db), so the per-lane (db, dend) pair is loaded once
// by the caller instead of a chain of dependent parent loads per contact.
__device__ __forceinline__ void jac_dof_root(const Lay& L, const float* s, const float* point, int bodyid, int root, int dofid, int db,
                                             int dend, float* jacp, float* jacr) {
  const bool in_tree = db == 0 || (bodyid >= db && bodyid < dend);
  if (!in_tree) { jacp[0] = jacp[1] = jacp[2] = jacr[0] = jacr[1] = jacr[2] = 0.0f; return; }
  float off[3];
  for (int i = 0; i < 3; i++) off[i] = point[i] - s[L.subtree_com + 3 * root + i];
  const float* cd = s + L.cdof + 6 * dofid;
  float c[3];
  cross3(c, cd, off);
  for (int i = 0; i < 3; i++) { jacp[i] = cd[3 + i] + c[i]; jacr[i] = cd[i]; }
}

__device__ __forceinline__ void jac_dof(const mjw_model_t& m, const Lay& L, const float* s, const float* point, int bodyid,
                                        int dofid, int db, int dend, float* jacp, float* jacr) {
  jac_dof_root(L, s, point, bodyid, m.body_rootid[bodyid], dofid, db, dend, jacp, jacr);
}

// constraint.py:124-365 (_equality_connect) and :792-1110 (_equality_weld): rows r0 .. r0+2 (+5).
// The anchor / orientation geometry is wave-uniform; lane i holds dof i of the Jacobian rows, and
// each row's J.qvel is a wave sum.  Lane k < nrow then writes row r0 + k's scalars.
__device__ __forceinline__ void eq_connect_weld(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, float* s, int wid, int lane,
                                                int e, int r0, bool weld, int dof_db, int dof_dend, int kJ, int np) {
  const float* data = MR(eq_data) + 11 * e;
  const int o1 = m.eq_obj1id[e], o2 = m.eq_obj2id[e];
  const bool site = m.eq_objtype[e] == OBJ_SITE && m.nsite > 0;
  const float* xpos = s + L.xpos;
  const float* xquat = s + L.xquat;
  const float* xmat = s + L.xmat;
  int b1, b2;
  float p1[3], p2[3], q[4] = {1, 0, 0, 0}, q1[4] = {1, 0, 0, 0};
  if (site) {
    const float* site_pos = MR(site_pos);
    const float* site_quat = MR(site_quat);
    b1 = m.site_bodyid[o1];
    b2 = m.site_bodyid[o2];
    rot_vec_quat(p1, site_pos + 3 * o1, xquat + 4 * b1);  // smooth.py:223 site_xpos
    rot_vec_quat(p2, site_pos + 3 * o2, xquat + 4 * b2);
    for (int k = 0; k < 3; k++) { p1[k] += xpos[3 * b1 + k]; p2[k] += xpos[3 * b2 + k]; }
    if (weld) {
      float t[4];
      mul_quat(q, xquat + 4 * b1, site_quat + 4 * o1);
      mul_quat(t, xquat + 4 * b2, site_quat + 4 * o2);
      q1[0] = t[0]; q1[1] = -t[1]; q1[2] = -t[2]; q1[3] = -t[3];
    }
  } else {
    b1 = o1;
    b2 = o2;
    // connect: anchor1 = data[0:3] on body1, anchor2 = data[3:6] on body2; weld swaps them
    const float* a1 = weld ? data + 3 : data;
    const float* a2 = weld ? data : data + 3;
    matvec3(p1, xmat + 9 * b1, a1);
    matvec3(p2, xmat + 9 * b2, a2);
    for (int k = 0; k < 3; k++) { p1[k] = xpos[3 * b1 + k] + p1[k]; p2[k] = xpos[3 * b2 + k] + p2[k]; }
    if (weld) {
      mul_quat(q, xquat + 4 * b1, data + 6);
      q1[0] = xquat[4 * b2]; q1[1] = -xquat[4 * b2 + 1]; q1[2] = -xquat[4 * b2 + 2]; q1[3] = -xquat[4 * b2 + 3];
    }
  }
  const float torquescale = data[10];
  float jp[3] = {0, 0, 0}, jr[3] = {0, 0, 0};
  if (lane < m.nv) {
    float j1p[3], j1r[3], j2p[3], j2r[3];
    jac_dof(m, L, s, p1, b1, lane, dof_db, dof_dend, j1p, j1r);
    jac_dof(m, L, s, p2, b2, lane, dof_db, dof_dend, j2p, j2r);
    for (int k = 0; k < 3; k++) jp[k] = j1p[k] - j2p[k];
    if (weld) {
      float dr[3], t[4], u[4];
      for (int k = 0; k < 3; k++) dr[k] = (j1r[k] - j2r[k]) * torquescale;
      quat_mul_axis(t, q1, dr);
      mul_quat(u, t, q);
      for (int k = 0; k < 3; k++) jr[k] = 0.5f * u[1 + k];
    }
  }
  const float qv = lane < m.nv ? s[L.qvel + lane] : 0.0f;
  const int nrow = weld ? 6 : 3;
  float myjq = 0.0f;
  for (int k = 0; k < nrow; k++) {
    const float v = k < 3 ? sel3(jp, k) : sel3(jr, k - 3);
    if (lane < kJ) put_J(d, L, s, wid, np, r0 + k, lane, lane < m.nv ? v : 0.0f);
    const float jq = dsum(lane < m.nv ? v * qv : 0.0f);
    if (lane == k) myjq = jq;
  }
  float cpos[3], crot[3] = {0, 0, 0};
  for (int k = 0; k < 3; k++) cpos[k] = p1[k] - p2[k];
  float pos_imp;
  if (weld) {
    float cq[4];
    mul_quat(cq, q1, q);
    for (int k = 0; k < 3; k++) crot[k] = cq[1 + k] * torquescale;
    pos_imp = sqrtf(dot3(cpos, cpos) + dot3(crot, crot));
  } else {
    pos_imp = sqrtf(dot3(cpos, cpos));
  }
  if (lane < nrow) {
    const float* biw = MR(body_invweight0);
    const int c = lane < 3 ? 0 : 1;
    const float invweight = biw[2 * b1 + c] + biw[2 * b2 + c];
    const float pos = lane < 3 ? sel3(cpos, lane) : sel3(crot, lane - 3);
    efc_row(m, d, L, s, wid, r0 + lane, pos, pos_imp, invweight, MR(eq_solref) + 2 * e, MR(eq_solimp) + 5 * e, 0.0f, myjq, 0.0f,
            CNSTR_EQUALITY, e);
  }
}

// collision_driver.py:754-789 + constraint.py:2209-2779 (friction-dof, limits, pyramidal contacts)
// friction (limit = false, constraint.py:1204-1313) or limit (limit = true, :1547-1665) rows of the
// fixed tendons from row nefc on; returns the rows added.  collision_and_constraints counts these rows
// where the reference emits them (after the dof friction / joint limit rows) and fills them in here
// once the contact rows are done, so that the tendon code does not overlap the narrowphase's
// register peak (inline there it pushed the forward kernel into 16 B/lane of scratch).
__device__ __forceinline__ int tendon_rows(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, float* s, int wid, int lane, int nefc,
                                        int kJ, bool limit) {
  const int nv = m.nv, np = m.nv_pad, njmax = d.njmax;
  const float* qvel = s + L.qvel;
  const float* tiw = MR(tendon_invweight0);
  const float* tfl = MR(tendon_frictionloss);
  const float* trng = MR(tendon_range);
  const float* tmar = MR(tendon_margin);
  const float* tsr = limit ? MR(tendon_solref_lim) : MR(tendon_solref_fri);
  const float* tsi = limit ? MR(tendon_solimp_lim) : MR(tendon_solimp_fri);
  int added = 0;
  for (int base = 0; base < m.ntendon; base += LPW) {
    const int t = base + lane;
    bool act = false;
    float pos = 0.0f, scl = 1.0f, tm = 0.0f;
    if (t < m.ntendon) {
      if (limit) {
        if (m.tendon_limited[t]) {
          const float len = ten_len(m, d, wid, s + L.qpos, t);
          const float dmn = len - trng[2 * t], dmx = trng[2 * t + 1] - len;
          tm = tmar[t];
          pos = fminf(dmn, dmx) - tm;
          scl = (float)(dmn < dmx) * 2.0f - 1.0f;
          act = pos < 0.0f;
        }
      } else {
        act = tfl[t] > 0.0f;
      }
    }
    unsigned long long bal = __ballot(act);
    int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0));
    int r = nefc + added + rank;
    if (act && r < njmax) {
      for (int k = 0; k < kJ; k++) put_J(d, L, s, wid, np, r, k, k < nv ? scl * ten_coef(m, d, wid, t, k) : 0.0f);
      if (limit)
        efc_row(m, d, L, s, wid, r, pos, pos, tiw[t], tsr + 2 * t, tsi + 5 * t, tm, scl * ten_vel(m, d, wid, qvel, t), 0.0f,
                CNSTR_LIMIT_TENDON, t);
      else
        efc_row(m, d, L, s, wid, r, 0.0f, 0.0f, tiw[t], tsr + 2 * t, tsi + 5 * t, 0.0f, ten_vel(m, d, wid, qvel, t), tfl[t],
                CNSTR_FRICTION_TENDON, t);
    }
    added += __popcll(bal);
  }
  return added;
}

template <bool BOX, bool TEN, bool POOL = false>
__device__ __forceinline__ void collision_and_constraints(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, WS& w) {
  const int wid = w.wid, lane = w.lane;
  float* s = w.s;
  int* si = w.si;
  const int nv = m.nv, nvs = L.nvs, njmax = d.njmax;
  const float* qvel = s + L.qvel;
  int nefc = 0, nf = 0, nl = 0, ne = 0;
  const bool dsbl_constraint = m.opt_disableflags & DSBL_CONSTRAINT;
  const int np = m.nv_pad;
  const int kJ = L.J >= 0 ? nv : np;  // global rows also get their zero padding
  const int CM = L.cmax;
  // this lane's dof body and its DFS subtree end (jac_dof's ancestor test), loaded once
  const int dof_db = lane < nv ? m.dof_bodyid[lane] : 0;
  const int dof_dend = lane < nv ? m.body_subtree_end[dof_db] : 0;
  WSYNC();  // contact staging may alias the qM region read by crb_qM
  PROF_T0_SUB();

  // --- connect rows, then weld rows (constraint.py:124-365, 792-1110), each in equality index order
  if (!dsbl_constraint && !(m.opt_disableflags & DSBL_EQUALITY) && m.neq_cw > 0) {
    for (int weld = 0; weld < 2; weld++) {
      for (int e = 0; e < m.neq; e++) {
        if (m.eq_type[e] != (weld ? EQ_WELD : EQ_CONNECT) || !d.eq_active[(long)wid * m.neq + e]) continue;
        const int nrow = weld ? 6 : 3, r0 = nefc;
        nefc += nrow;
        ne += nrow;
        if (r0 + nrow <= njmax) eq_connect_weld(m, d, L, s, wid, lane, e, r0, weld != 0, dof_db, dof_dend, kJ, np);
      }
    }
  }
  // --- joint equality rows (constraint.py:367-495), in equality index order
  if (!dsbl_constraint && !(m.opt_disableflags & DSBL_EQUALITY) && m.neq > 0) {
    const float* eq_data = MR(eq_data);
    const float* eq_solref = MR(eq_solref);
    const float* eq_solimp = MR(eq_solimp);
    const float* qpos0 = MR(qpos0);
    const float* dof_invweight0 = MR(dof_invweight0);
    const float* qpos = s + L.qpos;
    for (int base = 0; base < m.neq; base += LPW) {
      int e = base + lane;
      bool act = e < m.neq && m.eq_type[e] == EQ_JOINT && d.eq_active[(long)wid * m.neq + e] != 0;
      unsigned long long bal = __ballot(act);
      int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0));
      int r = nefc + rank;
      int da1 = -1, da2 = -1;
      float d2 = 0.0f;
      if (act && r < njmax) {
        const float* data = eq_data + 11 * e;
        int j1 = m.eq_obj1id[e], j2 = m.eq_obj2id[e];
        da1 = m.jnt_dofadr[j1];
        int qa1 = m.jnt_qposadr[j1];
        float pos, Jqvel, invweight;
        if (j2 > -1) {
          int qa2 = m.jnt_qposadr[j2];
          da2 = m.jnt_dofadr[j2];
          float dif = qpos[qa2] - qpos0[qa2];
          float rhs = data[0] + dif * (data[1] + dif * (data[2] + dif * (data[3] + dif * data[4])));
          d2 = data[1] + dif * (2.0f * data[2] + dif * (3.0f * data[3] + dif * 4.0f * data[4]));
          pos = qpos[qa1] - qpos0[qa1] - rhs;
          Jqvel = qvel[da1] - qvel[da2] * d2;
          invweight = dof_invweight0[da1] + dof_invweight0[da2];
        } else {
          pos = qpos[qa1] - qpos0[qa1] - data[0];
          Jqvel = qvel[da1];
          invweight = dof_invweight0[da1];
        }
        efc_row(m, d, L, s, wid, r, pos, pos, invweight, eq_solref + 2 * e, eq_solimp + 5 * e, 0.0f, Jqvel, 0.0f,
                CNSTR_EQUALITY, e);
      }
      put_J_rows(d, L, s, wid, np, kJ, njmax, lane, bal, nefc, da1, 1.0f, da2, -d2);
      int cnt = __popcll(bal);
      nefc += cnt;
      ne += cnt;
    }
  }
  // --- tendon equality rows (constraint.py:498-674), in equality index order: L1 - L1_0 = poly(L2 - L2_0),
  // J = J1 - poly'(L2 - L2_0) J2 (lane = dof)
  if (TEN && !dsbl_constraint && !(m.opt_disableflags & DSBL_EQUALITY) && m.neq > 0 && m.ntendon > 0) {
    const float* eq_data = MR(eq_data);
    const float* len0 = MR(tendon_length0);
    const float* tiw = MR(tendon_invweight0);
    const float* qpos = s + L.qpos;
    for (int e = 0; e < m.neq; e++) {
      if (m.eq_type[e] != EQ_TENDON || !d.eq_active[(long)wid * m.neq + e]) continue;
      const int r = nefc;
      nefc++;
      ne++;
      if (r >= njmax) continue;
      const float* data = eq_data + 11 * e;
      const int t1 = m.eq_obj1id[e], t2 = m.eq_obj2id[e];
      const float pos1 = ten_len(m, d, wid, qpos, t1) - len0[t1];
      float pos, deriv = 0.0f, invweight = tiw[t1];
      if (t2 > -1) {
        invweight += tiw[t2];
        const float dif = ten_len(m, d, wid, qpos, t2) - len0[t2];
        pos = pos1 - (data[0] + data[1] * dif + data[2] * dif * dif + data[3] * dif * dif * dif + data[4] * dif * dif * dif * dif);
        deriv = data[1] + 2.0f * data[2] * dif + 3.0f * data[3] * dif * dif + 4.0f * data[4] * dif * dif * dif;
      } else {
        pos = pos1 - data[0];
      }
      float Jk = 0.0f;
      if (lane < nv) {
        Jk = ten_coef(m, d, wid, t1, lane);
        if (deriv != 0.0f) Jk += ten_coef(m, d, wid, t2, lane) * -deriv;
      }
      for (int k = lane; k < kJ; k += LPW) put_J(d, L, s, wid, np, r, k, k == lane ? Jk : 0.0f);
      const float Jqvel = dsum(lane < nv ? Jk * qvel[lane] : 0.0f);
      if (lane == 0)
        efc_row(m, d, L, s, wid, r, pos, pos, invweight, MR(eq_solref) + 2 * e, MR(eq_solimp) + 5 * e, 0.0f, Jqvel, 0.0f, CNSTR_EQUALITY, e);
    }
  }
  // --- friction dof rows (constraint.py:1113-1190)
  if (!dsbl_constraint && !(m.opt_disableflags & DSBL_FRICTIONLOSS)) {
    const float* dof_frictionloss = MR(dof_frictionloss);
    const float* dof_invweight0 = MR(dof_invweight0);
    const float* dof_solref = MR(dof_solref);
    const float* dof_solimp = MR(dof_solimp);
    for (int base = 0; base < nv; base += LPW) {
      int i = base + lane;
      bool act = i < nv && dof_frictionloss[i] > 0.0f;
      unsigned long long bal = __ballot(act);
      int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0));
      int r = nefc + rank;
      if (act && r < njmax)
        efc_row(m, d, L, s, wid, r, 0.0f, 0.0f, dof_invweight0[i], dof_solref + 2 * i, dof_solimp + 5 * i, 0.0f, qvel[i],
                dof_frictionloss[i], CNSTR_FRICTION_DOF, i);
      put_J_rows(d, L, s, wid, np, kJ, njmax, lane, bal, nefc, i, 1.0f);
      int cnt = __popcll(bal);
      nefc += cnt;
      nf += cnt;
    }
    // --- friction tendon rows (constraint.py:1204-1313): counted here, filled after the contacts
    if (TEN && m.ntendon) {
      const float* tfl = MR(tendon_frictionloss);
      int cnt = 0;
      for (int base = 0; base < m.ntendon; base += LPW) cnt += __popcll(__ballot(base + lane < m.ntendon && tfl[base + lane] > 0.0f));
      if (lane == 0) si[L.iscratch + 56] = nefc;  // first friction tendon row (filled after the contacts)
      nefc += cnt;
      nf += cnt;
    }
  }
  // --- ball joint limits (constraint.py:1421-1543): one row on the joint's 3 dofs along -axis
  if (!dsbl_constraint && !(m.opt_disableflags & DSBL_LIMIT) && m.nlimited_ball > 0) {
    const float* jnt_range = MR(jnt_range);
    const float* jnt_margin = MR(jnt_margin);
    const float* jnt_solref = MR(jnt_solref);
    const float* jnt_solimp = MR(jnt_solimp);
    const float* dof_invweight0 = MR(dof_invweight0);
    for (int base = 0; base < m.nlimited_ball; base += LPW) {
      const int idx = base + lane;
      bool act = false;
      int j = 0;
      float pos = 0.0f, axis[3] = {0, 0, 0}, jm = 0.0f;
      if (idx < m.nlimited_ball) {
        j = m.jnt_limited_ball_adr[idx];
        const float* qp = s + L.qpos + m.jnt_qposadr[j];
        float q[4] = {qp[0], qp[1], qp[2], qp[3]}, aa[3];
        normalize4(q);
        quat_to_vel(aa, q);
        const float angle = sqrtf(dot3(aa, aa));  // math.py:261-265 normalize_with_norm
        for (int k = 0; k < 3; k++) axis[k] = angle == 0.0f ? aa[k] : aa[k] / angle;
        jm = jnt_margin[j];
        pos = fmaxf(jnt_range[2 * j], jnt_range[2 * j + 1]) - angle - jm;
        act = pos < 0.0f;
      }
      unsigned long long bal = __ballot(act);
      int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0));
      int r = nefc + rank;
      const int dab = act ? m.jnt_dofadr[j] : -3;
      put_J_rows(d, L, s, wid, np, kJ, njmax, lane, bal, nefc, dab, -axis[0], dab + 1, -axis[1], dab + 2, -axis[2]);
      if (act && r < njmax) {
        const int da = dab;
        float Jqvel = -axis[0] * qvel[da];
        Jqvel -= axis[1] * qvel[da + 1];
        Jqvel -= axis[2] * qvel[da + 2];
        efc_row(m, d, L, s, wid, r, pos, pos, dof_invweight0[da], jnt_solref + 2 * j, jnt_solimp + 5 * j, jm, Jqvel, 0.0f,
                CNSTR_LIMIT_JOINT, j);
      }
      int cnt = __popcll(bal);
      nefc += cnt;
      nl += cnt;
    }
  }
  // --- joint limits (constraint.py:1316-1418)
  if (!dsbl_constraint && !(m.opt_disableflags & DSBL_LIMIT)) {
    const float* jnt_range = MR(jnt_range);
    const float* jnt_margin = MR(jnt_margin);
    const float* jnt_solref = MR(jnt_solref);
    const float* jnt_solimp = MR(jnt_solimp);
    const float* dof_invweight0 = MR(dof_invweight0);
    for (int base = 0; base < m.nlimited; base += LPW) {
      int idx = base + lane;
      bool act = false;
      int j = 0;
      float pos = 0.0f, dmn = 0.0f, dmx = 0.0f, jm = 0.0f;
      if (idx < m.nlimited) {
        j = m.jnt_limited_slide_hinge_adr[idx];
        float q = s[L.qpos + m.jnt_qposadr[j]];
        dmn = q - jnt_range[2 * j];
        dmx = jnt_range[2 * j + 1] - q;
        jm = jnt_margin[j];
        pos = fminf(dmn, dmx) - jm;
        act = pos < 0.0f;
      }
      unsigned long long bal = __ballot(act);
      int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0));
      int r = nefc + rank;
      const int da = act ? m.jnt_dofadr[j] : -1;
      const float Jv = (float)(dmn < dmx) * 2.0f - 1.0f;
      if (act && r < njmax)
        efc_row(m, d, L, s, wid, r, pos, pos, dof_invweight0[da], jnt_solref + 2 * j, jnt_solimp + 5 * j, jm, Jv * qvel[da], 0.0f,
                CNSTR_LIMIT_JOINT, j);
      put_J_rows(d, L, s, wid, np, kJ, njmax, lane, bal, nefc, da, Jv);
      int cnt = __popcll(bal);
      nefc += cnt;
      nl += cnt;
    }
    // --- tendon limits (constraint.py:1547-1665): counted here, filled after the contacts
    if (TEN && m.ntendon) {
      const float* trng = MR(tendon_range);
      const float* tmar = MR(tendon_margin);
      int cnt = 0;
      for (int base = 0; base < m.ntendon; base += LPW) {
        const int t = base + lane;
        bool act = false;
        if (t < m.ntendon && m.tendon_limited[t]) {
          const float len = ten_len(m, d, wid, s + L.qpos, t);
          act = fminf(len - trng[2 * t], trng[2 * t + 1] - len) - tmar[t] < 0.0f;
        }
        cnt += __popcll(__ballot(act));
      }
      if (lane == 0) si[L.iscratch + 57] = nefc;  // first limit tendon row
      nefc += cnt;
      nl += cnt;
    }
  }

  PROF_MARK_SUB(PH_C_ROWS0);
  // --- collision + contact rows (collision_driver.py:697-789, constraint.py:1668-1936)
  int ncon_total = 0;
  const bool do_contact = d.naconmax > 0 && !(m.opt_disableflags & (DSBL_CONSTRAINT | DSBL_CONTACT));
  if (do_contact) {
    const float* body_invweight0 = MR(body_invweight0);
    const float impratio_invsqrt = MR(opt_impratio_invsqrt)[0];
    // broadphase over all pairs once; survivors (in pair order) -> plist
    int npass = 0;
    int* plist = si + L.plist;
    // POOL: the candidates are this world's contacts in the pool (a contactfilter callback may have
    // edited them), in slot order = the pair order the narrowphase wrote them in
    // the world's slot range [pool_k0, pool_k1) from pool_ranges_kernel (ncon_world: first slot, span), so a
    // world scans its own contacts instead of the whole pool
    const int npool = POOL ? min(d.nacon[0], d.naconmax) : 0;
    const int pool_k0 = POOL ? d.ncon_world[2L * wid] : 0;
    const int pool_k1 = POOL ? min(npool, pool_k0 + d.ncon_world[2L * wid + 1]) : 0;
    for (int base = 0; base < (POOL ? 0 : m.nxn); base += LPW) {
      int p = base + lane;
      bool pass = false;
      if (p < m.nxn) {
        int g1 = m.nxn_geom_pair[2 * p], g2 = m.nxn_geom_pair[2 * p + 1];
        pass = m.nxn_pairid[2 * p + 1] >= 0 || broadphase_filter(m, L, s, wid, g1, g2);
      }
      unsigned long long bal = __ballot(pass);
      int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0));
      if (pass) plist[npass + rank] = p;
      npass += __popcll(bal);
    }
    // the broadphase count joins the world's first contact-slot reservation below when ncollision sits
    // right after nacon (io.py allocates them so): one 64-bit atomic per world instead of two same-address
    // 32-bit ones -- the separate ncollision atomic measured 2.5 % of the step kernel (humanoid CG, 0.453 ->
    // 0.443 ms without it) and 5 % of the Newton forward kernel (profiles/r06_ab_ncoll.log); the combined atomic
    // against the two: step kernel 0.493 -> 0.442 ms, Newton forward 0.310 -> 0.247 ms (profiles/r06_ab_cnt64.log)
    const bool cnt64 = d.ncollision == d.nacon + 1;
    int pend = POOL ? 0 : npass;
    if (!cnt64 && pend > 0 && lane == 0) atomicAdd(d.ncollision, pend);
    if (!cnt64) pend = 0;
    WSYNC();
    PROF_MARK_SUB(PH_C_BROAD);
    const float* geom_margin = MR(geom_margin);
    int round = 0;
    while (true) {
      const int rbeg = round * CM, rend = rbeg + CM;
      int running = 0;  // contacts found so far (world-local, in pair order)
      for (int base = POOL ? pool_k0 : 0; base < (POOL ? pool_k1 : npass); base += LPW) {
        int k = base + lane;
        if constexpr (POOL) {
          // constraint.py:1731: contacts without the CONSTRAINT type bit get no rows (and no row address)
          const bool mine = k < pool_k1 && d.contact_worldid[k] == wid;
          const bool sel = mine && (d.contact_type[k] & 1);
          if (mine && !sel)
            for (int i = 0; i < m.nmaxpyramid; i++) d.contact_efc_address[(long)k * m.nmaxpyramid + i] = -1;
          const int incl = wave_scan_incl((int)sel);
          const int idx = running + incl - (int)sel;
          if (sel && idx >= rbeg && idx < rend) {
            float* rec = s + L.con + (idx - rbeg) * CREC;
            int* reci = reinterpret_cast<int*>(rec);
            const int g1 = d.contact_geom[2L * k], g2 = d.contact_geom[2L * k + 1];
            const int cb1 = m.geom_bodyid[g1], cb2 = m.geom_bodyid[g2];
            rec[0] = d.contact_dist[k];
            rec[1] = d.contact_includemargin[k];
            for (int i = 0; i < 3; i++) rec[2 + i] = d.contact_pos[3L * k + i];
            for (int i = 0; i < 9; i++) rec[5 + i] = d.contact_frame[9L * k + i];
            for (int i = 0; i < 5; i++) rec[14 + i] = d.contact_friction[5L * k + i];
            rec[19] = d.contact_solref[2L * k]; rec[20] = d.contact_solref[2L * k + 1];
            reci[21] = m.body_weldid[cb1] | (m.body_weldid[cb2] << 16);
            reci[22] = cb1 | (cb2 << 16);
            reci[32] = m.body_rootid[cb1] | (m.body_rootid[cb2] << 16);
            for (int i = 0; i < 5; i++) rec[23 + i] = d.contact_solimp[5L * k + i];
            reci[28] = d.contact_dim[k];
            reci[29] = g1;
            reci[30] = g2;
            reci[31] = k;  // the pool slot (set from the reserved range in the narrowphase mode)
          }
          running += __shfl(incl, 63, 64);
          continue;
        }
        Con2 c;
        c.n = 0;
        int g1 = 0, g2 = 0, pairid0 = -2;
        float margin = 0.0f;
        unsigned bmask = 0;  // plane-box: active corners (collision_primitive.py:737-790 writes all 8)
        bool pbox = false;
        bool ccd = false;  // convex pair: GJK/EPA below (collision_driver.py:74, collision_convex.py:701-890)
        if (k < npass) {
          int p = plist[k];
          g1 = m.nxn_geom_pair[2 * p];
          g2 = m.nxn_geom_pair[2 * p + 1];
          pairid0 = m.nxn_pairid[2 * p];
          margin = pairid0 > -1 ? MR(pair_margin)[pairid0] : geom_margin[g1] + geom_margin[g2];
          pbox = BOX && m.geom_type[g1] == GEOM_PLANE && m.geom_type[g2] == GEOM_BOX;
          ccd = BOX && m.nxn_ccdid[p] >= 0;
          if (ccd) {
            // pre-pass record (ccd_kernel): up to 4 points, each with its own distance
            const float* out = d.ccd_out + ((long)wid * m.nxn_ccd + m.nxn_ccdid[p]) * CCD_OUT;
            const int n = (int)out[0];
            for (int q = 0; q < 4; q++)
              if (q < n && out[4 + 4 * q] < margin && pairid0 >= -1) bmask |= 1u << q;
          } else if (pbox) {
            const float* r1 = s + L.gxmat + 9 * g1;
            float n1[3] = {r1[2], r1[5], r1[8]}, cp[3];
            for (int q = 0; q < 8; q++) {
              float dist = plane_box_corner(q, n1, s + L.gxpos + 3 * g1, s + L.gxpos + 3 * g2, s + L.gxmat + 9 * g2,
                                            MR(geom_size) + 3 * g2, cp);
              if (dist < margin && pairid0 >= -1) bmask |= 1u << q;
            }
          } else {
            narrowphase<BOX>(m, L, s, wid, g1, g2, margin, c);
          }
        }
        // active contacts (write_contact collision_core.py:199-213); plane-box corners and pre-pass points
        // (convex pairs, multi-point primitives) by their bit masks
        bool a0 = !ccd && c.n > 0 && c.dist[0] < margin && pairid0 >= -1;
        bool a1 = !ccd && c.n > 1 && c.dist[1] < margin && pairid0 >= -1;
        int cnt = (pbox || ccd) ? __popc(bmask) : (int)a0 + (int)a1;
        int incl = wave_scan_incl(cnt);
        int first = running + incl - cnt;
        bool stage0 = a0 && first >= rbeg && first < rend;
        bool stage1 = a1 && first + (int)a0 >= rbeg && first + (int)a0 < rend;
        bool stagebox = cnt > 0 && (pbox || ccd) && first < rend && first + cnt > rbeg;
        if (stage0 || stage1 || stagebox) {
          float gap, friction[5], solref[2], solimp[5];
          int condim;
          contact_params(m, wid, g1, g2, pairid0, &margin, &gap, &condim, friction, solref, solimp);
          // body and weld-body ids, packed: resolved here for all staged pairs at once instead of
          // per contact inside the serial row loops below
          const int cb1 = m.geom_bodyid[g1], cb2 = m.geom_bodyid[g2];
          const int cbodies = cb1 | (cb2 << 16), cwelds = m.body_weldid[cb1] | (m.body_weldid[cb2] << 16);
          const int croots = m.body_rootid[cb1] | (m.body_rootid[cb2] << 16);
          if (pbox) {
            const float* r1 = s + L.gxmat + 9 * g1;
            float n1[3] = {r1[2], r1[5], r1[8]}, frame[9];
            make_frame(frame, n1);
            int kk = 0;
            for (int q = 0; q < 8; q++) {
              if (!(bmask & (1u << q))) continue;
              int idx = first + kk;
              kk++;
              if (idx < rbeg || idx >= rend) continue;
              float* rec = s + L.con + (idx - rbeg) * CREC;
              float cp[3];
              rec[0] = plane_box_corner(q, n1, s + L.gxpos + 3 * g1, s + L.gxpos + 3 * g2, s + L.gxmat + 9 * g2,
                                        MR(geom_size) + 3 * g2, cp);
              rec[1] = margin - gap;
              for (int i = 0; i < 3; i++) rec[2 + i] = cp[i];
              for (int i = 0; i < 9; i++) rec[5 + i] = frame[i];
              for (int i = 0; i < 5; i++) rec[14 + i] = friction[i];
              rec[19] = solref[0]; rec[20] = solref[1];
              reinterpret_cast<int*>(rec)[21] = cwelds; reinterpret_cast<int*>(rec)[22] = cbodies;
              reinterpret_cast<int*>(rec)[32] = croots;
              for (int i = 0; i < 5; i++) rec[23 + i] = solimp[i];
              int* reci = reinterpret_cast<int*>(rec);
              reci[28] = condim | ((pairid0 + 1) << 8);  // + the explicit <pair> id
              reci[29] = g1;
              reci[30] = g2;
            }
          }
          if (ccd) {
            const float* out = d.ccd_out + ((long)wid * m.nxn_ccd + m.nxn_ccdid[plist[k]]) * CCD_OUT;
            int kk = 0;
            for (int q = 0; q < 4; q++) {
              if (!(bmask & (1u << q))) continue;
              int idx = first + kk;
              kk++;
              if (idx < rbeg || idx >= rend) continue;
              float* rec = s + L.con + (idx - rbeg) * CREC;
              float frame[9];
              make_frame(frame, out + 20 + 3 * q);  // each point's own normal (heightfield pairs)
              rec[0] = out[4 + 4 * q];
              rec[1] = margin - gap;
              for (int i = 0; i < 3; i++) rec[2 + i] = out[5 + 4 * q + i];
              for (int i = 0; i < 9; i++) rec[5 + i] = frame[i];
              for (int i = 0; i < 5; i++) rec[14 + i] = friction[i];
              rec[19] = solref[0]; rec[20] = solref[1];
              reinterpret_cast<int*>(rec)[21] = cwelds; reinterpret_cast<int*>(rec)[22] = cbodies;
              reinterpret_cast<int*>(rec)[32] = croots;
              for (int i = 0; i < 5; i++) rec[23 + i] = solimp[i];
              int* reci = reinterpret_cast<int*>(rec);
              reci[28] = condim | ((pairid0 + 1) << 8);  // + the explicit <pair> id
              reci[29] = g1;
              reci[30] = g2;
            }
          }
          int kk = 0;
#pragma unroll
          for (int sub = 0; sub < 2; sub++) {
            bool a = sub == 0 ? a0 : a1;
            if (!a) continue;
            int idx = first + kk;
            kk++;
            if (idx >= rbeg && idx < rend) {
              float* rec = s + L.con + (idx - rbeg) * CREC;
              rec[0] = c.dist[sub];
              rec[1] = margin - gap;
              for (int i = 0; i < 3; i++) rec[2 + i] = c.pos[sub][i];
              for (int i = 0; i < 9; i++) rec[5 + i] = c.frame[sub][i];
              for (int i = 0; i < 5; i++) rec[14 + i] = friction[i];
              rec[19] = solref[0]; rec[20] = solref[1];
              reinterpret_cast<int*>(rec)[21] = cwelds; reinterpret_cast<int*>(rec)[22] = cbodies;
              reinterpret_cast<int*>(rec)[32] = croots;
              for (int i = 0; i < 5; i++) rec[23 + i] = solimp[i];
              int* reci = reinterpret_cast<int*>(rec);
              reci[28] = condim | ((pairid0 + 1) << 8);  // + the explicit <pair> id
              reci[29] = g1;
              reci[30] = g2;
            }
          }
        }
        running += __shfl(incl, 63, 64);
      }
      ncon_total = running;
      int nstage = min(CM, running - rbeg);
      PROF_MARK_SUB(PH_C_NARROW);
      if (nstage <= 0) break;
      // global pool slot for this round (one atomic per world per round; the first also adds the
      // broadphase count into ncollision, the high word)
      int gbase = 0;
      if (!POOL && lane == 0) {
        if (pend > 0)
          gbase = (int)(unsigned)atomicAdd(reinterpret_cast<unsigned long long*>(d.nacon), ((unsigned long long)pend << 32) | (unsigned)nstage);
        else
          gbase = atomicAdd(d.nacon, nstage);
      }
      pend = 0;
      gbase = __shfl(gbase, 0, 64);
      WSYNC();
      // rows per staged contact (pyramidal: 1 or 2*(condim-1); elliptic: condim), prefix over contacts
      const bool ell = m.opt_cone == CONE_ELLIPTIC;
      int nrow = 0;
      if (lane < nstage) {
        const float* rec = s + L.con + lane * CREC;
        int condim = reinterpret_cast<const int*>(rec)[28] & 0xff;
        float pos = rec[0] - rec[1];
        // a contact past the global pool is dropped with its rows (collision_core.py:212-231)
        nrow = (pos < 0.0f && (POOL || gbase + lane < d.naconmax)) ? (condim == 1 ? 1 : (ell ? condim : 2 * (condim - 1))) : 0;
        if (!POOL) reinterpret_cast<int*>(s + L.con + lane * CREC)[31] = gbase + lane;
      }
      int rincl = wave_scan_incl(nrow);
      int rfirst = nefc + rincl - nrow;
      if (lane < nstage) si[L.iscratch + lane] = rfirst;
      int nrow_total = __shfl(rincl, 63, 64);
      WSYNC();
      // write contacts to the global pool (collision_core.py:213-231)
      if (lane < nstage) {
        const float* rec = s + L.con + lane * CREC;
        const int* reci = reinterpret_cast<const int*>(rec);
        int cid = POOL ? reci[31] : gbase + lane;
        if (POOL) {
          for (int i = 0; i < m.nmaxpyramid; i++) {
            int r = rfirst + i;
            d.contact_efc_address[(long)cid * m.nmaxpyramid + i] = (i < nrow && r < njmax) ? r : -1;
          }
        } else if (cid < d.naconmax) {
          d.contact_dist[cid] = rec[0];
          for (int i = 0; i < 3; i++) d.contact_pos[3L * cid + i] = rec[2 + i];
          for (int i = 0; i < 9; i++) d.contact_frame[9L * cid + i] = rec[5 + i];
          d.contact_includemargin[cid] = rec[1];
          for (int i = 0; i < 5; i++) d.contact_friction[5L * cid + i] = rec[14 + i];
          const int pid = (reci[28] >> 8) - 1;
          for (int i = 0; i < 2; i++) {
            d.contact_solref[2L * cid + i] = rec[19 + i];
            d.contact_solreffriction[2L * cid + i] = pid > -1 ? MR(pair_solreffriction)[2 * pid + i] : 0.0f;
          }
          for (int i = 0; i < 5; i++) d.contact_solimp[5L * cid + i] = rec[23 + i];
          d.contact_dim[cid] = reci[28] & 0xff;
          d.contact_geom[2L * cid] = reci[29];
          d.contact_geom[2L * cid + 1] = reci[30];
          d.contact_worldid[cid] = wid;
          d.contact_type[cid] = 1;
          d.contact_geomcollisionid[cid] = 0;
          int npr = nrow;
          for (int i = 0; i < m.nmaxpyramid; i++) {
            int r = rfirst + i;
            d.contact_efc_address[(long)cid * m.nmaxpyramid + i] = (i < npr && r < njmax) ? r : -1;
          }
        }
      }
      PROF_MARK_SUB(PH_C_POOL);
      // J entries: lane = dof, loop over staged contacts; efc_vel = J qvel by wave reduction
      for (int cc = 0; cc < nstage; cc++) {
        const float* rec = s + L.con + cc * CREC;
        const int* reci = reinterpret_cast<const int*>(rec);
        int condim = reci[28] & 0xff;
        int r0 = si[L.iscratch + cc];
        float pos = rec[0] - rec[1];
        if (TEN && m.nbodytrn && (POOL || gbase + cc < d.naconmax) && reci[29] >= 0 && reci[30] >= 0)  // smooth.py:2448-2602
          body_trn_contact(m, s + L.subtree_com, s + L.cdof, rec + 2, rec + 5, reci[22] & 0xffff, reci[22] >> 16, s + L.act_mom, si + L.act_nnz,
                           L.amax, lane);
        if (!(pos < 0.0f) || (!POOL && gbase + cc >= d.naconmax)) continue;
        int nr = condim == 1 ? 1 : (ell ? condim : 2 * (condim - 1));
        const int b1 = reci[21] & 0xffff, b2 = reci[21] >> 16;
        const float* cpos = rec + 2;
        const float* frame = rec + 5;
        const int i = lane;
        float jdp[3] = {0.0f, 0.0f, 0.0f}, jdr[3] = {0.0f, 0.0f, 0.0f};
        if (i < nv) {
          float j1p[3], j1r[3], j2p[3], j2r[3];
          jac_dof_root(L, s, cpos, b1, reci[32] & 0xffff, i, dof_db, dof_dend, j1p, j1r);
          jac_dof_root(L, s, cpos, b2, reci[32] >> 16, i, dof_db, dof_dend, j2p, j2r);
          for (int k = 0; k < 3; k++) { jdp[k] = j2p[k] - j1p[k]; jdr[k] = j2r[k] - j1r[k]; }
        }
        const float qv = i < nv ? qvel[i] : 0.0f;
        float Jn = frame[0] * jdp[0] + frame[1] * jdp[1] + frame[2] * jdp[2];
        for (int dimid = 0; dimid < nr; dimid++) {
          int r = r0 + dimid;
          if (r >= njmax) break;
          float Jval = Jn;
          if (ell && condim > 1) {
            // elliptic (constraint.py:2151-2160): row dimid is frame row dimid applied to the relative
            // translational (dimid < 3) or rotational jacobian
            if (dimid > 0) {
              const float* fr = dimid < 3 ? frame + 3 * dimid : frame + 3 * (dimid - 3);
              const float* jd = dimid < 3 ? jdp : jdr;
              Jval = fr[0] * jd[0] + fr[1] * jd[1] + fr[2] * jd[2];
            }
          } else if (condim > 1) {
            int dimid2 = dimid / 2 + 1;
            float frii = rec[14 + dimid2 - 1];
            float Ji;
            if (dimid2 < 3) Ji = frame[3 * dimid2] * jdp[0] + frame[3 * dimid2 + 1] * jdp[1] + frame[3 * dimid2 + 2] * jdp[2];
            else Ji = frame[3 * (dimid2 - 3)] * jdr[0] + frame[3 * (dimid2 - 3) + 1] * jdr[1] + frame[3 * (dimid2 - 3) + 2] * jdr[2];
            Jval = (dimid % 2 == 0) ? Jval + Ji * frii : Jval - Ji * frii;
          }
          if (i < kJ) put_J(d, L, s, wid, np, r, i, i < nv ? Jval : 0.0f);
          float jq = dsum(i < nv ? Jval * qv : 0.0f);
          if (lane == 0) s[L.jqvel + r] = jq;
        }
      }
      WSYNC();
      PROF_MARK_SUB(PH_C_JROWS);
      // row scalars: lane = contact row (constraint.py:1776-1936)
      for (int rr = lane; rr < nrow_total; rr += LPW) {
        int r = nefc + rr;
        if (r >= njmax) continue;
        // find owning staged contact (rows are contiguous per contact)
        int cc = 0;
        while (cc + 1 < nstage && si[L.iscratch + cc + 1] <= r) cc++;
        const float* rec = s + L.con + cc * CREC;
        const int* reci = reinterpret_cast<const int*>(rec);
        int condim = reci[28] & 0xff;
        int dimid = r - si[L.iscratch + cc];
        const int body1 = reci[22] & 0xffff, body2 = reci[22] >> 16;
        float invweight = body_invweight0[2 * body1] + body_invweight0[2 * body2];
        float Jqvel = s[L.jqvel + r];
        float pos = rec[0] - rec[1];
        if (ell && condim > 1) {
          // constraint.py:2168-2195: friction rows scale invweight by impratio^-1 (fri0 / frii)^2 and have
          // no position term; they use solreffriction when an explicit <pair> sets it (:2160-2165)
          float pos_aref = pos;
          const float* sref = rec + 19;
          if (dimid > 0) {
            const int pid = (reci[28] >> 8) - 1;
            const float* srf = POOL ? d.contact_solreffriction + 2L * reci[31] : (pid > -1 ? MR(pair_solreffriction) + 2 * pid : nullptr);
            if (srf && (srf[0] != 0.0f || srf[1] != 0.0f)) sref = srf;
            invweight = invweight * impratio_invsqrt * impratio_invsqrt;
            if (dimid > 1) {
              const float fri0 = rec[14], frii = rec[14 + dimid - 1];
              invweight *= fri0 * fri0 / (frii * frii);
            }
            pos_aref = 0.0f;
          }
          efc_row(m, d, L, s, wid, r, pos_aref, pos, invweight, sref, rec + 23, rec[1], Jqvel, 0.0f, CNSTR_CONTACT_ELLIPTIC, reci[31]);
          if (L.ecoef >= 0) {  // the generic solver's cone coefficient and contact extent of the row
            s[L.efc_pos + r] = dimid == 0 ? rec[14] * impratio_invsqrt : rec[14 + dimid - 1];
            si[L.efc_margin + r] = (r - dimid) | (condim << 16);
          }
          continue;
        }
        if (condim > 1) {
          float fri0 = rec[14];
          invweight = invweight + fri0 * fri0 * invweight;
          invweight = invweight * 2.0f * fri0 * fri0 * impratio_invsqrt * impratio_invsqrt;
        }
        int type = condim == 1 ? CNSTR_CONTACT_FRICTIONLESS : CNSTR_CONTACT_PYRAMIDAL;
        efc_row(m, d, L, s, wid, r, pos, pos, invweight, rec + 19, rec + 23, rec[1], Jqvel, 0.0f, type, reci[31]);
      }
      nefc += nrow_total;
      WSYNC();
      PROF_MARK_SUB(PH_C_SCAL);
      if (running <= rend) break;
      round++;
    }
    if (pend > 0 && lane == 0) atomicAdd(d.ncollision, pend);  // no contact staged: the count alone
  }
  (void)ncon_total;
  if (TEN && m.ntendon && !dsbl_constraint) {
    WSYNC();
    if (!(m.opt_disableflags & DSBL_FRICTIONLOSS)) tendon_rows(m, d, L, s, wid, lane, si[L.iscratch + 56], kJ, false);
    if (!(m.opt_disableflags & DSBL_LIMIT)) tendon_rows(m, d, L, s, wid, lane, si[L.iscratch + 57], kJ, true);
  }
  WSYNC();
  // write rows to global (efc arrays are (nworld, njmax[_pad]))
  const int nrows = min(nefc, njmax);
  if (L.J >= 0) {
    float* gJ = d.efc_J + (long)wid * d.njmax_pad * np;
    for (int e = lane; e < nrows * np; e += LPW) {
      int r = e / np, c = e - r * np;
      gJ[e] = c < nv ? s[L.J + r * nvs + c] : 0.0f;
    }
  }
  if (lane == 0) {
    d.ne[wid] = ne;
    d.nf[wid] = nf;
    d.nl[wid] = nl;
    d.nefc[wid] = nefc;
    si[L.iscratch + 60] = ne;
    si[L.iscratch + 61] = nf;
    si[L.iscratch + 62] = nefc;
  }
  WSYNC();
  PROF_MARK_SUB(PH_C_TAIL);
}

// smooth.py:2041-2147 (joint transmissions; moment rows packed in actuator order)
template <bool TEN>
__device__ __forceinline__ void transmission(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, WS& w) {
  const int wid = w.wid, lane = w.lane;
  float* s = w.s;
  int* si = w.si;
  const float* gear_all = MR(actuator_gear);
  int carry = 0;  // moment rows are packed in actuator order: rowadr = exclusive scan of nnz
  for (int a0 = 0; a0 < m.nu; a0 += LPW) {
    const int a = a0 + lane;
    int my_nnz = 0;
    if (a < m.nu) {
      const int tt = m.actuator_trntype[a];
      if (TEN && tt == TRN_TENDON) {
        my_nnz = m.ten_J_rownnz[m.actuator_trnid[2 * a]];
      } else if (TEN && (tt == TRN_SITE || tt == TRN_SLIDERCRANK || tt == TRN_BODY)) {
        my_nnz = trn_site_nnz(m, a);
      } else {
        const int jt0 = m.jnt_type[m.actuator_trnid[2 * a]];
        my_nnz = jt0 == JNT_FREE ? 6 : (jt0 == JNT_BALL ? 3 : 1);
      }
    }
    const int incl = wave_scan_incl(my_nnz);
    const int rowadr = carry + incl - my_nnz;
    carry += __shfl(incl, 63, 64);
    if (a >= m.nu) continue;
    const float* gear = gear_all + 6 * a;
    int trn = m.actuator_trntype[a];
    if (TEN && trn == TRN_TENDON) {
      // smooth.py:2244-2260: length = ten_length gear0, moment row = gear0 ten_J (the tendon's dofs)
      const int t = m.actuator_trnid[2 * a];
      const float length = ten_len(m, d, wid, s + L.qpos, t) * gear[0];
      const int nnz = my_nnz;
      s[L.act_len + a] = length;
      si[L.act_nnz + a] = nnz;
      const long gu = (long)wid * m.nu + a;
      d.actuator_length[gu] = length;
      d.moment_rownnz[gu] = nnz;
      d.moment_rowadr[gu] = rowadr;
      for (int k = 0; k < L.amax; k++) {
        const int dof = k < nnz ? m.ten_J_colind[m.ten_J_rowadr[t] + k] : 0;
        const float mk = k < nnz ? gear[0] * ten_coef(m, d, wid, t, dof) : 0.0f;
        s[L.act_mom + L.amax * a + k] = mk;
        si[L.act_momdof + L.amax * a + k] = dof;
        if (k < nnz) {
          d.actuator_moment[(long)wid * m.nJmom + rowadr + k] = mk;
          d.moment_colind[(long)wid * m.nJmom + rowadr + k] = dof;
        }
      }
      continue;
    }
    if (TEN && (trn == TRN_SITE || trn == TRN_SLIDERCRANK || trn == TRN_BODY)) {
      const long gu = (long)wid * m.nu + a;
      float* mom = s + L.act_mom + L.amax * a;
      int* momdof = si + L.act_momdof + L.amax * a;
      float* gm = d.actuator_moment + (long)wid * m.nJmom + rowadr;
      int* gc = d.moment_colind + (long)wid * m.nJmom + rowadr;
      float length = 0.0f;
      if (trn == TRN_BODY) {  // smooth.py:2597-2602: the contact sum (collision stage) over -ncon
        const int ncon = si[L.act_nnz + a];
        const float sc = ncon > 0 ? -1.0f / (float)ncon : 0.0f;
        for (int i = 0; i < my_nnz; i++) {
          const float v = ncon > 0 ? mom[i] * sc : 0.0f;
          mom[i] = v;
          momdof[i] = i;
          gm[i] = v;
          gc[i] = i;
        }
      } else {
        length = trn_site(m, wid, a, my_nnz, d.site_xpos + (long)wid * m.nsite * 3, d.site_xmat + (long)wid * m.nsite * 9, s + L.xquat,
                          s + L.subtree_com, s + L.cdof, mom, momdof, gm, gc);
      }
      for (int k = my_nnz; k < L.amax; k++) { mom[k] = 0.0f; momdof[k] = 0; }
      s[L.act_len + a] = length;
      si[L.act_nnz + a] = my_nnz;
      d.actuator_length[gu] = length;
      d.moment_rownnz[gu] = my_nnz;
      d.moment_rowadr[gu] = rowadr;
      continue;
    }
    int j = m.actuator_trnid[2 * a];
    int jt = m.jnt_type[j], qa = m.jnt_qposadr[j], va = m.jnt_dofadr[j];
    const float* qpos = s + L.qpos;
    float mom[6] = {0, 0, 0, 0, 0, 0};
    int nnz;
    float length;
    if (jt == JNT_FREE) {
      nnz = 6;
      length = 0.0f;
      if (trn == 1) {
        float q[4] = {qpos[qa + 3], qpos[qa + 4], qpos[qa + 5], qpos[qa + 6]}, qn[4], ga[3];
        normalize4(q);
        qn[0] = q[0]; qn[1] = -q[1]; qn[2] = -q[2]; qn[3] = -q[3];
        rot_vec_quat(ga, gear + 3, qn);
        for (int i = 0; i < 3; i++) { mom[i] = gear[i]; mom[3 + i] = ga[i]; }
      } else {
        for (int i = 0; i < 6; i++) mom[i] = gear[i];
      }
    } else if (jt == JNT_BALL) {
      nnz = 3;
      float q[4] = {qpos[qa], qpos[qa + 1], qpos[qa + 2], qpos[qa + 3]}, aa[3];
      normalize4(q);
      quat_to_vel(aa, q);
      float ga[3] = {gear[0], gear[1], gear[2]};
      if (trn == 1) {
        float qn[4] = {q[0], -q[1], -q[2], -q[3]};
        rot_vec_quat(ga, ga, qn);
      }
      length = dot3(aa, ga);
      for (int i = 0; i < 3; i++) mom[i] = ga[i];
    } else {
      nnz = 1;
      length = qpos[qa] * gear[0];
      mom[0] = gear[0];
    }
    s[L.act_len + a] = length;
    si[L.act_nnz + a] = nnz;
    long gu = (long)wid * m.nu + a;
    d.actuator_length[gu] = length;
    d.moment_rownnz[gu] = nnz;
    d.moment_rowadr[gu] = rowadr;
    for (int k = 0; k < L.amax; k++) {
      s[L.act_mom + L.amax * a + k] = k < nnz ? mom[k] : 0.0f;
      si[L.act_momdof + L.amax * a + k] = k < nnz ? va + k : 0;
    }
#pragma unroll
    for (int k = 0; k < 6; k++) {
      if (k < nnz) {
        d.actuator_moment[(long)wid * m.nJmom + rowadr + k] = mom[k];
        d.moment_colind[(long)wid * m.nJmom + rowadr + k] = va + k;
      }
    }
  }
  WSYNC();
}

// -------------------------------------------------------------------------------------------
// velocity (forward.py:592-613): actuator velocity, com_vel, passive, rne
// -------------------------------------------------------------------------------------------
// POS_LDS: the position stage ran in this launch, so the body / geom frames are in LDS (else they are read
// from the Data).  PARTS (the stage launches, sub_kernel): bit 0 actuator velocity + com_vel, bit 1 passive,
// bit 2 tendon bias + rne; the step runs all three
template <bool TEN, bool POS_LDS, int PARTS = 7>
__device__ __forceinline__ void fwd_velocity(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, WS& w) {
  const int wid = w.wid, lane = w.lane;
  float* s = w.s;
  int* si = w.si;
  const float* qvel = s + L.qvel;
  const float* qpos = s + L.qpos;
  const int nv = m.nv;
  float* cvel = s + L.cvel;
  float* cdof_dot = s + L.cdof_dot;
  float* cacc = s + L.cacc;
  const float* cd = s + L.cdof;
  float* spring = s + L.vec;
  float* damper = s + L.vec + nv;
  if constexpr ((PARTS & 1) != 0) {
  // forward.py:540-562
  for (int a = lane; a < m.nu; a += LPW) {
    float v = 0.0f;
    for (int k = 0; k < si[L.act_nnz + a]; k++) v += s[L.act_mom + L.amax * a + k] * qvel[si[L.act_momdof + L.amax * a + k]];
    s[L.act_vel + a] = v;
    d.actuator_velocity[(long)wid * m.nu + a] = v;
  }
  // smooth.py:1935-2038 com_vel.  Inside a body the joint loop adds cdof*qvel joint by joint
  // and takes cdof_dot = cvel_partial x cdof; the partial sum is split into the parent's cvel
  // (level pass, LDS only) and the body-local part (one pass over dofs in parallel).
  float* dv = s + L.cfrc;  // per-body local increments (cfrc is produced later)
  for (int b = lane; b < m.nbody; b += LPW) {
    float acc[6] = {0, 0, 0, 0, 0, 0};
    const int adr = m.body_dofadr[b], num = m.body_dofnum[b];
    for (int k = adr; k < adr + num; k++)
      for (int i = 0; i < 6; i++) acc[i] += cd[6 * k + i] * qvel[k];
    for (int i = 0; i < 6; i++) { dv[6 * b + i] = acc[i]; cvel[6 * b + i] = 0.0f; }
  }
  WSYNC();
  for (int b0 = 0; b0 < m.nbody; b0 += LPW) {
    const int b = b0 + lane;
    const bool ok = b > 0 && b < m.nbody;
    const int par = ok ? m.body_parentid[b] : 0, lv = ok ? m.body_level[b] : 0;
    for (int lvl = 1; lvl < m.nlevel; lvl++) {
      if (ok && lv == lvl)
        for (int i = 0; i < 6; i++) cvel[6 * b + i] = cvel[6 * par + i] + dv[6 * b + i];
      WSYNC();
    }
  }
  // cdof_dot per dof: (cvel[parent] + dofs of the body added before this joint) x cdof;
  // a free joint's rotational dofs also see its translational dofs, which get cdof_dot = 0
  for (int k = lane; k < nv; k += LPW) {
    const int b = m.dof_bodyid[k], j = m.dof_jntid[k], jt = m.jnt_type[j];
    const int ja = m.jnt_dofadr[j], p = m.body_parentid[b];
    float out[6] = {0, 0, 0, 0, 0, 0};
    if (!(jt == JNT_FREE && k < ja + 3)) {
      float cv[6];
      for (int i = 0; i < 6; i++) cv[i] = cvel[6 * p + i];
      const int end = jt == JNT_FREE ? ja + 3 : ja;
      for (int q = m.body_dofadr[b]; q < end; q++)
        for (int i = 0; i < 6; i++) cv[i] += cd[6 * q + i] * qvel[q];
      motion_cross(out, cv, cd + 6 * k);
    }
    for (int i = 0; i < 6; i++) cdof_dot[6 * k + i] = out[i];
  }
  WSYNC();
  for (int e = lane; e < m.nbody * 6; e += LPW) d.cvel[(long)wid * m.nbody * 6 + e] = cvel[e];
  for (int e = lane; e < nv * 6; e += LPW) d.cdof_dot[(long)wid * nv * 6 + e] = cdof_dot[e];
  }
  if constexpr ((PARTS & 2) != 0) {
  // passive.py:70-179, 535-563
  const int dsbl_spring = m.opt_disableflags & DSBL_SPRING, dsbl_damper = m.opt_disableflags & DSBL_DAMPER;
  float* qfrc_passive = s + L.qfrc_passive;
  for (int i = lane; i < nv; i += LPW) { spring[i] = 0.0f; damper[i] = 0.0f; }
  WSYNC();
  if (!(dsbl_spring && dsbl_damper)) {
    const float* jnt_stiffness = MR(jnt_stiffness);
    const float* dof_damping = MR(dof_damping);
    const float* qpos_spring = MR(qpos_spring);
    for (int j = lane; j < m.njnt; j += LPW) {
      int da = m.jnt_dofadr[j], qa = m.jnt_qposadr[j], jt = m.jnt_type[j];
      float stiff = jnt_stiffness[j], damp = dof_damping[da];
      bool hs = stiff != 0.0f && !dsbl_spring, hd = damp != 0.0f && !dsbl_damper;
      if (jt == JNT_FREE) {
        if (hs) {
          for (int i = 0; i < 3; i++) spring[da + i] = -stiff * (qpos[qa + i] - qpos_spring[qa + i]);
          float rot[4] = {qpos[qa + 3], qpos[qa + 4], qpos[qa + 5], qpos[qa + 6]}, dif[3];
          normalize4(rot);
          quat_sub(dif, rot, qpos_spring + qa + 3);
          for (int i = 0; i < 3; i++) spring[da + 3 + i] = -stiff * dif[i];
        }
        if (hd)
          for (int i = 0; i < 6; i++) damper[da + i] = -damp * qvel[da + i];
      } else if (jt == JNT_BALL) {
        if (hs) {
          float rot[4] = {qpos[qa], qpos[qa + 1], qpos[qa + 2], qpos[qa + 3]}, dif[3];
          normalize4(rot);
          quat_sub(dif, rot, qpos_spring + qa);
          for (int i = 0; i < 3; i++) spring[da + i] = -stiff * dif[i];
        }
        if (hd)
          for (int i = 0; i < 3; i++) damper[da + i] = -damp * qvel[da + i];
      } else {
        if (hs) spring[da] = -stiff * (qpos[qa] - qpos_spring[qa]);
        if (hd) damper[da] = -damp * qvel[da];
      }
    }
  }
  WSYNC();
  if (TEN && m.ntendon) tendon_passive(m, d, qpos, qvel, spring, damper, wid, lane);  // passive.py:183-252
  // passive.py:829-869: gravity compensation (unless gravity is off) and fluid forces, both body forces at
  // xipos mapped through the body Jacobian (mjw_passive.h); in the extended instantiation only.  The cacc /
  // cfrc LDS slots hold the two per-body wrenches (rne fills them afterwards).  nv <= 64: dof i is lane i.
  float gcomp = 0.0f, fluid = 0.0f;
  const bool gc_on = TEN && m.ngravcomp && !(m.opt_disableflags & DSBL_GRAVITY) && !(dsbl_spring && dsbl_damper);
  const bool fl_on = TEN && m.has_fluid && !(dsbl_spring && dsbl_damper);
  if (gc_on || fl_on) {
    float* Wg = s + L.cacc;
    float* Wf = s + L.cfrc;
    const float* xipos = s + L.xipos;
    const float* gxpos = POS_LDS ? s + L.gxpos : d.geom_xpos + (long)wid * m.ngeom * 3;
    const float* gxmat = POS_LDS ? s + L.gxmat : d.geom_xmat + (long)wid * m.ngeom * 9;
    const float zero3[3] = {0.0f, 0.0f, 0.0f};
    for (int b = lane; b < m.nbody; b += LPW) {
      const float* sr = s + L.subtree_com + 3 * m.body_rootid[b];
      float f[3], t[3];
      if (gc_on) {
        gravcomp_force(m, wid, b, f);
        body_wrench(Wg + 6 * b, f, zero3, xipos + 3 * b, sr);
      }
      if (fl_on) {
        float xm[9];
        if (POS_LDS) {  // the inertial frame as kinematics() computes it (its LDS copy is gone in direct mode)
          const float q[4] = {s[L.xquat + 4 * b], s[L.xquat + 4 * b + 1], s[L.xquat + 4 * b + 2], s[L.xquat + 4 * b + 3]};
          float qi[4];
          mul_quat(qi, q, MR(body_iquat) + 4 * b);
          quat_to_mat(xm, qi);
        } else {
          for (int k = 0; k < 9; k++) xm[k] = d.ximat[((long)wid * m.nbody + b) * 9 + k];
        }
        fluid_force(m, wid, b, xipos + 3 * b, xm, cvel + 6 * b, sr, gxpos, gxmat, f, t);
        body_wrench(Wf + 6 * b, f, t, xipos + 3 * b, sr);
      }
    }
    WSYNC();
    for (int i = lane; i < nv; i += LPW) {
      const float* cd = s + L.cdof + 6 * i;
      const int db = m.dof_bodyid[i], end = m.body_subtree_end[db];
      for (int b = db; b < end; b++) {
        if (gc_on) gcomp += cd[0] * Wg[6 * b] + cd[1] * Wg[6 * b + 1] + cd[2] * Wg[6 * b + 2] + cd[3] * Wg[6 * b + 3] + cd[4] * Wg[6 * b + 4] + cd[5] * Wg[6 * b + 5];
        if (fl_on) fluid += cd[0] * Wf[6 * b] + cd[1] * Wf[6 * b + 1] + cd[2] * Wf[6 * b + 2] + cd[3] * Wf[6 * b + 3] + cd[4] * Wf[6 * b + 4] + cd[5] * Wf[6 * b + 5];
      }
    }
    WSYNC();
  }
  for (int i = lane; i < nv; i += LPW) {
    float p = spring[i] + damper[i];
    // passive.py:555-561: gravcomp unless the joint routes it to the actuators, then the fluid force
    if (gc_on && !m.jnt_actgravcomp[m.dof_jntid[i]]) p += gcomp;
    if (fl_on) p += fluid;
    qfrc_passive[i] = p;
    long gi = (long)wid * nv + i;
    d.qfrc_spring[gi] = spring[i];
    d.qfrc_damper[gi] = damper[i];
    d.qfrc_gravcomp[gi] = gcomp;
    d.qfrc_fluid[gi] = fluid;
    d.qfrc_passive[gi] = p;
    if (TEN) spring[i] = gcomp;  // kept for the actuation stage of this launch (L.vec is free until the solver)
  }
  }
  if constexpr ((PARTS & 4) != 0) {
  // smooth.py:1878-1932 tendon_bias: armature J (Jdot qvel) of the spatial tendons, kept in damper[] (free
  // after the passive forces) until qfrc_bias is written; needs cvel before rne reuses its slot
  const bool ten_bias = TEN && m.nten_spatial;
  if (ten_bias) {
    const TenFrames f{d.site_xpos + (long)wid * m.nsite * 3, nullptr, nullptr, s + L.subtree_com, s + L.cdof};
    tendon_bias(m, d, wid, lane, qvel, f, cvel, cdof_dot, s + L.scratch, damper);
  }
  // rne (smooth.py:1112-1274, flg_acc = False): cacc[b] = cacc[parent] + sum cdof_dot qvel
  for (int b = lane; b < m.nbody; b += LPW) {
    float acc[6] = {0, 0, 0, 0, 0, 0};
    if (b == 0) {
      const float* grav = MR(opt_gravity);
      if (!(m.opt_disableflags & DSBL_GRAVITY))
        for (int i = 0; i < 3; i++) acc[3 + i] = -grav[i];
    } else {
      const int adr = m.body_dofadr[b], num = m.body_dofnum[b];
      for (int k = adr; k < adr + num; k++)
        for (int i = 0; i < 6; i++) acc[i] += cdof_dot[6 * k + i] * qvel[k];
    }
    for (int i = 0; i < 6; i++) cacc[6 * b + i] = acc[i];
  }
  WSYNC();
  for (int b0 = 0; b0 < m.nbody; b0 += LPW) {
    const int b = b0 + lane;
    const bool ok = b > 0 && b < m.nbody;
    const int par = ok ? m.body_parentid[b] : 0, lv = ok ? m.body_level[b] : 0;
    for (int lvl = 1; lvl < m.nlevel; lvl++) {
      if (ok && lv == lvl)
        for (int i = 0; i < 6; i++) cacc[6 * b + i] += cacc[6 * par + i];
      WSYNC();
    }
  }
  float* cfrc = s + L.cfrc;
  for (int b = lane; b < m.nbody; b += LPW) {
    float f[6] = {0, 0, 0, 0, 0, 0};
    if (b > 0) {
      float f1[6], iv[6], f2[6];
      inert_vec(f1, s + L.cinert + 10 * b, cacc + 6 * b);
      inert_vec(iv, s + L.cinert + 10 * b, cvel + 6 * b);
      motion_cross_force(f2, cvel + 6 * b, iv);
      for (int i = 0; i < 6; i++) f[i] = f1[i] + f2[i];
    }
    for (int i = 0; i < 6; i++) cfrc[6 * b + i] = f[i];
  }
  WSYNC();
  // backward accumulation = subtree sums; keep result in cvel-sized scratch (cfrc_int)
  for (int b = lane; b < m.nbody; b += LPW) {
    float acc[6] = {0, 0, 0, 0, 0, 0};
    int end = m.body_subtree_end[b];
    for (int j = (b == 0 ? 1 : b); j < end; j++)
      for (int i = 0; i < 6; i++) acc[i] += cfrc[6 * j + i];
    long gb = (long)wid * m.nbody + b;
    for (int i = 0; i < 6; i++) { d.cfrc_int[gb * 6 + i] = acc[i]; d.cacc[gb * 6 + i] = cacc[6 * b + i]; }
    // store back into cacc slot? no: qfrc_bias needs cfrc_int of dof bodies -> reuse cdof_dot-free scratch below
    for (int i = 0; i < 6; i++) s[L.cvel + 6 * b + i] = acc[i];  // cvel no longer needed after this point
  }
  WSYNC();
  for (int i = lane; i < nv; i += LPW) {
    int b = m.dof_bodyid[i];
    const float* cd = s + L.cdof + 6 * i;
    const float* ci = s + L.cvel + 6 * b;
    float v = cd[0] * ci[0] + cd[1] * ci[1] + cd[2] * ci[2] + cd[3] * ci[3] + cd[4] * ci[4] + cd[5] * ci[5];
    if (ten_bias) v += damper[i];
    s[L.qfrc_bias + i] = v;
    d.qfrc_bias[(long)wid * nv + i] = v;
  }
  WSYNC();
  }
}

// forward.py:616-927 (actuator force, qfrc_actuator); VEL_LDS: the velocity stage ran in this launch and
// left qfrc_gravcomp in L.vec (else it is read from the Data)
template <bool TEN, bool VEL_LDS>
__device__ __forceinline__ void fwd_actuation(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, WS& w) {
  const int wid = w.wid, lane = w.lane;
  float* s = w.s;
  int* si = w.si;
  const int nv = m.nv;
  float* qfrc_act = s + L.qfrc_actuator;
  if (!m.nu || (m.opt_disableflags & DSBL_ACTUATION)) {
    for (int i = lane; i < nv; i += LPW) { qfrc_act[i] = 0.0f; d.qfrc_actuator[(long)wid * nv + i] = 0.0f; }
    for (int a = lane; a < m.na; a += LPW) d.act_dot[(long)wid * m.na + a] = 0.0f;
    WSYNC();
    return;
  }
  const float* ctrlrange = MR(actuator_ctrlrange);
  const float* forcerange = MR(actuator_forcerange);
  const float* gainprm = MR(actuator_gainprm);
  const float* biasprm = MR(actuator_biasprm);
  const float* dynprm = MR(actuator_dynprm);
  for (int a = lane; a < m.nu; a += LPW) {
    float ctrl = d.ctrl[(long)wid * m.nu + a];
    if (m.actuator_ctrllimited[a] && !(m.opt_disableflags & DSBL_CLAMPCTRL))
      ctrl = clampf(ctrl, ctrlrange[2 * a], ctrlrange[2 * a + 1]);
    float ctrl_act = ctrl;
    int act_first = m.actuator_actadr[a];
    if (m.na && act_first >= 0) {
      int act_last = act_first + m.actuator_actnum[a] - 1;
      int dt = m.actuator_dyntype[a];
      float act = d.act[(long)wid * m.na + act_last];
      float act_dot = 0.0f;
      if (dt == DYN_INTEGRATOR) act_dot = ctrl;
      else if (dt == DYN_FILTER || dt == DYN_FILTEREXACT) act_dot = (ctrl - act) / fmaxf(dynprm[10 * a], MJW_MINVAL);
      else if (TEN && dt == DYN_MUSCLE) act_dot = muscle_dynamics(ctrl, act, dynprm + 10 * a);  // forward.py:671-674
      d.act_dot[(long)wid * m.na + act_last] = act_dot;
      // actearly (forward.py:682-697): the force sees the activation of the next step
      ctrl_act = m.actuator_actearly[a] ? next_act(MR(opt_timestep)[0], dt, dynprm[10 * a], MR(actuator_actrange) + 2 * a, act, act_dot, 1.0f,
                                                   m.actuator_actlimited[a] != 0)
                                        : act;
    }
    float len = s[L.act_len + a], vel = s[L.act_vel + a];
    const float* gp = gainprm + 10 * a;
    const float* bp = biasprm + 10 * a;
    float gain = 0.0f, bias = 0.0f;
    int gt = m.actuator_gaintype[a], bt = m.actuator_biastype[a];
    if (gt == 0) gain = gp[0];
    else if (gt == 1) gain = gp[0] + gp[1] * len + gp[2] * vel;
    if (bt == 1) bias = bp[0] + bp[1] * len + bp[2] * vel;
    if (TEN && (gt == GAIN_MUSCLE || bt == BIAS_MUSCLE)) {  // forward.py:711-727 (the extended instantiation)
      const float* lr = MR(actuator_lengthrange) + 2 * a;
      const float acc0 = MR(actuator_acc0)[a];
      if (gt == GAIN_MUSCLE) gain = muscle_gain(len, vel, lr, acc0, gp);
      if (bt == BIAS_MUSCLE) bias = muscle_bias(len, lr, acc0, bp);
    }
    float force = gain * ctrl_act + bias;
    if (m.actuator_forcelimited[a]) force = clampf(force, forcerange[2 * a], forcerange[2 * a + 1]);
    s[L.act_force + a] = force;
    d.actuator_force[(long)wid * m.nu + a] = force;
  }
  WSYNC();
  if (TEN && m.ntendon) {
    tendon_actuator_clamp(m, s + L.act_force, wid, lane);  // forward.py:739-779
    for (int a = lane; a < m.nu; a += LPW)
      if (m.actuator_trntype[a] == TRN_TENDON) d.actuator_force[(long)wid * m.nu + a] = s[L.act_force + a];
    WSYNC();
  }
  const float* jnt_actfrcrange = MR(jnt_actfrcrange);
  for (int i = lane; i < nv; i += LPW) {
    float q = 0.0f;
    for (int a = 0; a < m.nu; a++)
      for (int k = 0; k < si[L.act_nnz + a]; k++)
        if (si[L.act_momdof + L.amax * a + k] == i) q += s[L.act_mom + L.amax * a + k] * s[L.act_force + a];
    int j = m.dof_jntid[i];
    // forward.py:824-826: actuator-level gravity compensation
    if (TEN && m.ngravcomp && m.jnt_actgravcomp[j]) q += VEL_LDS ? s[L.vec + i] : d.qfrc_gravcomp[(long)wid * nv + i];
    if (m.jnt_actfrclimited[j]) q = clampf(q, jnt_actfrcrange[2 * j], jnt_actfrcrange[2 * j + 1]);
    qfrc_act[i] = q;
    d.qfrc_actuator[(long)wid * nv + i] = q;
  }
  WSYNC();
}

// forward.py:930-969 + support.py:174-237 (xfrc) + factor_solve_i (smooth.py:2860-2928)
__device__ __forceinline__ void fwd_acceleration(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, WS& w) {
  const int wid = w.wid, lane = w.lane;
  float* s = w.s;
  const int nv = m.nv, nvs = L.nvs;
  // xfrc_accumulate (support.py:174-237): the body force (f, t) applied at xipos maps to dof i as
  // jac(xipos)^T (f, t) = cdof_i . W_b with W_b = (t + off x f, f), off = xipos - subtree_com(root).
  // Summing W over the DFS subtree range [db, subtree_end) of the dof's body gives one 6-vector
  // dot per dof; the xfrc rows are read once, coalesced (cacc / cfrc LDS slots are dead here).
  float* Wb = s + L.cacc;
  float* Ws = s + L.cfrc;
  const float* xfrc = d.xfrc_applied + (long)wid * m.nbody * 6;
  for (int b = lane; b < m.nbody; b += LPW) {
    float f[3] = {xfrc[6 * b], xfrc[6 * b + 1], xfrc[6 * b + 2]}, off[3], c[3];
    for (int k = 0; k < 3; k++) off[k] = s[L.xipos + 3 * b + k] - s[L.subtree_com + 3 * m.body_rootid[b] + k];
    cross3(c, off, f);
    for (int k = 0; k < 3; k++) { Wb[6 * b + k] = xfrc[6 * b + 3 + k] + c[k]; Wb[6 * b + 3 + k] = f[k]; }
  }
  WSYNC();
  for (int b = lane; b < m.nbody; b += LPW) {
    float acc[6] = {0, 0, 0, 0, 0, 0};
    const int end = m.body_subtree_end[b];
    for (int j = b; j < end; j++)
      for (int k = 0; k < 6; k++) acc[k] += Wb[6 * j + k];
    for (int k = 0; k < 6; k++) Ws[6 * b + k] = acc[k];
  }
  WSYNC();
  float qs = 0.0f;
  if (lane < nv) {
    int i = lane;
    long gi = (long)wid * nv + i;
    qs = s[L.qfrc_passive + i] - s[L.qfrc_bias + i] + s[L.qfrc_actuator + i] + d.qfrc_applied[gi];
    const float* cd = s + L.cdof + 6 * i;
    const float* W = Ws + 6 * m.dof_bodyid[i];
    qs += cd[0] * W[0] + cd[1] * W[1] + cd[2] * W[2] + cd[3] * W[3] + cd[4] * W[4] + cd[5] * W[5];
    s[L.qfrc_smooth + i] = qs;
    d.qfrc_smooth[gi] = qs;
  }
  if (L.nofactor) return;  // the dense kernel factors qM (mjw_dense.h)
  // factor qM -> L (copy then in-place Cholesky)
  float* Lm = s + L.L;
  for (int e = lane; e < nv * nvs; e += LPW) Lm[e] = s[L.qM + e];
  WSYNC();
  cholesky(Lm, nv, nvs, lane);
  float qacc_smooth = cholesky_solve(Lm, nv, nvs, lane, qs);
  if (lane < nv) {
    s[L.qacc_smooth + lane] = qacc_smooth;
    d.qacc_smooth[(long)wid * nv + lane] = qacc_smooth;
  }
  float* gL = d.qLD + (long)wid * nv * nv;
  for (int e = lane; e < nv * nv; e += LPW) {
    int r = e / nv, c = e - r * nv;
    gL[e] = Lm[r * nvs + c];
  }
  WSYNC();
}

// -------------------------------------------------------------------------------------------
// solver.py: primal CG / Newton (pyramidal), per-world convergence loop
// -------------------------------------------------------------------------------------------
struct Vec3 {
  float c, g, h;
};

__device__ __forceinline__ void eval_row(float D, float jaref, float jv, float fl, int r, int ne, int nf, float alpha, Vec3& o) {
  float x = jaref + alpha * jv;
  if (r >= ne + nf) {
    if (x < 0.0f) { float jvD = jv * D; o.c += 0.5f * D * x * x; o.g += jvD * x; o.h += jv * jvD; }
    return;
  }
  if (r >= ne) {
    float rf = safe_div(fl, D);
    if ((-rf < x) && (x < rf)) { float jvD = jv * D; o.c += 0.5f * D * x * x; o.g += jvD * x; o.h += jv * jvD; }
    else if (x <= -rf) { o.c += fl * (-0.5f * rf - x); o.g += -fl * jv; }
    else { o.c += fl * (-0.5f * rf + x); o.g += fl * jv; }
    return;
  }
  float jvD = jv * D;
  o.c += 0.5f * D * x * x; o.g += jvD * x; o.h += jv * jvD;
}

__device__ __forceinline__ bool in_bracket(const Vec3& x, const Vec3& y) {
  return (x.g < y.g && y.g < 0.0f) || (x.g > y.g && y.g > 0.0f);
}

// update_constraint (solver.py:2154-2219): returns (cost, gauss); sets force/state; qfrc_constraint per lane
// elliptic rows of the generic solver (L.ecoef >= 0): row r is an elliptic contact row; its contact's first
// row and dimension (efc_margin slot), and whether all of the contact's rows fit in nefc
__device__ __forceinline__ bool ell_row(const Lay& L, const int* si, int r, int ne, int nf) {
  return L.ecoef >= 0 && r >= ne + nf && si[L.efc_type + r] == CNSTR_CONTACT_ELLIPTIC;
}
__device__ __forceinline__ void ell_extent(const Lay& L, const int* si, int r, int& r0, int& dim) {
  const int x = si[L.efc_margin + r];
  r0 = x & 0xffff;
  dim = x >> 16;
}

// one row's line-search terms at alpha, elliptic rows through their contact's cone at the first row
// (solver.py:263-323, the other rows of the contact add nothing)
__device__ __forceinline__ void eval_row_g(const Lay& L, const float* s, int rr, int nefc, int ne, int nf, float alpha, Vec3& o) {
  const int* si = reinterpret_cast<const int*>(s);
  if (ell_row(L, si, rr, ne, nf)) {
    int r0, dim;
    ell_extent(L, si, rr, r0, dim);
    if (rr != r0 || r0 + dim > nefc) return;
    const float* q = s + L.ecoef + EC_WORDS * rr;
    const Ell e = {q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7], q[8], q[9]};
    float c, g, hh;
    eval_elliptic(e, alpha, c, g, hh);
    o.c += c; o.g += g; o.h += hh;
    return;
  }
  eval_row(s[L.efc_D + rr], s[L.Jaref + rr], s[L.jv + rr], s[L.efc_frictionloss + rr], rr, ne, nf, alpha, o);
}

__device__ __forceinline__ void update_constraint(const Lay& L, float* s, int lane, int nv, int nvs, int nefc, int ne, int nf, float ma,
                                  float qfrc_smooth, float qacc, float qacc_smooth, float& cost, float& gauss, float& qfrc_c) {
  int* si = reinterpret_cast<int*>(s);
  float c = 0.0f;
  float* u = s + L.efc_vel;        // elliptic: u = Jaref * cone coefficient
  const float* ef = s + L.efc_pos;  // elliptic: cone coefficient
  if (L.ecoef >= 0) {
    for (int r = lane; r < nefc; r += LPW) u[r] = s[L.Jaref + r] * ef[r];
    WSYNC();
  }
  for (int r = lane; r < nefc; r += LPW) {
    float D = s[L.efc_D + r], Jaref = s[L.Jaref + r];
    float f;
    int st;
    if (ell_row(L, si, r, ne, nf)) {
      // elliptic cone zones (solver.py:1886-1942): N from the first row, T from the friction rows; a
      // contact cut by njmax contributes nothing
      int r0, dim;
      ell_extent(L, si, r, r0, dim);
      const float mu = ef[r0];
      f = 0.0f;
      st = STATE_SATISFIED;
      if (r0 + dim <= nefc) {
        float TT = 0.0f;
        for (int j = 1; j < dim; j++) TT += u[r0 + j] * u[r0 + j];
        const float N = u[r0];
        const float T = TT <= 0.0f ? 0.0f : sqrtf(TT);
        if (N >= mu * T || (T <= 0.0f && N >= 0.0f)) {
        } else if (mu * N + T <= 0.0f || (T <= 0.0f && N < 0.0f)) {
          f = -D * Jaref; st = STATE_QUADRATIC; c += 0.5f * D * Jaref * Jaref;
        } else {
          const float dm = safe_div(s[L.efc_D + r0], mu * mu * (1.0f + mu * mu));
          const float nmt = N - mu * T;
          const float f0 = -dm * nmt * mu;
          if (r == r0) { f = f0; c += 0.5f * dm * nmt * nmt; }
          else f = -safe_div(f0, T) * (u[r] * ef[r]);
          st = STATE_CONE;
        }
      }
    } else if (r < ne) { f = -D * Jaref; st = STATE_QUADRATIC; c += 0.5f * D * Jaref * Jaref; }
    else if (r < ne + nf) {
      float fl = s[L.efc_frictionloss + r], rf = safe_div(fl, D);
      if (Jaref <= -rf) { f = fl; st = STATE_LINEARNEG; c += -fl * (0.5f * rf + Jaref); }
      else if (Jaref >= rf) { f = -fl; st = STATE_LINEARPOS; c += -fl * (0.5f * rf - Jaref); }
      else { f = -D * Jaref; st = STATE_QUADRATIC; c += 0.5f * D * Jaref * Jaref; }
    } else {
      if (Jaref >= 0.0f) { f = 0.0f; st = STATE_SATISFIED; }
      else { f = -D * Jaref; st = STATE_QUADRATIC; c += 0.5f * D * Jaref * Jaref; }
    }
    s[L.efc_force + r] = f;
    si[L.efc_state + r] = st;
  }
  WSYNC();
  float q = 0.0f;
  if (lane < nv)
    for (int r = 0; r < nefc; r++) q += s[L.J + r * nvs + lane] * s[L.efc_force + r];
  qfrc_c = q;
  float gl = lane < nv ? (ma - qfrc_smooth) * (qacc - qacc_smooth) : 0.0f;
  float g = 0.5f * wave_sum(gl);
  gauss = g;
  cost = wave_sum(c) + g;
}

__device__ __forceinline__ void solve(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, WS& w) {
  const int wid = w.wid, lane = w.lane;
  float* s = w.s;
  int* si = w.si;
  const int nv = m.nv, nvs = L.nvs, njmax = d.njmax;
  const int nefc_all = si[L.iscratch + 62];
  const int nefc = min(nefc_all, njmax);
  const int ne = si[L.iscratch + 60], nf = si[L.iscratch + 61];
  const bool inl = lane < nv;
  float qfrc_smooth = inl ? s[L.qfrc_smooth + lane] : 0.0f;
  float qacc_smooth = inl ? s[L.qacc_smooth + lane] : 0.0f;
  long gi = (long)wid * nv + lane;
  if (njmax == 0 || nv == 0) {
    if (inl) d.qacc[gi] = qacc_smooth;
    if (lane == 0) d.solver_niter[wid] = 0;
    return;
  }
  const float* M = s + L.qM;
  const float* Lm = s + L.L;
  float* vec = s + L.vec;
  const float tolerance = MR(opt_tolerance)[0];
  const float ls_tolerance = MR(opt_ls_tolerance)[0];
  const float meaninertia = MR(stat_meaninertia)[0];
  const bool newton = m.opt_solver == SOLVER_NEWTON;
  // qacc init (solver.py:3308-3311)
  float qacc = 0.0f;
  if (inl) qacc = (m.opt_disableflags & DSBL_WARMSTART) ? qacc_smooth : d.qacc_warmstart[gi];
  // Jaref = J qacc - aref, Ma = M qacc
  if (inl) vec[lane] = qacc;
  WSYNC();
  for (int r = lane; r < nefc; r += LPW) {
    float acc = 0.0f;
    for (int k = 0; k < nv; k++) acc += s[L.J + r * nvs + k] * vec[k];
    s[L.Jaref + r] = acc - s[L.efc_aref + r];
  }
  float ma = 0.0f;
  if (inl)
    for (int k = 0; k < nv; k++) ma += M[lane * nvs + k] * vec[k];
  WSYNC();
  float cost = MJW_MAXVAL, prev_cost, gauss, qfrc_c;
  prev_cost = cost;
  update_constraint(L, s, lane, nv, nvs, nefc, ne, nf, ma, qfrc_smooth, qacc, qacc_smooth, cost, gauss, qfrc_c);
  float* H = s + L.H;
  // update_gradient (solver.py:2879-3008)
  auto update_gradient = [&](float& grad, float& Mgrad, float& grad_dot) {
    grad = inl ? ma - qfrc_smooth - qfrc_c : 0.0f;
    grad_dot = wave_sum(grad * grad);
    if (!newton) {
      Mgrad = cholesky_solve(Lm, nv, nvs, lane, grad);
    } else {
      // H = M + J' diag(D * QUADRATIC) J, Cholesky, solve
      float* C = s + L.econe;
      if (L.econe >= 0) {
        // cone-state contacts add J_c' C J_c (solver.py:2430-2585); C's row a, from u = Jaref * coefficient
        // of update_constraint, as in mjw_dense.h
        const float* u = s + L.efc_vel;
        const float* ef = s + L.efc_pos;
        for (int r = lane; r < nefc; r += LPW) {
          if (si[L.efc_state + r] != STATE_CONE) continue;
          int r0, dim;
          ell_extent(L, si, r, r0, dim);
          const int ea = r - r0;
          const float mu = ef[r0], mu2 = mu * mu;
          const float dm = safe_div(s[L.efc_D + r0], mu2 * (1.0f + mu2));
          const float n = u[r0];
          float tt = 0.0f;
          for (int j = 1; j < dim; j++) tt += u[r0 + j] * u[r0 + j];
          float t = tt <= 0.0f ? 0.0f : sqrtf(tt);
          t = fmaxf(t, MJW_MINVAL);
          const float ttt = fmaxf(t * t * t, MJW_MINVAL);
          const float mu_over_t = safe_div(mu, t), mu_n_over_ttt = mu * safe_div(n, ttt), diag = mu2 - mu * safe_div(n, t);
          const float ua = u[r];
          for (int k = 0; k < dim; k++) {
            const float ub = u[r0 + k];
            float hc;
            if (ea == 0 && k == 0) hc = 1.0f;
            else if (ea == 0) hc = -mu_over_t * ub;
            else if (k == 0) hc = -mu_over_t * ua;
            else hc = mu_n_over_ttt * ua * ub + (ea == k ? diag : 0.0f);
            C[6 * r + k] = hc * dm * ef[r] * ef[r0 + k];
          }
        }
        WSYNC();
      }
      if (inl)
        for (int k = 0; k < nv; k++) {
          float h = M[lane * nvs + k];
          for (int r = 0; r < nefc; r++) {
            const int st = si[L.efc_state + r];
            if (st == STATE_QUADRATIC) {
              h += s[L.efc_D + r] * s[L.J + r * nvs + lane] * s[L.J + r * nvs + k];
            } else if (L.econe >= 0 && st == STATE_CONE) {
              int r0, dim;
              ell_extent(L, si, r, r0, dim);
              float w = 0.0f;
              for (int b = 0; b < dim; b++) w += C[6 * r + b] * s[L.J + (r0 + b) * nvs + k];
              h += s[L.J + r * nvs + lane] * w;
            }
          }
          H[lane * nvs + k] = h;
        }
      WSYNC();
      cholesky(H, nv, nvs, lane);
      Mgrad = cholesky_solve(H, nv, nvs, lane, grad);
    }
  };
  float grad, Mgrad, grad_dot;
  update_gradient(grad, Mgrad, grad_dot);
  float search = -Mgrad;
  float search_dot = wave_sum(search * search);
  int niter = 0;
  const float scale = 1.0f / (meaninertia * (float)nv);
  if (m.opt_iterations != 0) {
    bool done = false;
    while (!done) {
      // ---- linesearch (solver.py:886-1341, 1662-1703)
      if (inl) vec[lane] = search;
      WSYNC();
      float mv = 0.0f;
      if (inl)
        for (int k = 0; k < nv; k++) mv += M[lane * nvs + k] * vec[k];
      const int r = lane;  // row per lane (njmax <= 64 handled below by rows loop)
      for (int rr = lane; rr < nefc; rr += LPW) {
        float acc = 0.0f;
        for (int k = 0; k < nv; k++) acc += s[L.J + rr * nvs + k] * vec[k];
        s[L.jv + rr] = acc;
      }
      WSYNC();
      (void)r;
      if (L.ecoef >= 0) {
        // per-contact quad / quad1 / quad2 at the first row, once per line search (solver.py:1550-1611)
        for (int rr = lane; rr < nefc; rr += LPW) {
          if (!ell_row(L, si, rr, ne, nf)) continue;
          int r0, dim;
          ell_extent(L, si, rr, r0, dim);
          if (rr != r0 || r0 + dim > nefc) continue;
          const float D0 = s[L.efc_D + rr], ja = s[L.Jaref + rr], jv0 = s[L.jv + rr], mu = s[L.efc_pos + rr];
          float q0 = 0.5f * ja * ja * D0, q1 = jv0 * ja * D0, q2 = 0.5f * jv0 * jv0 * D0;
          float uu = 0.0f, uv = 0.0f, vv = 0.0f;
          for (int j = 1; j < dim; j++) {
            const int rj = rr + j;
            const float jaj = s[L.Jaref + rj], jvj = s[L.jv + rj], dj = s[L.efc_D + rj], fj = s[L.efc_pos + rj], DJj = dj * jaj;
            q0 += 0.5f * jaj * DJj; q1 += jvj * DJj; q2 += 0.5f * jvj * dj * jvj;
            const float uj = jaj * fj, vj = jvj * fj;
            uu += uj * uj; uv += uj * vj; vv += vj * vj;
          }
          float* e = s + L.ecoef + EC_WORDS * rr;
          e[0] = q0; e[1] = q1; e[2] = q2; e[3] = ja * mu; e[4] = jv0 * mu;
          e[5] = uu; e[6] = uv; e[7] = vv; e[8] = D0 / (mu * mu * (1.0f + mu * mu)); e[9] = mu;
        }
        WSYNC();
      }
      float snorm = sqrtf(search_dot);
      float gtol = fmaxf(tolerance * ls_tolerance * snorm * meaninertia * (float)nv, 1e-6f);
      // quad_gauss
      float q1 = wave_sum(inl ? search * (ma - qfrc_smooth) : 0.0f);
      float q2 = wave_sum(inl ? 0.5f * search * mv : 0.0f);
      float qg0 = gauss;
      auto eval_all = [&](float alpha) {
        Vec3 o = {0.0f, 0.0f, 0.0f};
        for (int rr = lane; rr < nefc; rr += LPW) eval_row_g(L, s, rr, nefc, ne, nf, alpha, o);
        o.c = wave_sum(o.c); o.g = wave_sum(o.g); o.h = wave_sum(o.h);
        return o;
      };
      float alpha;
      Vec3 p0 = {0.0f, 0.0f, 0.0f}, lo_in = {0.0f, 0.0f, 0.0f};
      float lo_alpha_in = 0.0f;
      bool initial_converged = false;
      if (m.opt_ls_parallel) {
        // solver.py:325-478 parallel linesearch: the cheapest of ls_iterations log-spaced step sizes
        alpha = 0.0f;
        float best = MJW_MAXVAL;
        for (int i = 0; i < m.opt_ls_iterations; i++) {
          const float al = ls_parallel_alpha(MR(opt_ls_parallel_min_step)[0], m.opt_ls_iterations, i);
          const float cst = eval_all(al).c + al * al * q2 + al * q1 + qg0;
          if (cst < best) { best = cst; alpha = al; }
        }
        initial_converged = true;  // skip the iterative search below
        lo_alpha_in = alpha;
      } else {
        p0 = eval_all(0.0f);
        p0.c += qg0; p0.g += q1; p0.h += 2.0f * q2;
        lo_alpha_in = -safe_div(p0.g, p0.h);
        lo_in = eval_all(lo_alpha_in);
        lo_in.c += lo_alpha_in * lo_alpha_in * q2 + lo_alpha_in * q1 + qg0;
        lo_in.g += 2.0f * lo_alpha_in * q2 + q1;
        lo_in.h += 2.0f * q2;
        initial_converged = fabsf(lo_in.g) < gtol && lo_in.c < p0.c;
      }
      if (!initial_converged) {
        alpha = 0.0f;
        bool lo_less = lo_in.g < p0.g;
        Vec3 lo = lo_less ? lo_in : p0;
        float lo_alpha = lo_less ? lo_alpha_in : 0.0f;
        Vec3 hi = lo_less ? p0 : lo_in;
        float hi_alpha = lo_less ? 0.0f : lo_alpha_in;
        for (int it = 0; it < m.opt_ls_iterations; it++) {
          float lo_next_alpha = lo_alpha - safe_div(lo.g, lo.h);
          float hi_next_alpha = hi_alpha - safe_div(hi.g, hi.h);
          float mid_alpha = 0.5f * (lo_alpha + hi_alpha);
          Vec3 ln = {0.0f, 0.0f, 0.0f}, hn = {0.0f, 0.0f, 0.0f}, md = {0.0f, 0.0f, 0.0f};
          for (int rr = lane; rr < nefc; rr += LPW) {
            eval_row_g(L, s, rr, nefc, ne, nf, lo_next_alpha, ln);
            eval_row_g(L, s, rr, nefc, ne, nf, hi_next_alpha, hn);
            eval_row_g(L, s, rr, nefc, ne, nf, mid_alpha, md);
          }
          ln.c = wave_sum(ln.c); ln.g = wave_sum(ln.g); ln.h = wave_sum(ln.h);
          hn.c = wave_sum(hn.c); hn.g = wave_sum(hn.g); hn.h = wave_sum(hn.h);
          md.c = wave_sum(md.c); md.g = wave_sum(md.g); md.h = wave_sum(md.h);
          ln.c += lo_next_alpha * lo_next_alpha * q2 + lo_next_alpha * q1 + qg0; ln.g += 2.0f * lo_next_alpha * q2 + q1; ln.h += 2.0f * q2;
          hn.c += hi_next_alpha * hi_next_alpha * q2 + hi_next_alpha * q1 + qg0; hn.g += 2.0f * hi_next_alpha * q2 + q1; hn.h += 2.0f * q2;
          md.c += mid_alpha * mid_alpha * q2 + mid_alpha * q1 + qg0; md.g += 2.0f * mid_alpha * q2 + q1; md.h += 2.0f * q2;
          bool s1 = in_bracket(lo, ln);
          if (s1) { lo = ln; lo_alpha = lo_next_alpha; }
          bool s2 = in_bracket(lo, md);
          if (s2) { lo = md; lo_alpha = mid_alpha; }
          bool s3 = in_bracket(lo, hn);
          if (s3) { lo = hn; lo_alpha = hi_next_alpha; }
          bool swap_lo = s1 || s2 || s3;
          bool h1 = in_bracket(hi, hn);
          if (h1) { hi = hn; hi_alpha = hi_next_alpha; }
          bool h2 = in_bracket(hi, md);
          if (h2) { hi = md; hi_alpha = mid_alpha; }
          bool h3 = in_bracket(hi, ln);
          if (h3) { hi = ln; hi_alpha = lo_next_alpha; }
          bool swap_hi = h1 || h2 || h3;
          bool ls_done = (!swap_lo && !swap_hi) || (lo.g < 0.0f && lo.g > -gtol) || (hi.g > 0.0f && hi.g < gtol);
          bool improved = lo.c < p0.c || hi.c < p0.c;
          bool lo_better = lo.c < hi.c;
          if (improved && lo_better) alpha = lo_alpha;
          if (improved && !lo_better) alpha = hi_alpha;
          if (ls_done) break;
        }
      } else {
        alpha = lo_alpha_in;
      }
      qacc += alpha * search;
      ma += alpha * mv;
      for (int rr = lane; rr < nefc; rr += LPW) s[L.Jaref + rr] += alpha * s[L.jv + rr];
      WSYNC();
      // ---- CG bookkeeping, update constraint + gradient (solver.py:3187-3254)
      float prev_grad = grad, prev_Mgrad = Mgrad;
      prev_cost = cost;
      update_constraint(L, s, lane, nv, nvs, nefc, ne, nf, ma, qfrc_smooth, qacc, qacc_smooth, cost, gauss, qfrc_c);
      update_gradient(grad, Mgrad, grad_dot);
      float beta = 0.0f;
      if (!newton) {
        float num = wave_sum(inl ? grad * (Mgrad - prev_Mgrad) : 0.0f);
        float den = wave_sum(inl ? prev_grad * prev_Mgrad : 0.0f);
        beta = fmaxf(0.0f, num / fmaxf(MJW_MINVAL, den));
      }
      search = inl ? (-Mgrad + (newton ? 0.0f : beta * search)) : 0.0f;
      search_dot = wave_sum(search * search);
      niter++;
      float improvement = (prev_cost - cost) * scale;
      float gradient = sqrtf(grad_dot) * scale;
      done = (improvement < tolerance) || (gradient < tolerance) || niter == m.opt_iterations;
    }
  }
  // outputs
  if (inl) {
    s[L.qacc + lane] = qacc;
    s[L.Ma + lane] = ma;
    d.qacc[gi] = qacc;
    d.efc_Ma[gi] = ma;
    d.qfrc_constraint[gi] = qfrc_c;
  }
  for (int rr = lane; rr < nefc; rr += LPW) {
    d.efc_force[(long)wid * njmax + rr] = s[L.efc_force + rr];
    d.efc_state[(long)wid * d.njmax_pad + rr] = si[L.efc_state + rr];
  }
  if (lane == 0) d.solver_niter[wid] = niter;
  WSYNC();
}

// forward.py:51-354 (_advance + euler; implicit damping when EULERDAMP is enabled) and implicitfast
// (forward.py:494-510: (M - dt qDeriv) qacc_adv = M qacc, qDeriv = sum_a vel_a m_a m_a' - diag(damping)
// - tendon damping, on the ancestor pattern of qM; derivative.py:320-416), as in the dense kernel
__device__ __forceinline__ void euler(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, WS& w) {
  const int wid = w.wid, lane = w.lane;
  float* s = w.s;
  const int nv = m.nv, nvs = L.nvs;
  const float dt = MR(opt_timestep)[0];
  float qacc = lane < nv ? s[L.qacc + lane] : 0.0f;
  float qacc_adv = qacc;
  const int fl = m.opt_disableflags;
  const bool implicitfast = m.opt_integrator == INT_IMPLICITFAST;
  const bool need_implicit = implicitfast ? (fl & (DSBL_ACTUATION | DSBL_SPRING | DSBL_DAMPER)) != (DSBL_ACTUATION | DSBL_SPRING | DSBL_DAMPER)
                                          : !(fl & (DSBL_EULERDAMP | DSBL_DAMPER));
  if (need_implicit) {
    const float* dof_damping = MR(dof_damping);
    const bool damp = !(fl & DSBL_DAMPER);
    float* Lm = s + L.L;
    for (int e = lane; e < nv * nvs; e += LPW) {
      int r = e / nvs, c = e - r * nvs;
      Lm[e] = s[L.qM + e] + ((damp && r == c && r < nv) ? dt * dof_damping[r] : 0.0f);
    }
    WSYNC();
    if (implicitfast && m.nu > 0 && !(fl & DSBL_ACTUATION)) {
      for (int u = 0; u < m.nu; u++) {
        const float vel = actuator_vel_deriv(m, d, wid, u);
        if (vel == 0.0f) continue;
        const long gu = (long)wid * m.nu + u;
        const int nnz = d.moment_rownnz[gu], adr = d.moment_rowadr[gu];
        const long base = (long)wid * m.nJmom + adr;
        for (int p = lane; p < nnz * nnz; p += LPW) {
          const int k1 = p / nnz, k2 = p - k1 * nnz;
          const int i = d.moment_colind[base + k1], j = d.moment_colind[base + k2];
          int a = i;
          while (a > j) a = m.dof_parentid[a];
          if (a != j) continue;
          const float v = dt * vel * d.actuator_moment[base + k1] * d.actuator_moment[base + k2];
          Lm[i * nvs + j] -= v;
          if (i != j) Lm[j * nvs + i] -= v;
        }
        WSYNC();
      }
    }
    if (implicitfast && m.ntendon && !(fl & DSBL_DAMPER)) {
      const float* tdamp = MR(tendon_damping);
      for (int t = 0; t < m.ntendon; t++) {
        if (tdamp[t] == 0.0f) continue;
        const int rn = m.ten_J_rownnz[t], ra = m.ten_J_rowadr[t];
        for (int p = lane; p < rn * rn; p += LPW) {
          const int k1 = p / rn, k2 = p - k1 * rn;
          if (k2 > k1) continue;
          const int i = m.ten_J_colind[ra + k1], j = m.ten_J_colind[ra + k2];
          int a = i;
          while (a > j) a = m.dof_parentid[a];
          if (a != j) continue;
          const float v = dt * tdamp[t] * ten_coef(m, d, wid, t, i) * ten_coef(m, d, wid, t, j);
          Lm[i * nvs + j] += v;
          if (i != j) Lm[j * nvs + i] += v;
        }
        WSYNC();
      }
    }
    cholesky(Lm, nv, nvs, lane);
    qacc_adv = cholesky_solve(Lm, nv, nvs, lane, lane < nv ? s[L.Ma + lane] : 0.0f);
  }
  // activations (forward.py:132-168)
  const float* actrange = MR(actuator_actrange);
  for (int a = lane; a < m.nu; a += LPW) {
    int adr = m.actuator_actadr[a];
    for (int j = adr; adr >= 0 && j < adr + m.actuator_actnum[a]; j++) {
      long ga = (long)wid * m.na + j;
      d.act[ga] = next_act(dt, m.actuator_dyntype[a], MR(actuator_dynprm)[10 * a], actrange + 2 * a, d.act[ga], d.act_dot[ga], 1.0f,
                           m.actuator_actlimited[a] != 0);
    }
  }
  float* qvel = s + L.qvel;
  if (lane < nv) {
    float v = qvel[lane] + qacc_adv * dt;
    qvel[lane] = v;
    d.qvel[(long)wid * nv + lane] = v;
    d.qacc_warmstart[(long)wid * nv + lane] = qacc;
  }
  WSYNC();
  for (int j = lane; j < m.njnt; j += LPW) {
    int qa = m.jnt_qposadr[j], da = m.jnt_dofadr[j], jt = m.jnt_type[j];
    float* gq = d.qpos + (long)wid * m.nq;
    const float* qpos = s + L.qpos;
    if (jt == JNT_FREE) {
      for (int i = 0; i < 3; i++) gq[qa + i] = qpos[qa + i] + dt * qvel[da + i];
      float qn[4];
      quat_integrate(qn, qpos + qa + 3, qvel + da + 3, dt);
      for (int i = 0; i < 4; i++) gq[qa + 3 + i] = qn[i];
    } else if (jt == JNT_BALL) {
      float qn[4];
      quat_integrate(qn, qpos + qa, qvel + da, dt);
      for (int i = 0; i < 4; i++) gq[qa + i] = qn[i];
    } else {
      gq[qa] = qpos[qa] + dt * qvel[da];
    }
  }
  if (lane == 0) d.time[wid] = d.time[wid] + dt;
}

// -------------------------------------------------------------------------------------------
// input loaders for stage kernels that do not start at fwd_position
// -------------------------------------------------------------------------------------------
__device__ __forceinline__ void load_state(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, WS& w) {
  const int wid = w.wid, lane = w.lane;
  for (int i = lane; i < m.nq; i += LPW) w.s[L.qpos + i] = d.qpos[(long)wid * m.nq + i];
  for (int i = lane; i < m.nv; i += LPW) w.s[L.qvel + i] = d.qvel[(long)wid * m.nv + i];
}

__device__ __forceinline__ void load_smooth(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, WS& w, int stages) {
  const int wid = w.wid, lane = w.lane;
  float* s = w.s;
  int* si = w.si;
  const int nv = m.nv, nvs = L.nvs, np = m.nv_pad;
  // only inputs whose producing stage is not part of this launch
  if ((stages & (ST_VEL | ST_ACC)) && !(stages & ST_POS)) {
    for (int e = lane; e < nv * 6; e += LPW) s[L.cdof + e] = d.cdof[(long)wid * nv * 6 + e];
    for (int e = lane; e < m.nbody * 10; e += LPW) s[L.cinert + e] = d.cinert[(long)wid * m.nbody * 10 + e];
    for (int e = lane; e < m.nbody * 3; e += LPW) {
      s[L.xipos + e] = d.xipos[(long)wid * m.nbody * 3 + e];
      s[L.subtree_com + e] = d.subtree_com[(long)wid * m.nbody * 3 + e];
    }
  }
  if ((stages & (ST_VEL | ST_ACT)) && !(stages & ST_POS)) {
    for (int a = lane; a < m.nu; a += LPW) {
      long gu = (long)wid * m.nu + a;
      int nnz = d.moment_rownnz[gu], adr = d.moment_rowadr[gu];
      si[L.act_nnz + a] = nnz;
      for (int k = 0; k < L.amax; k++) {
        s[L.act_mom + L.amax * a + k] = k < nnz ? d.actuator_moment[(long)wid * m.nJmom + adr + k] : 0.0f;
        si[L.act_momdof + L.amax * a + k] = k < nnz ? d.moment_colind[(long)wid * m.nJmom + adr + k] : 0;
      }
      s[L.act_len + a] = d.actuator_length[gu];
      if (!(stages & ST_VEL)) s[L.act_vel + a] = d.actuator_velocity[gu];
    }
  }
  if ((stages & (ST_ACC | ST_SOLVE | ST_EULER)) && !(stages & ST_POS) && !(stages & ST_NOFACTOR)) {
    for (int e = lane; e < nv * nvs; e += LPW) {
      int r = e / nvs, c = e - r * nvs;
      s[L.qM + e] = c < nv ? d.qM[(long)wid * np * np + r * np + c] : 0.0f;
    }
  }
  if ((stages & ST_ACC) && !(stages & ST_VEL)) {
    for (int i = lane; i < nv; i += LPW) {
      long gi = (long)wid * nv + i;
      s[L.qfrc_passive + i] = d.qfrc_passive[gi];
      s[L.qfrc_bias + i] = d.qfrc_bias[gi];
    }
  }
  if ((stages & ST_ACC) && !(stages & ST_ACT)) {
    for (int i = lane; i < nv; i += LPW) s[L.qfrc_actuator + i] = d.qfrc_actuator[(long)wid * nv + i];
  }
  if ((stages & ST_SOLVE) && !(stages & ST_ACC)) {
    for (int e = lane; e < nv * nvs; e += LPW) {
      int r = e / nvs, c = e - r * nvs;
      s[L.L + e] = (c < nv) ? d.qLD[(long)wid * nv * nv + r * nv + c] : 0.0f;
    }
    for (int i = lane; i < nv; i += LPW) {
      long gi = (long)wid * nv + i;
      s[L.qfrc_smooth + i] = d.qfrc_smooth[gi];
      s[L.qacc_smooth + i] = d.qacc_smooth[gi];
    }
  }
  if ((stages & ST_SOLVE) && !(stages & ST_POS)) {
    int nefc = d.nefc[wid];
    int nrows = min(nefc, d.njmax);
    for (int e = lane; e < nrows * nvs; e += LPW) {
      int r = e / nvs, c = e - r * nvs;
      s[L.J + e] = c < nv ? d.efc_J[(long)wid * d.njmax_pad * np + r * np + c] : 0.0f;
    }
    for (int r = lane; r < nrows; r += LPW) {
      long gr = (long)wid * d.njmax + r;
      s[L.efc_D + r] = d.efc_D[(long)wid * d.njmax_pad + r];
      s[L.efc_aref + r] = d.efc_aref[gr];
      s[L.efc_frictionloss + r] = d.efc_frictionloss[gr];
    }
    if (lane == 0) {
      si[L.iscratch + 60] = d.ne[wid];
      si[L.iscratch + 61] = d.nf[wid];
      si[L.iscratch + 62] = nefc;
    }
    if (L.ecoef >= 0) {
      // elliptic rows (the position stage ran in an earlier launch): each row's contact extent from the
      // run of equal efc_id behind it, its cone coefficient from the contact (constraint.py:2151-2195)
      for (int r = lane; r < nrows; r += LPW) {
        const long gr = (long)wid * d.njmax + r;
        const int typ = d.efc_type[gr];
        si[L.efc_type + r] = typ;
        if (typ != CNSTR_CONTACT_ELLIPTIC) continue;
        const int cid = d.efc_id[gr];
        int r0 = r;
        while (r0 > 0 && d.efc_type[gr - (r - r0) - 1] == CNSTR_CONTACT_ELLIPTIC && d.efc_id[gr - (r - r0) - 1] == cid) r0--;
        const float* fr = d.contact_friction + 5L * cid;
        const int k = r - r0;
        s[L.efc_pos + r] = k == 0 ? fr[0] * MR(opt_impratio_invsqrt)[0] : fr[k - 1];
        si[L.efc_margin + r] = r0 | (d.contact_dim[cid] << 16);
      }
    }
  }
  if ((stages & ST_EULER) && !(stages & ST_SOLVE)) {
    for (int i = lane; i < nv; i += LPW) {
      long gi = (long)wid * nv + i;
      s[L.qacc + i] = d.qacc[gi];
      s[L.Ma + i] = d.efc_Ma[gi];
    }
  }
  WSYNC();
}

// the stages in STAGES of world w.wid by the calling wavefront
// BOX: the box narrowphase paths; TEN: the tendon paths.  The lean instantiations keep the
// humanoid-class kernel (neither) and the box models' kernel (no tendons) free of the register
// pressure of code they never run.
// the forward kernel's arguments (mjw_kernel's parameter list), re-read per stage through fresh_args
struct FwdArgs {
  mjw_model_t m;
  mjw_data_t d;
  Lay L;
  int w0;
};
#define FA (fresh_args<FwdArgs>())

template <int STAGES, bool BOX, bool TEN>
__device__ __forceinline__ void run_stages(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, WS& w) {
  PROF_T0();
  load_state(FA.m, FA.d, FA.L, w);
  load_smooth(FA.m, FA.d, FA.L, w, STAGES);
  WSYNC();
  PROF_MARK(PH_LOAD);
  if (STAGES & ST_POS) {
    kinematics(FA.m, FA.d, FA.L, w);
    PROF_MARK(PH_KIN);
    com_pos(FA.m, FA.d, FA.L, w);
    PROF_MARK(PH_COM);
    camlight(FA.m, FA.d, FA.L, w);
    PROF_MARK(PH_CAM);
    if (TEN && m.ntendon) {  // smooth.py:3085-3465 (fwd_position: before crb)
      const TenFrames f{d.site_xpos + (long)w.wid * m.nsite * 3, w.s + L.gxpos, w.s + L.gxmat, w.s + L.subtree_com, w.s + L.cdof};
      tendon_pos(m, d, w.s + L.qpos, f, w.wid, w.lane);
      WSYNC();  // spatial rows are read back by other lanes from here on
    }
    crb_qM<TEN>(FA.m, FA.d, FA.L, w);
    PROF_MARK(PH_CRB);
    if (TEN && m.nbodytrn) {  // BODY transmissions accumulate over the contacts as they are staged
      body_trn_init(m, w.s + L.act_mom, w.si + L.act_nnz, L.amax, w.lane);
      WSYNC();
    }
    collision_and_constraints<BOX, TEN, (STAGES & ST_POOL) != 0>(FA.m, FA.d, FA.L, w);
    PROF_MARK(PH_COLL);
    transmission<TEN>(FA.m, FA.d, FA.L, w);
    PROF_MARK(PH_TRN);
  }
  if (STAGES & ST_VEL) fwd_velocity<TEN, (STAGES & ST_POS) != 0>(FA.m, FA.d, FA.L, w);
  if ((STAGES & ST_POS) && (STAGES & ST_VEL) && w.lane < 2 && !(m.opt_enableflags & ENBL_ENERGY))
    d.energy[(long)w.wid * 2 + w.lane] = 0.0f;
  PROF_MARK(PH_VEL);
  if (STAGES & ST_ACT) fwd_actuation<TEN, (STAGES & ST_VEL) != 0>(FA.m, FA.d, FA.L, w);
  PROF_MARK(PH_ACT);
  if (STAGES & ST_ACC) fwd_acceleration(FA.m, FA.d, FA.L, w);
  PROF_MARK(PH_ACC);
  if (STAGES & ST_SOLVE) solve(FA.m, FA.d, FA.L, w);
  PROF_MARK(PH_GSOLVE);
  if (STAGES & ST_EULER) euler(FA.m, FA.d, FA.L, w);
  PROF_MARK(PH_GEULER);
}

// 4 waves per SIMD (<= 128 VGPRs): with the direct-mode LDS layout (9.8 KB per humanoid world)
// this is 16 worlds per CU; the collision narrowphase spills ~40 registers to scratch for it
// (measured: forward kernel 0.326 -> 0.303 ms at nworld 8192 against the unconstrained 160 VGPRs)
// The cap applies to the direct-mode (ST_NOFACTOR) instantiations the dense path launches and to the
// single-stage ones; the generic kernels that factor and solve in-kernel (nv 33-64 or njmax > 64) keep
// their registers (at the cap they spilled 80 B/lane).
template <int STAGES>
constexpr int fwd_waves_per_eu() { return ((STAGES & ST_SOLVE) && !(STAGES & ST_NOFACTOR)) ? 1 : 4; }
template <int STAGES, bool BOX = true, bool TEN = true>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(fwd_waves_per_eu<STAGES>()))) mjw_kernel(const mjw_model_t m, const mjw_data_t d, const Lay L, int w0) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  WS w;
  w.s = smem;
  w.si = reinterpret_cast<int*>(smem);
  w.wid = w0 + (int)blockIdx.x;
  w.lane = lane_id();
  if (w.wid >= d.nworld) return;
  WLOG_T0();
  run_stages<STAGES, BOX, TEN>(m, d, L, w);
  WLOG_END(w.wid, 0);
}

// One wave runs the whole step of one world: the forward stages (direct mode, run_stages) and then,
// in the same LDS, the dense factor / CG-or-Newton solve / Euler of mjw_dense.h.  No kernel boundary
// between the two halves, so the forward kernel's tail and the dense kernel's ramp-up do not serialise
// and a world's qM / J hand-off is read back while still L2-resident.  4 waves / SIMD: the forward half
// needs 113 VGPRs, the dense half (NB <= 28, CG) 128.  Launched for the full step when neither sensors
// nor an implicit integration split the dense work (run(); MJW_FUSED=0 keeps the two kernels).
template <int STAGES, bool BOX, int FLAGS, bool NEWTON, int NB>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) step_kernel(const mjw_model_t m, const mjw_data_t d, const Lay L, int w0) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = w0 + (int)blockIdx.x;
  if (b >= d.nworld) return;
  WS w;
  w.s = smem;
  w.si = reinterpret_cast<int*>(smem);
  // the longest-first order of the previous step's solve (a permutation) when the step built it
  w.wid = d.sched ? d.world_order[b] : b;
  w.lane = lane_id();
  run_stages<STAGES, BOX, false>(m, d, L, w);
  __syncthreads();  // the forward outputs (global) and the LDS are the dense half's from here
  dense_world<FLAGS, NEWTON, false, NB>(m, d, w.wid, smem);
}

// -------------------------------------------------------------------------------------------
// stage launches (the reference's finer stage functions, mujoco_warp/__init__.py:26-112): one stage of one
// world per wave, its inputs the Data fields the earlier stages wrote (an edit a caller made to them is what
// the stage reads, as in the reference), its outputs written to the Data.  Dense-path models only.
// -------------------------------------------------------------------------------------------
// the position-stage LDS state (frames, com / inertia, cdof, crb, qM) of world w.wid from the Data
__device__ __forceinline__ void load_pos_fields(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, WS& w) {
  const int wid = w.wid, lane = w.lane;
  float* s = w.s;
  const long nb = m.nbody, ng = m.ngeom, nj = m.njnt, nv = m.nv;
  auto cp = [&](int off, const float* src, long n) {
    for (long e = lane; e < n; e += LPW) s[off + e] = src[e];
  };
  cp(L.xpos, d.xpos + wid * nb * 3, nb * 3);
  cp(L.xquat, d.xquat + wid * nb * 4, nb * 4);
  cp(L.xmat, d.xmat + wid * nb * 9, nb * 9);
  cp(L.xipos, d.xipos + wid * nb * 3, nb * 3);
  cp(L.ximat, d.ximat + wid * nb * 9, nb * 9);
  cp(L.xanchor, d.xanchor + wid * nj * 3, nj * 3);
  cp(L.xaxis, d.xaxis + wid * nj * 3, nj * 3);
  cp(L.gxpos, d.geom_xpos + wid * ng * 3, ng * 3);
  cp(L.gxmat, d.geom_xmat + wid * ng * 9, ng * 9);
  cp(L.subtree_com, d.subtree_com + wid * nb * 3, nb * 3);
  cp(L.cinert, d.cinert + wid * nb * 10, nb * 10);
  cp(L.crb, d.crb + wid * nb * 10, nb * 10);
  cp(L.cdof, d.cdof + wid * nv * 6, nv * 6);
  const int nvs = L.nvs, np = m.nv_pad;
  for (long e = lane; e < nv * nvs; e += LPW) {
    const int r = (int)(e / nvs), c = (int)(e - (long)r * nvs);
    s[L.qM + e] = c < nv ? d.qM[(long)wid * np * np + r * np + c] : 0.0f;
  }
}

// SUB_*: the stage a sub_kernel launch runs (include/mjw_amd.h MJW_STAGE_*)
enum : int { SUB_KINEMATICS = 1, SUB_COM_POS = 2, SUB_CAMLIGHT = 3, SUB_TENDON = 4, SUB_CRB = 5, SUB_MAKE_CONSTRAINT = 6,
             SUB_TRANSMISSION = 7, SUB_COM_VEL = 8, SUB_PASSIVE = 9, SUB_RNE = 10 };
template <int SUB>
__global__ void __launch_bounds__(64) sub_kernel(const mjw_model_t m, const mjw_data_t d, const Lay L, int w0) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  WS w;
  w.s = smem;
  w.si = reinterpret_cast<int*>(smem);
  w.wid = w0 + (int)blockIdx.x;
  w.lane = lane_id();
  if (w.wid >= d.nworld) return;
  load_state(m, d, L, w);
  if constexpr (SUB != SUB_KINEMATICS) load_pos_fields(m, d, L, w);
  if constexpr (SUB >= SUB_COM_VEL) {
    // the velocity stage's inputs beyond the frames: the actuator moment rows (com_vel's actuator velocity)
    // and com_vel's outputs for passive / rne
    load_smooth(m, d, L, w, ST_VEL);
    const long nb = m.nbody, nv = m.nv;
    for (long e = w.lane; e < nb * 6; e += LPW) w.s[L.cvel + e] = d.cvel[w.wid * nb * 6 + e];
    for (long e = w.lane; e < nv * 6; e += LPW) w.s[L.cdof_dot + e] = d.cdof_dot[w.wid * nv * 6 + e];
  }
  WSYNC();
  if constexpr (SUB == SUB_KINEMATICS) kinematics(m, d, L, w);
  if constexpr (SUB == SUB_COM_POS) com_pos(m, d, L, w);
  if constexpr (SUB == SUB_CAMLIGHT) camlight(m, d, L, w);
  if constexpr (SUB == SUB_TENDON) {
    if (m.ntendon) {
      const TenFrames f{d.site_xpos + (long)w.wid * m.nsite * 3, w.s + L.gxpos, w.s + L.gxmat, w.s + L.subtree_com, w.s + L.cdof};
      tendon_pos(m, d, w.s + L.qpos, f, w.wid, w.lane);
    }
  }
  if constexpr (SUB == SUB_CRB) crb_qM<true>(m, d, L, w);
  if constexpr (SUB == SUB_MAKE_CONSTRAINT) collision_and_constraints<true, true, true>(m, d, L, w);
  if constexpr (SUB == SUB_TRANSMISSION) transmission<true>(m, d, L, w);
  if constexpr (SUB == SUB_COM_VEL) fwd_velocity<true, true, 1>(m, d, L, w);
  if constexpr (SUB == SUB_PASSIVE) fwd_velocity<true, true, 2>(m, d, L, w);
  if constexpr (SUB == SUB_RNE) fwd_velocity<true, true, 4>(m, d, L, w);
}

// -------------------------------------------------------------------------------------------
// collision pre-pass: one wave per world recomputes the geom frames (the forward kernel's own
// kinematics()) and, for the pairs with a pre-pass slot (nxn_ccdid >= 0), applies the broadphase
// filter and writes each survivor's contact record to d.ccd_out, which the forward kernel's
// narrowphase reads in pair order.  Two kinds of pairs:
//  * multi-point and rare primitives (plane-ellipsoid, plane-cylinder, sphere-cylinder, plane-mesh;
//    collision_primitive.py:665-1040, 810-880 plane_convex), one pair per lane;
//  * convex pairs (collision_driver.py:43-77 CONVEX: GJK / EPA, box-box multi-contact;
//    collision_convex.py:701-890), one pair at a time with the whole wave in lockstep over an LDS
//    workspace (mesh support points by a wave-parallel vertex scan).
// So the long, branchy CCD and the 4-point primitives never share a kernel (or registers) with the
// hot path.
// -------------------------------------------------------------------------------------------
// pre-pass kind of a type-sorted pair: 1 = lane-parallel primitive, 0 = convex (lockstep)
__device__ __forceinline__ int prepass_prim(int t1, int t2) {
  return (t1 == GEOM_PLANE && (t2 == GEOM_ELLIPSOID || t2 == GEOM_CYLINDER || t2 == GEOM_MESH)) || (t1 == GEOM_SPHERE && t2 == GEOM_CYLINDER);
}

// HF: the instantiation with the heightfield pairs (models with heightfields only: hfield_pair inlined
// next to the convex path doubles the kernel's registers, measured on apollo 0.077 -> 0.154 ms)
template <bool HF>
__device__ __forceinline__ void ccd_body(const mjw_model_t& m, const mjw_data_t& d, const Lay& L, int w0) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  WS w;
  w.s = smem;
  w.si = reinterpret_cast<int*>(smem);
  w.wid = w0 + (int)blockIdx.x;
  w.lane = lane_id();
  if (w.wid >= d.nworld) return;
  const int wid = w.wid, lane = w.lane;
  load_state(m, d, L, w);
  WSYNC();
  kinematics(m, d, L, w);
  float* s = w.s;
  const float* geom_margin = MR(geom_margin);
  const float* gsize = MR(geom_size);
  const float* mesh_vert = MR(mesh_vert);
  for (int p = lane; p < m.nxn; p += LPW) {
    const int slot = m.nxn_ccdid[p];
    if (slot < 0) continue;
    const int g1 = m.nxn_geom_pair[2 * p], g2 = m.nxn_geom_pair[2 * p + 1];
    const int t1 = m.geom_type[g1], t2 = m.geom_type[g2];
    if (!prepass_prim(t1, t2)) continue;
    if (!(m.nxn_pairid[2 * p + 1] >= 0 || broadphase_filter(m, L, s, wid, g1, g2))) continue;
    const float *p1 = s + L.gxpos + 3 * g1, *p2 = s + L.gxpos + 3 * g2, *r1 = s + L.gxmat + 9 * g1, *r2 = s + L.gxmat + 9 * g2;
    const float *s1 = gsize + 3 * g1, *s2 = gsize + 3 * g2;
    const float n1[3] = {r1[2], r1[5], r1[8]}, n2[3] = {r2[2], r2[5], r2[8]};
    float dist[4], pos[4][3], nrm[3] = {n1[0], n1[1], n1[2]};
    int n = 0;
    if (t1 == GEOM_PLANE && t2 == GEOM_ELLIPSOID) {
      dist[0] = plane_ellipsoid(pos[0], n1, p1, p2, r2, s2);
      n = 1;
    } else if (t1 == GEOM_PLANE && t2 == GEOM_CYLINDER) {
      for (int k = 0; k < 4; k++) plane_cylinder_k(k, n1, p1, p2, n2, s2[0], s2[1], &dist[k], pos[k]);
      n = 4;
    } else if (t1 == GEOM_SPHERE && t2 == GEOM_CYLINDER) {
      dist[0] = sphere_cylinder(pos[0], nrm, p1, s1[0], p2, n2, s2[0], s2[1]);
      n = 1;
    } else {  // plane-mesh
      const int md = m.geom_dataid[g2];
      n = plane_mesh(n1, p1, p2, r2, mesh_vert + 3 * (long)m.mesh_vertadr[md], m.mesh_vertnum[md], dist, pos);
    }
    float* out = d.ccd_out + ((long)wid * m.nxn_ccd + slot) * CCD_OUT;
    out[0] = (float)n;
    for (int i = 0; i < 3; i++) out[1 + i] = nrm[i];
    for (int q = 0; q < 4; q++) {
      out[4 + 4 * q] = q < n ? dist[q] : 0.0f;
      for (int i = 0; i < 3; i++) out[5 + 4 * q + i] = q < n ? pos[q][i] : 0.0f;
      for (int i = 0; i < 3; i++) out[20 + 3 * q + i] = nrm[i];
    }
  }
  if (L.ccd < 0) return;  // no convex pair (the lockstep workspace is not allocated)
  const CcdLay CL = ccd_layout(m.ccd_epa_iterations, HF && m.nhfield > 0, m.nmaxpolygon, m.nmaxmeshdeg);
  float* W = s + L.ccd;
  const MeshPoly MP = mesh_poly(m);
  for (int p = 0; p < m.nxn; p++) {
    const int slot = m.nxn_ccdid[p];
    if (slot < 0) continue;
    const int g1 = m.nxn_geom_pair[2 * p], g2 = m.nxn_geom_pair[2 * p + 1];
    const int t1 = m.geom_type[g1], t2 = m.geom_type[g2];
    if (prepass_prim(t1, t2)) continue;
    const bool pass = m.nxn_pairid[2 * p + 1] >= 0 || broadphase_filter(m, L, s, wid, g1, g2);
    int nc = 0;
    if (HF && pass && t1 == GEOM_HFIELD) {
      // heightfield-convex pair (collision_convex.py:158-697): its record is built whole in the workspace
      const int hid = m.geom_dataid[g1], md2 = t2 == GEOM_MESH ? m.geom_dataid[g2] : -1;
      const int pid = m.nxn_pairid[2 * p];
      CcdWS cw;
      cw.W = W;
      cw.L = CL;
      hfield_pair(cw, m.ccd_epa_iterations, MR(opt_ccd_tolerance)[0], m.opt_ccd_iterations, geom_margin[g1] + geom_margin[g2],
                  pid > -1 ? MR(pair_margin)[pid] : geom_margin[g1] + geom_margin[g2], s + L.gxpos + 3 * g1, s + L.gxmat + 9 * g1,
                  MR(hfield_size) + 4 * hid, m.hfield_nrow[hid], m.hfield_ncol[hid], MR(hfield_data) + m.hfield_adr[hid],
                  s + L.gxpos + 3 * g2, s + L.gxmat + 9 * g2, gsize + 3 * g2, MR(geom_rbound)[g2], t2,
                  md2 >= 0 ? mesh_vert + 3 * (long)m.mesh_vertadr[md2] : nullptr, md2 >= 0 ? m.mesh_vertnum[md2] : 0, W + CL.out);
      float* out = d.ccd_out + ((long)wid * m.nxn_ccd + slot) * CCD_OUT;
      if (lane < CCD_OUT) out[lane] = W[CL.out + lane];
      continue;
    }
    if (pass) {
      const int md1 = t1 == GEOM_MESH ? m.geom_dataid[g1] : -1, md2 = t2 == GEOM_MESH ? m.geom_dataid[g2] : -1;
      put_cgeom(W + CL.geoms, s + L.gxpos + 3 * g1, s + L.gxmat + 9 * g1, gsize + 3 * g1, t1, md1 >= 0 ? m.mesh_vertadr[md1] : 0,
                md1 >= 0 ? m.mesh_vertnum[md1] : 0, md1);
      put_cgeom(W + CL.geoms + CGEOM_WORDS, s + L.gxpos + 3 * g2, s + L.gxmat + 9 * g2, gsize + 3 * g2, t2,
                md2 >= 0 ? m.mesh_vertadr[md2] : 0, md2 >= 0 ? m.mesh_vertnum[md2] : 0, md2);
      const int pid = m.nxn_pairid[2 * p];  // explicit <pair>: its own margin (collision_core.py:271)
      nc = ccd_pair(W, m.ccd_epa_iterations, MR(opt_ccd_tolerance)[0], m.opt_ccd_iterations,
                    pid > -1 ? MR(pair_margin)[pid] : geom_margin[g1] + geom_margin[g2], mesh_vert, 0.0f, &MP,
                    (m.opt_enableflags & ENBL_MULTICCD) != 0, m.nmaxpolygon, m.nmaxmeshdeg);
    }
    float* out = d.ccd_out + ((long)wid * m.nxn_ccd + slot) * CCD_OUT;
    if (lane < CCD_OUT) out[lane] = ccd_record_word(lane, nc, W + CL.out);
  }
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) ccd_kernel(const mjw_model_t m, const mjw_data_t d, const Lay L, int w0) {
  ccd_body<false>(m, d, L, w0);
}
__global__ void __launch_bounds__(64) ccd_hf_kernel(const mjw_model_t m, const mjw_data_t d, const Lay L, int w0) {
  ccd_body<true>(m, d, L, w0);
}

// -------------------------------------------------------------------------------------------
// The collision sub-stages as entry points of their own (mujoco_warp/__init__.py:33-35).  The step runs
// broad- and narrowphase fused in the forward kernel, one wave per world, without materialising the
// candidate list; these two kernels expose the same computations over the reference's intermediate
// arrays (collision_core.py:345-365 CollisionContext), reading the geom frames from HBM (d.geom_xpos /
// d.geom_xmat, as left by the position stage).
// -------------------------------------------------------------------------------------------
// collision_driver.py:697-731 nxn_broadphase, :325-358 _add_geom_pair: one thread per (world, filtered
// pair); survivors of opt.broadphase_filter (and pairs with a collision sensor) take an atomically
// reserved slot, slots past naconmax only counted.  nxn_geom_pair is type-ordered on the host already.
__global__ void __launch_bounds__(256) nxn_broadphase_kernel(const mjw_model_t m, const mjw_data_t d, int* cpair, int* cpairid, int* cworld) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)d.nworld * m.nxn) return;
  const int wid = (int)(t / m.nxn), p = (int)(t - (long)wid * m.nxn);
  const int g1 = m.nxn_geom_pair[2 * p], g2 = m.nxn_geom_pair[2 * p + 1];
  const float* gx = d.geom_xpos + (long)wid * m.ngeom * 3;
  const float* gm = d.geom_xmat + (long)wid * m.ngeom * 9;
  if (!(m.nxn_pairid[2 * p + 1] >= 0 || broadphase_filter_g(m, gx, gm, wid, g1, g2))) return;
  const int k = atomicAdd(d.ncollision, 1);
  if (k >= d.naconmax) return;
  cpair[2 * k] = g1;
  cpair[2 * k + 1] = g2;
  cpairid[2 * k] = m.nxn_pairid[2 * p];
  cpairid[2 * k + 1] = m.nxn_pairid[2 * p + 1];
  cworld[k] = wid;
}

// collision_primitive.py:1461-1549 primitive_narrowphase (+ collision_core.py:160-232 write_contact): one
// thread per candidate [0, min(ncollision, naconmax)) whose type pair is set in `typemask` (bit 8 t1 + t2 of
// the type-ordered pair; the PRIMITIVE entries of collision_driver.py:43-77 by default).  Every point is
// written at an atomically reserved pool slot unless it is inactive (dist >= margin) or its pair is
// excluded (pairid -2) and no collision sensor asked for it; its type carries CONSTRAINT (active, not
// excluded) and SENSOR bits, geomcollisionid the point's index within the pair, efc_address -1 (the rows
// come from make_constraint).  Same geometry routines as the fused path: plane-sphere / capsule,
// sphere-sphere / capsule / box, capsule-capsule / box (narrowphase), plane-box corners, plane-ellipsoid /
// cylinder / mesh and sphere-cylinder (the pre-pass routines).
// collision_driver.py:554-643 sap_broadphase (SAP_TILE / SAP_SEGMENTED; one workgroup per world here): every
// geom's bounding sphere (rbound + margin; planes unbounded) projected on the reference's fixed direction, the
// lower ends sorted in LDS (bitonic, padded to a power of two), and for each sorted geom i the candidates j in
// (i, min(ngeom - 1, first j with lower_j > upper_i)] (:421-441 _sap_range with _binary_search :362-370, the
// first geom past the overlap included, as there); a candidate that is not an NXN pair (excluded: contype /
// conaffinity, parent, self, <exclude>) is skipped, the others pass the same broadphase filter as the NXN
// path (or always, with a collision-sensor id) and are appended as mjw_nxn_broadphase does
constexpr int SAP_MAX_GEOM = 4096;  // LDS: lower / index of the padded sort + upper per geom
__global__ void __launch_bounds__(256) sap_broadphase_kernel(const mjw_model_t m, const mjw_data_t d, int* cpair, int* cpairid, int* cworld) {
  extern __shared__ __attribute__((aligned(16))) float sap_sh[];
  const int wid = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
  if (wid >= d.nworld) return;
  const int ng = m.ngeom;
  int np2 = 1;
  while (np2 < ng) np2 <<= 1;
  float* lo = sap_sh;
  int* ix = reinterpret_cast<int*>(sap_sh + np2);
  float* up = sap_sh + 2 * np2;
  const float* gx = d.geom_xpos + (long)wid * ng * 3;
  const float* gm = d.geom_xmat + (long)wid * ng * 9;
  const float* geom_rbound = MR(geom_rbound);
  const float* geom_margin = MR(geom_margin);
  float dir[3] = {0.5935f, 0.7790f, 0.1235f};
  const float dn = 1.0f / sqrtf(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
  for (int i = 0; i < 3; i++) dir[i] *= dn;
  for (int g = t; g < np2; g += nt) {
    if (g < ng) {
      float rb = geom_rbound[g];
      if (rb == 0.0f) rb = MJW_MAXVAL;  // a plane
      const float radius = rb + geom_margin[g];
      const float center = dir[0] * gx[3 * g] + dir[1] * gx[3 * g + 1] + dir[2] * gx[3 * g + 2];
      const bool nan = center != center;
      lo[g] = nan ? MJW_MAXVAL : center - radius;
      up[g] = nan ? MJW_MAXVAL : center + radius;
      ix[g] = g;
    } else {
      lo[g] = __builtin_huge_valf();  // padding sorts last
      ix[g] = -1;
    }
  }
  __syncthreads();
  // bitonic sort of (lo, ix) ascending
  for (int k = 2; k <= np2; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = t; i < np2; i += nt) {
        const int l = i ^ j;
        if (l > i) {
          const bool asc = (i & k) == 0;
          const float a = lo[i], b = lo[l];
          if ((a > b) == asc) {
            lo[i] = b; lo[l] = a;
            const int x = ix[i]; ix[i] = ix[l]; ix[l] = x;
          }
        }
      }
      __syncthreads();
    }
  for (int i = t; i < ng; i += nt) {
    const int g1 = ix[i];
    const float upper = up[g1];
    int a = i + 1, b = ng;  // first position past i whose lower end exceeds upper
    while (a < b) {
      const int mid = (a + b) >> 1;
      if (lo[mid] > upper) b = mid;
      else a = mid + 1;
    }
    const int limit = min(ng - 1, b);
    for (int j = i + 1; j <= limit; j++) {
      const int g2 = ix[j];
      const int ga = min(g1, g2), gb = max(g1, g2);
      const long key = (long)ga * ng + gb;
      // the NXN pair of (ga, gb): the filtered list is in upper-triangle order (its entries type-ordered)
      int pa = 0, pb = m.nxn, p = -1;
      while (pa < pb) {
        const int mid = (pa + pb) >> 1;
        const int h1 = m.nxn_geom_pair[2 * mid], h2 = m.nxn_geom_pair[2 * mid + 1];
        const long km = (long)min(h1, h2) * ng + max(h1, h2);
        if (km == key) { p = mid; break; }
        if (km < key) pa = mid + 1;
        else pb = mid;
      }
      if (p < 0) continue;
      if (!(m.nxn_pairid[2 * p + 1] >= 0 || broadphase_filter_g(m, gx, gm, wid, ga, gb))) continue;
      const int k = atomicAdd(d.ncollision, 1);
      if (k >= d.naconmax) continue;
      cpair[2 * k] = m.nxn_geom_pair[2 * p];
      cpair[2 * k + 1] = m.nxn_geom_pair[2 * p + 1];
      cpairid[2 * k] = m.nxn_pairid[2 * p];
      cpairid[2 * k + 1] = m.nxn_pairid[2 * p + 1];
      cworld[k] = wid;
    }
  }
}

__global__ void __launch_bounds__(256) primitive_narrowphase_kernel(const mjw_model_t m, const mjw_data_t d, const int* cpair, const int* cpairid,
                                                                    const int* cworld, unsigned long long typemask) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= min(d.ncollision[0], d.naconmax)) return;
  const int g1 = cpair[2 * k], g2 = cpair[2 * k + 1], wid = cworld[k];
  const int pid0 = cpairid[2 * k], pid1 = cpairid[2 * k + 1];
  if (g1 < 0 || g2 < 0 || wid < 0 || wid >= d.nworld) return;
  const int t1 = m.geom_type[g1], t2 = m.geom_type[g2];
  if (t1 > 7 || t2 > 7 || !((typemask >> (8 * t1 + t2)) & 1ull)) return;
  const float* gx = d.geom_xpos + (long)wid * m.ngeom * 3;
  const float* gm = d.geom_xmat + (long)wid * m.ngeom * 9;
  float margin, gap, friction[5], solref[2], solimp[5], srf[2];
  int condim;
  contact_params(m, wid, g1, g2, pid0, &margin, &gap, &condim, friction, solref, solimp, srf);
  const float* gsize = MR(geom_size);
  const float *p1 = gx + 3 * g1, *p2 = gx + 3 * g2, *r1 = gm + 9 * g1, *r2 = gm + 9 * g2;
  const float n1[3] = {r1[2], r1[5], r1[8]}, n2[3] = {r2[2], r2[5], r2[8]};
  // gid: the candidate point's index within the pair (the corner index for plane-box, collision_primitive.py:
  // 774-778), whether or not earlier candidates were written
  auto write = [&](int gid, float dist, const float* pos, const float* frame) {
    const bool active = dist < margin;
    if ((pid0 == -2 || !active) && pid1 == -1) return;
    const int type = ((pid0 >= -1 && active) ? 1 : 0) | (pid1 >= 0 ? 2 : 0);
    const int cid = atomicAdd(d.nacon, 1);
    if (cid >= d.naconmax) return;
    d.contact_dist[cid] = dist;
    for (int i = 0; i < 3; i++) d.contact_pos[3L * cid + i] = pos[i];
    for (int i = 0; i < 9; i++) d.contact_frame[9L * cid + i] = frame[i];
    d.contact_includemargin[cid] = margin - gap;
    for (int i = 0; i < 5; i++) d.contact_friction[5L * cid + i] = friction[i];
    for (int i = 0; i < 2; i++) {
      d.contact_solref[2L * cid + i] = solref[i];
      d.contact_solreffriction[2L * cid + i] = srf[i];
    }
    for (int i = 0; i < 5; i++) d.contact_solimp[5L * cid + i] = solimp[i];
    d.contact_dim[cid] = condim;
    d.contact_geom[2L * cid] = g1;
    d.contact_geom[2L * cid + 1] = g2;
    d.contact_worldid[cid] = wid;
    d.contact_type[cid] = type;
    d.contact_geomcollisionid[cid] = gid;
    for (int i = 0; i < m.nmaxpyramid; i++) d.contact_efc_address[(long)cid * m.nmaxpyramid + i] = -1;
  };
  float frame[9];
  if (t1 == GEOM_PLANE && t2 == GEOM_BOX) {
    make_frame(frame, n1);
    for (int q = 0; q < 8; q++) {
      float cp[3];
      const float dist = plane_box_corner(q, n1, p1, p2, r2, gsize + 3 * g2, cp);
      write(q, dist, cp, frame);
    }
  } else if (prepass_prim(t1, t2)) {
    float dist[4], pos[4][3], nrm[3] = {n1[0], n1[1], n1[2]};
    int n = 0;
    if (t1 == GEOM_PLANE && t2 == GEOM_ELLIPSOID) {
      dist[0] = plane_ellipsoid(pos[0], n1, p1, p2, r2, gsize + 3 * g2);
      n = 1;
    } else if (t1 == GEOM_PLANE && t2 == GEOM_CYLINDER) {
      for (int q = 0; q < 4; q++) plane_cylinder_k(q, n1, p1, p2, n2, gsize[3 * g2], gsize[3 * g2 + 1], &dist[q], pos[q]);
      n = 4;
    } else if (t1 == GEOM_SPHERE && t2 == GEOM_CYLINDER) {
      dist[0] = sphere_cylinder(pos[0], nrm, p1, gsize[3 * g1], p2, n2, gsize[3 * g2], gsize[3 * g2 + 1]);
      n = 1;
    } else {  // plane-mesh
      const int md = m.geom_dataid[g2];
      n = plane_mesh(n1, p1, p2, r2, MR(mesh_vert) + 3 * (long)m.mesh_vertadr[md], m.mesh_vertnum[md], dist, pos);
    }
    make_frame(frame, nrm);
    for (int q = 0; q < n; q++) write(q, dist[q], pos[q], frame);
  } else {
    Con2 c;
    narrowphase_g<true>(m, gx, gm, wid, g1, g2, margin, c);
    for (int q = 0; q < c.n; q++) write(q, c.dist[q], c.pos[q], c.frame[q]);
  }
}

// benchmark.py:41-83
// clears the contact pool counters at the start of the position stage.  A kernel, not
// hipMemsetAsync: in a captured hipGraph the 4-byte memset node was observed to race the
// forward kernel (stale counts, contacts dropped past the pool), kernel nodes stay ordered
//
// It also builds the dense kernel's longest-first world order for this step from the iteration bucket the
// previous step's solving dense kernel stored per world (world_key, plain stores): a counting sort over the
// buckets in this one workgroup writes world_order, a permutation of the worlds with the most iterations
// first.  The histogram is counted here with LDS atomics, not by the dense kernels: they used to bump the
// 32 bucket words with a global atomicAdd per world, and with one bucket holding nearly every world
// (franka, 1-2 Newton iterations) those same-address atomics held each wave's slot until they drained --
// franka's dense kernel measured 0.246 ms with them against 0.147 ms with the order off
// (profiles/r06_ab_order.log).  (A wave-aggregated count -- one ballot and one LDS add per distinct key
// of a 64-world chunk -- measured 0.022 ms for this kernel against 0.009 ms: humanoid CG has ~20 keys.)
// The histogram and the scatter read the same keys (clamped to the bucket range), so world_order is a
// permutation whatever the keys hold; stale keys only cost order quality.  One bucket holding 7/8 of the
// worlds orders nothing: world_order is then the identity.
constexpr int RESET_THREADS = 1024;
__global__ void __launch_bounds__(RESET_THREADS) reset_counters_kernel(int* nacon, int* ncollision, int* sched, int* world_order,
                                                                       const int* world_key, int nworld) {
  const int t = threadIdx.x;
  if (t == 0) { nacon[0] = 0; ncollision[0] = 0; }
  if (!sched) return;
  constexpr int NB = MJW_SCHED_BUCKETS;
  static_assert(NB <= 64, "one wave scans the buckets");
  // a 64-world chunk whose worlds share one key is counted with one LDS add by its first lane: with one
  // bucket holding every world (franka, 16 k worlds) per-lane adds serialised 64 ways in every
  // wave-instruction (0.024 ms for this kernel); mixed chunks add per lane, into per-wave histograms (row
  // stride NB + 1)
  constexpr int NWV = RESET_THREADS / 64;
  __shared__ int hist[NWV * (NB + 1)];
  __shared__ int cursor[NB];
  __shared__ int valid;
  const int wv = t >> 6, lane = t & 63;
  for (int i = t; i < NWV * (NB + 1); i += RESET_THREADS) hist[i] = 0;
  // the keys of the first KPT * RESET_THREADS worlds stay in registers for the scatter (all loads issued
  // before the first LDS add)
  constexpr int KPT = 16;
  int kk[KPT];
#pragma unroll
  for (int q = 0; q < KPT; q++) {
    const int w = t + q * RESET_THREADS;
    kk[q] = w < nworld ? min(max(world_key[w], 0), NB - 1) : -1;
  }
  __syncthreads();
  int* hw = hist + wv * (NB + 1);
#pragma unroll
  for (int q = 0; q < KPT; q++) {
    const int k = kk[q];
    const int k0 = __shfl(k, 0);
    if (__ballot(k != k0 && k >= 0) == 0ull) {  // every valid key equals the first lane's
      const int n = __popcll(__ballot(k >= 0));
      if (lane == 0 && k0 >= 0) atomicAdd(&hw[k0], n);
    } else if (k >= 0) {
      atomicAdd(&hw[k], 1);
    }
  }
  for (int w = t + KPT * RESET_THREADS; w < nworld; w += RESET_THREADS) atomicAdd(&hw[min(max(world_key[w], 0), NB - 1)], 1);
  __syncthreads();
  if (t < NB) {
    int h = 0;
#pragma unroll
    for (int v = 0; v < NWV; v++) h += hist[v * (NB + 1) + t];
    hist[t] = h;  // (row 0, bucket t: read back only by thread t's own wave below)
  }
  __syncthreads();
  if (t < 64) {
    const int h = t < NB ? hist[t] : 0;
    int x = h;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (t >= o) x += y;
    }
    int hmax = h;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) hmax = max(hmax, __shfl_xor(hmax, o));
    if (t < NB) cursor[t] = x - h;
    if (t == 0) valid = hmax < nworld - (nworld >> 3);
  }
  __syncthreads();
  if (valid) {
#pragma unroll
    for (int q = 0; q < KPT; q++)
      if (kk[q] >= 0) world_order[atomicAdd(&cursor[kk[q]], 1)] = t + q * RESET_THREADS;
    for (int w = t + KPT * RESET_THREADS; w < nworld; w += RESET_THREADS)
      world_order[atomicAdd(&cursor[min(max(world_key[w], 0), NB - 1)], 1)] = w;
  } else {
    for (int w = t; w < nworld; w += RESET_THREADS) world_order[w] = w;
  }
}

// forward.py:883-927 (_tendon_actuator_force_clamp, _qfrc_actuator, _qfrc_actuator_gravcomp_limits): the
// tendon actuator force range applied to the Data's actuator_force (written back), then qfrc_actuator =
// moment' force from the sparse moment rows, plus the actuator-level gravity compensation, clamped by the
// joint actuator force range; one wave per world, lanes over dofs.  The staged fwd_actuation runs it after
// the act_dyn / act_gain / act_bias callbacks (forward.py:876-881), which may rewrite actuator_force.  (The
// stage launch before the callbacks applied the tendon range already; forces it left in range pass unchanged.)
// per-world slot range of the contact pool for the POOL row pass (mjw_contact_rows): ncon_world[2w] = first
// slot of world w, ncon_world[2w + 1] = span to its last slot (0 when it has none); the narrowphase reserves
// one block per world and staging round, so the span is the world's own contacts unless it took several rounds
__global__ void pool_ranges_init_kernel(const mjw_data_t d) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= d.nworld) return;
  d.ncon_world[2L * w] = 0x7fffffff;
  d.ncon_world[2L * w + 1] = -1;  // last slot, turned into the span below
}
__global__ void pool_ranges_kernel(const mjw_data_t d) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = min(d.nacon[0], d.naconmax);
  if (k >= n) return;
  const int w = d.contact_worldid[k];
  if (w < 0 || w >= d.nworld) return;
  atomicMin(d.ncon_world + 2L * w, k);
  atomicMax(d.ncon_world + 2L * w + 1, k);
}
__global__ void pool_ranges_finish_kernel(const mjw_data_t d) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= d.nworld) return;
  const int k0 = d.ncon_world[2L * w], k1 = d.ncon_world[2L * w + 1];
  d.ncon_world[2L * w] = k1 < 0 ? 0 : k0;
  d.ncon_world[2L * w + 1] = k1 < 0 ? 0 : k1 - k0 + 1;
}

// host: the ranges above for every world of d (mjw_contact_rows, and sensor_launch for the contact and
// tactile sensors)
int pool_ranges_launch(const mjw_data_t* d, hipStream_t s) {
  if (d->nworld <= 0) return 0;
  const int nb = (d->nworld + 255) / 256, nk = (d->naconmax + 255) / 256;
  hipLaunchKernelGGL(pool_ranges_init_kernel, dim3(nb), dim3(256), 0, s, *d);
  if (nk > 0) hipLaunchKernelGGL(pool_ranges_kernel, dim3(nk), dim3(256), 0, s, *d);
  hipLaunchKernelGGL(pool_ranges_finish_kernel, dim3(nb), dim3(256), 0, s, *d);
  return (int)hipGetLastError();
}

__global__ void __launch_bounds__(64) actuator_map_kernel(const mjw_model_t m, const mjw_data_t d) {
  const int wid = blockIdx.x, lane = threadIdx.x;
  if (wid >= d.nworld) return;
  const int nv = m.nv, nu = m.nu;
  const bool off = !nu || (m.opt_disableflags & DSBL_ACTUATION);
  // each actuator drives one tendon, so a lane rescales only forces no other tendon's sum reads
  if (!off && m.ntendon) tendon_actuator_clamp(m, d.actuator_force + (long)wid * nu, wid, lane);
  const float* jnt_actfrcrange = MR(jnt_actfrcrange);
  for (int i = lane; i < nv; i += 64) {
    float q = 0.0f;
    if (!off) {
      for (int a = 0; a < nu; a++) {
        const long ga = (long)wid * nu + a;
        const int nnz = d.moment_rownnz[ga], adr = d.moment_rowadr[ga];
        const float f = d.actuator_force[ga];
        for (int k = 0; k < nnz; k++) {
          const long e = (long)wid * m.nJmom + adr + k;
          if (d.moment_colind[e] == i) q += d.actuator_moment[e] * f;
        }
      }
      const int j = m.dof_jntid[i];
      if (m.ngravcomp && m.jnt_actgravcomp[j]) q += d.qfrc_gravcomp[(long)wid * nv + i];
      if (m.jnt_actfrclimited[j]) q = clampf(q, jnt_actfrcrange[2 * j], jnt_actfrcrange[2 * j + 1]);
    }
    d.qfrc_actuator[(long)wid * nv + i] = q;
  }
}

__global__ void ctrl_noise_kernel(const mjw_model_t m, const mjw_data_t d, const float* center, int step, float std, float rate_) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= d.nworld * m.nu) return;
  int w = t / m.nu, a = t - w * m.nu;
  int wid = w;
  int worldid = d.world_offset + w;
  float rate = expf(-MR(opt_timestep)[0] / rate_);
  float scale = std * sqrtf(1.0f - rate * rate);
  float midpoint = 0.0f, halfrange = 1.0f;
  const float* cr = MR(actuator_ctrlrange) + 2 * a;
  bool lim = m.actuator_ctrllimited[a];
  if (lim) { midpoint = 0.5f * (cr[1] + cr[0]); halfrange = 0.5f * (cr[1] - cr[0]); }
  if (center) midpoint = center[a];
  float c = rate * d.ctrl[t] + (1.0f - rate) * midpoint;
  c += scale * halfrange * (2.0f * halton((step + 1) * (worldid + 1), a + 2) - 1.0f);
  if (lim) c = clampf(c, cr[0], cr[1]);
  d.ctrl[t] = c;
}

}  // namespace mjw

// =============================================================================================
// C ABI
// =============================================================================================
namespace mjw {
thread_local LaunchTrace* g_trace = nullptr;
}

namespace {
thread_local std::string g_err;

int set_err(hipError_t e, const char* where) {
  if (e == hipSuccess) return 0;
  g_err = std::string(where) + ": " + hipGetErrorString(e);
  return (int)e;
}

hipError_t reset_counters(const mjw_data_t* d, hipStream_t s, bool order = false) {
  // the order is built only for the dense path's full forward + solve (run() passes order = true)
  hipLaunchKernelGGL(mjw::reset_counters_kernel, dim3(1), dim3(order ? mjw::RESET_THREADS : 64), 0, s, d->nacon, d->ncollision,
                     order ? d->sched : nullptr, d->world_order, d->world_key, d->nworld);
  mjw::trace_launch(s, mjw::K_RESET);
  return hipGetLastError();
}

// worlds [w0, w0 + count) of d; the pool counters are cleared by the caller (run) before the
// position stage of any world range
template <int STAGES>
int launch_generic(const mjw_model_t* m, const mjw_data_t* d, hipStream_t s, const char* name, int w0 = 0, int count = -1) {
  constexpr bool nofactor = (STAGES & mjw::ST_NOFACTOR) != 0;
  if (count < 0) count = d->nworld - w0;
  if (count <= 0) return 0;
  mjw::Lay L = mjw::make_layout(*m, d->njmax, nofactor);
  size_t lds = (size_t)L.total * 4;
  static const size_t lds_pad = [] {  // occupancy experiments only (MJW_LDS_PAD bytes)
    const char* e = getenv("MJW_LDS_PAD");
    return e ? (size_t)atol(e) : (size_t)0;
  }();
  lds += lds_pad;
  if (lds > 160 * 1024) { g_err = std::string(name) + ": per-world LDS working set exceeds 160 KiB"; return -3; }
  if ((STAGES & mjw::ST_POS) && !(STAGES & mjw::ST_POOL)) {
    if (m->nxn_ccd > 0 && d->naconmax > 0 && !(m->opt_disableflags & (mjw::DSBL_CONSTRAINT | mjw::DSBL_CONTACT))) {
      static std::once_flag once_ccd;
      std::call_once(once_ccd, [] {
        (void)hipFuncSetAttribute((const void*)mjw::ccd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)mjw::ccd_hf_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      });
      const mjw::Lay LC = mjw::make_layout(*m, d->njmax, nofactor, true);
      if (m->nhfield > 0) {
        hipLaunchKernelGGL(mjw::ccd_hf_kernel, dim3(count), dim3(64), (size_t)LC.total * 4, s, *m, *d, LC, w0);
        mjw::trace_launch(s, mjw::K_CCD_HF);
      } else {
        hipLaunchKernelGGL(mjw::ccd_kernel, dim3(count), dim3(64), (size_t)LC.total * 4, s, *m, *d, LC, w0);
        mjw::trace_launch(s, mjw::K_CCD);
      }
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return set_err(e, name);
    }
  }
  static std::once_flag once;
  std::call_once(once, [] {
    (void)hipFuncSetAttribute((const void*)mjw::mjw_kernel<STAGES, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if constexpr ((STAGES & mjw::ST_POS) != 0) {
      (void)hipFuncSetAttribute((const void*)mjw::mjw_kernel<STAGES, false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)mjw::mjw_kernel<STAGES, true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    }
  });
  // position-stage kernels without the tendon / muscle paths, and without the box narrowphase, for
  // models that have none (kernel id: K_FWD + 4 STAGES + 2 BOX + TEN)
  if constexpr ((STAGES & mjw::ST_POS) != 0) {
    if (m->ntendon == 0 && m->nmuscle == 0 && m->ngravcomp == 0 && !m->has_fluid && m->nbodytrn == 0 && m->nsitetrn == 0) {
      if (m->nxn_box == 0) {
        hipLaunchKernelGGL((mjw::mjw_kernel<STAGES, false, false>), dim3(count), dim3(64), lds, s, *m, *d, L, w0);
        mjw::trace_launch(s, mjw::K_FWD + 4 * STAGES);
      } else {
        hipLaunchKernelGGL((mjw::mjw_kernel<STAGES, true, false>), dim3(count), dim3(64), lds, s, *m, *d, L, w0);
        mjw::trace_launch(s, mjw::K_FWD + 4 * STAGES + 2);
      }
      return set_err(hipGetLastError(), name);
    }
  }
  hipLaunchKernelGGL((mjw::mjw_kernel<STAGES, true, true>), dim3(count), dim3(64), lds, s, *m, *d, L, w0);
  mjw::trace_launch(s, mjw::K_FWD + 4 * STAGES + 3);
  return set_err(hipGetLastError(), name);
}

// the register-resident path (mjw_dense.h) covers worlds with nv <= 32 and njmax <= 64
bool dense_ok(const mjw_model_t* m, const mjw_data_t* d) { return m->nv <= 32 && d->njmax <= 64; }

// the fused whole-step kernel (step_kernel): instantiated for CG models without tendons / muscles /
// gravity compensation / fluid / site or body transmissions (the lean forward variant), without box
// pairs, with the dense factor bound NB = 28; returns kNotFused when it does not apply (the caller then
// launches the forward and dense kernels)
constexpr int kNotFused = 0x7fffffff;
template <bool NEWTON>
int launch_step_fused(const mjw_model_t* m, const mjw_data_t* d, hipStream_t s, const char* name) {
  constexpr int STAGES = mjw::ST_POS | mjw::ST_VEL | mjw::ST_ACT | mjw::ST_ACC | mjw::ST_NOFACTOR;
  mjw::Lay L = mjw::make_layout(*m, d->njmax, true);
  const size_t lds = std::max((size_t)L.total * 4, (size_t)mjw::dense_lds_words<7, NEWTON, false, 28>() * 4);
  if (lds > 160 * 1024) return kNotFused;
  static std::once_flag once;
  std::call_once(once, [] {
    (void)hipFuncSetAttribute((const void*)mjw::step_kernel<STAGES, false, 7, NEWTON, 28>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  });
  hipLaunchKernelGGL((mjw::step_kernel<STAGES, false, 7, NEWTON, 28>), dim3(d->nworld), dim3(64), lds, s, *m, *d, L, 0);
  mjw::trace_launch(s, mjw::K_STEP + (NEWTON ? 1 : 0));
  return set_err(hipGetLastError(), name);
}

int step_fused(const mjw_model_t* m, const mjw_data_t* d, hipStream_t s, const char* name) {
  using namespace mjw;
  static const bool on = [] {
    const char* e = getenv("MJW_FUSED");
    return !(e && e[0] == '0');
  }();
  if (!on) return kNotFused;
  const int fl = m->opt_disableflags;
  const bool implicit_int = m->opt_integrator == INT_IMPLICITFAST
                                ? (fl & (DSBL_ACTUATION | DSBL_SPRING | DSBL_DAMPER)) != (DSBL_ACTUATION | DSBL_SPRING | DSBL_DAMPER)
                                : !(fl & (DSBL_EULERDAMP | DSBL_DAMPER));
  const bool lean = m->ntendon == 0 && m->nmuscle == 0 && m->ngravcomp == 0 && !m->has_fluid && m->nbodytrn == 0 && m->nsitetrn == 0 && m->nxn_box == 0;
  const bool ccd = m->nxn_ccd > 0 && d->naconmax > 0 && !(fl & (DSBL_CONSTRAINT | DSBL_CONTACT));
  if (!lean || ccd || implicit_int || m->opt_cone == CONE_ELLIPTIC || m->opt_integrator == INT_RK4 || m->nv <= 16 || m->nv > 28)
    return kNotFused;
  // CG by default: the Newton dense half needs 131-134 VGPRs and spills at the fused kernel's 128 (humanoid
  // Newton measured 0.513 -> 0.558 ms fused, round 5); MJW_FUSED_NEWTON=1 launches it fused (A/B runs)
  static const bool newton_on = [] {
    const char* e = getenv("MJW_FUSED_NEWTON");
    return e && e[0] == '1';
  }();
  if (m->opt_solver == SOLVER_NEWTON) return newton_on ? launch_step_fused<true>(m, d, s, name) : kNotFused;
  return launch_step_fused<false>(m, d, s, name);
}

// optional timing events for the next run(): before the forward kernel, between it and
// the dense kernel, after the dense kernel (mjw_step_events)
thread_local hipEvent_t g_ev[3] = {nullptr, nullptr, nullptr};

// stage groups: ST_* bits of the stages to run, in pipeline order
int run(const mjw_model_t* m, const mjw_data_t* d, void* stream, int stages, const char* name) {
  using namespace mjw;
  if (!m || !d) { g_err = std::string(name) + ": null model/data"; return -1; }
  if (d->nworld <= 0) return 0;
  // sensors (all stages, one kernel after the solver and before the integrator): only the fused
  // forward / step (the stage entry points, like the reference's fwd_* functions, compute none)
  const bool full = (stages & (ST_POS | ST_VEL | ST_ACT | ST_ACC | ST_SOLVE)) == (ST_POS | ST_VEL | ST_ACT | ST_ACC | ST_SOLVE);
  const bool acc_sensors = full && m->nsensor > 0 && !(m->opt_disableflags & DSBL_SENSOR);
  if (m->is_sparse) {
    // workgroup-per-world sparse / flex pipeline (mjw_sparse.hip), the same sensor kernel after the solve
    if ((stages & ST_SOLVE) && m->opt_solver == SOLVER_NEWTON && m->sp_nH != m->nv) {
      g_err = std::string(name) + ": sparse Newton needs the Hessian workspace (put_model with opt.solver = NEWTON, nv <= 256)";
      return -5;
    }
    hipStream_t s = (hipStream_t)stream;
    if ((stages & ST_POS) && !(stages & ST_POOL)) {
      hipError_t e = reset_counters(d, s);
      if (e != hipSuccess) return set_err(e, name);
    }
    if (g_ev[0]) (void)hipEventRecord(g_ev[0], s);
    int rc = set_err((hipError_t)sparse_launch(stages & ~ST_EULER, m, d, s), name);
    if (!rc && acc_sensors) rc = set_err((hipError_t)sensor_launch(m, d, s, 7), name);
    if (g_ev[1]) (void)hipEventRecord(g_ev[1], s);
    if (!rc && (stages & ST_EULER)) rc = set_err((hipError_t)sparse_launch(ST_EULER, m, d, s), name);
    if (g_ev[2]) (void)hipEventRecord(g_ev[2], s);
    return rc;
  }
  if (m->nv > 64 || m->nbody > 4096) { g_err = std::string(name) + ": model too large for the dense world-per-wave path"; return -2; }
  hipStream_t s = (hipStream_t)stream;
  int rc = 0;
  // longest-first world order of the dense kernels (the counter-reset kernel sorts the worlds by the
  // iteration bucket the previous step's solving dense kernel recorded; the dense kernels read
  // world_order; the solving one records this step's buckets): full forward + solve on the dense path
  // only; every other launch sees sched = nullptr and runs worlds in identity order.
  // MJW_WORLD_ORDER=0 disables it (A/B measurements).
  static const bool order_on = [] {
    const char* e = getenv("MJW_WORLD_ORDER");
    return !(e && e[0] == '0');
  }();
  const bool order = order_on && full && d->sched && dense_ok(m, d);
  if ((stages & ST_POS) && !(stages & ST_POOL)) {
    rc = set_err(reset_counters(d, s, order), name);
    if (rc) return rc;
  }
  // every launch below sees the world orders only when this call built them (the generic path and
  // the stage launches run the worlds in identity order)
  mjw_data_t dv = *d;
  if (!order) dv.sched = nullptr;
  d = &dv;
  if (dense_ok(m, d) && !acc_sensors && stages == (ST_POS | ST_VEL | ST_ACT | ST_ACC | ST_SOLVE | ST_EULER) && !g_ev[0]) {
    const int r = step_fused(m, d, s, name);
    if (r != kNotFused) return r;
  }
  if (dense_ok(m, d)) {
    // generic kernel up to qfrc_smooth, then the dense factor / solve / euler kernel, for the
    // world range [w0, w0 + cnt) on stream st; `timed` records the optional bench events.
    // (Measured and dropped, DESIGN 4: a two-stream split of one batch inside the step -- the join
    // that ends the step serialises the halves' tails again -- and one fused forward + dense
    // kernel -- 128 VGPRs then spill in the solver loop, 0.637 vs 0.598 ms per step.)
    auto pipeline = [&](hipStream_t st, int w0, int cnt, bool timed) -> int {
      int r = 0;
      if (timed && g_ev[0]) (void)hipEventRecord(g_ev[0], st);
      switch (stages & (ST_POS | ST_VEL | ST_ACT | ST_ACC)) {
        case 0: break;
        case ST_POS | ST_VEL | ST_ACT | ST_ACC: r = launch_generic<ST_POS | ST_VEL | ST_ACT | ST_ACC | ST_NOFACTOR>(m, d, st, name, w0, cnt); break;
        case ST_POS:
          r = (stages & ST_POOL) ? launch_generic<ST_POS | ST_POOL>(m, d, st, name, w0, cnt) : launch_generic<ST_POS>(m, d, st, name, w0, cnt);
          break;
        case ST_VEL: r = launch_generic<ST_VEL>(m, d, st, name, w0, cnt); break;
        case ST_ACT: r = launch_generic<ST_ACT>(m, d, st, name, w0, cnt); break;
        case ST_ACC: r = launch_generic<ST_ACC | ST_NOFACTOR>(m, d, st, name, w0, cnt); break;
        default: g_err = std::string(name) + ": unsupported stage group"; return -4;
      }
      if (r) return r;
      if (timed && g_ev[1]) (void)hipEventRecord(g_ev[1], st);
      int f = ((stages & ST_ACC) ? DF_FACTOR : 0) | ((stages & ST_SOLVE) ? DF_SOLVE : 0) | ((stages & ST_EULER) ? DF_EULER : 0);
      if (acc_sensors) {
        // sensor_pos / _vel / _acc sit before the integrator (forward.py:981-998, step :1003-1018)
        r = set_err((hipError_t)dense_launch(f & ~DF_EULER, m, d, st, w0, cnt), name);
        if (!r) r = set_err((hipError_t)sensor_launch(m, d, st, 7, w0, cnt), name);
        if (!r && (f & DF_EULER)) r = set_err((hipError_t)dense_launch(DF_EULER, m, d, st, w0, cnt), name);
      } else if (f != 0) {
        r = set_err((hipError_t)dense_launch(f, m, d, st, w0, cnt), name);
      }
      if (timed && g_ev[2]) (void)hipEventRecord(g_ev[2], st);
      return r;
    };
    return pipeline(s, 0, d->nworld, true);
  }
  if (acc_sensors) {
    rc = launch_generic<ST_POS | ST_VEL | ST_ACT | ST_ACC | ST_SOLVE>(m, d, s, name);
    if (!rc) rc = set_err((hipError_t)sensor_launch(m, d, s), name);
    if (!rc && (stages & ST_EULER)) rc = launch_generic<ST_EULER>(m, d, s, name);
    return rc;
  }
  switch (stages) {
    case ST_POS | ST_VEL | ST_ACT | ST_ACC | ST_SOLVE | ST_EULER: return launch_generic<ST_POS | ST_VEL | ST_ACT | ST_ACC | ST_SOLVE | ST_EULER>(m, d, s, name);
    case ST_POS | ST_VEL | ST_ACT | ST_ACC | ST_SOLVE: return launch_generic<ST_POS | ST_VEL | ST_ACT | ST_ACC | ST_SOLVE>(m, d, s, name);
    case ST_POS: return launch_generic<ST_POS>(m, d, s, name);
    case ST_POS | ST_POOL: return launch_generic<ST_POS | ST_POOL>(m, d, s, name);
    case ST_VEL: return launch_generic<ST_VEL>(m, d, s, name);
    case ST_ACT: return launch_generic<ST_ACT>(m, d, s, name);
    case ST_ACC: return launch_generic<ST_ACC>(m, d, s, name);
    case ST_SOLVE: return launch_generic<ST_SOLVE>(m, d, s, name);
    case ST_EULER: return launch_generic<ST_EULER>(m, d, s, name);
    default: g_err = std::string(name) + ": unsupported stage group"; return -4;
  }
}

constexpr int ST_FORWARD = mjw::ST_POS | mjw::ST_VEL | mjw::ST_ACT | mjw::ST_ACC | mjw::ST_SOLVE;

// forward.py:457-491 rungekutta4, after `forward` ran on the current state: three more forward
// passes at the perturbed states, each followed by the accumulation of its stage derivative
int rungekutta4(const mjw_model_t* m, const mjw_data_t* d, void* stream, const char* name) {
  using namespace mjw;
  hipStream_t s = (hipStream_t)stream;
  const float A[3] = {0.5f, 0.5f, 1.0f};
  const float B[4] = {1.0f / 6.0f, 1.0f / 3.0f, 1.0f / 3.0f, 1.0f / 6.0f};
  int rc = set_err((hipError_t)rk4_launch(m, d, s, RK_BEGIN, B[0]), name);
  for (int i = 0; i < 3 && !rc; i++) {
    rc = set_err((hipError_t)rk4_launch(m, d, s, RK_PERTURB, A[i]), name);
    if (!rc) rc = run(m, d, stream, ST_FORWARD, name);
    if (!rc) rc = set_err((hipError_t)rk4_launch(m, d, s, RK_ACCUM, B[i + 1]), name);
  }
  return rc ? rc : set_err((hipError_t)rk4_launch(m, d, s, RK_END, 0.0f), name);
}

// forward.py:1003-1018 step: forward, then the integrator the model selects
int step(const mjw_model_t* m, const mjw_data_t* d, void* stream, const char* name) {
  if (m && d && m->opt_integrator == mjw::INT_RK4) {
    const int rc = run(m, d, stream, ST_FORWARD, name);
    return rc ? rc : rungekutta4(m, d, stream, name);
  }
  return run(m, d, stream, ST_FORWARD | mjw::ST_EULER, name);
}
}  // namespace

MJW_PROF_READER(mjw_prof_read)
MJW_WLOG_SETTER(mjw_prof_wlog_fwd)

extern "C" {

int mjw_abi_version(void) { return MJW_ABI_VERSION; }
const char* mjw_last_error(void) { return g_err.c_str(); }
int mjw_sizeof_model(void) { return (int)sizeof(mjw_model_t); }
int mjw_sizeof_data(void) { return (int)sizeof(mjw_data_t); }
int mjw_lds_bytes(const mjw_model_t* m, int njmax) {
  // per-world dynamic LDS of the forward kernel mjw_step launches (direct layout on the dense path)
  if (m->is_sparse) return 0;  // the sparse path keeps world state in HBM
  return mjw::make_layout(*m, njmax, m->nv <= 32 && njmax <= 64).total * 4;
}

int mjw_step(const mjw_model_t* m, const mjw_data_t* d, void* stream) { return step(m, d, stream, "mjw_step"); }
int mjw_rungekutta4(const mjw_model_t* m, const mjw_data_t* d, void* stream) {
  if (!m || !d) { g_err = "mjw_rungekutta4: null model/data"; return -1; }
  return rungekutta4(m, d, stream, "mjw_rungekutta4");
}
int mjw_rk4_op(const mjw_model_t* m, const mjw_data_t* d, int op, float scale, void* stream) {
  if (!m || !d) { g_err = "mjw_rk4_op: null model/data"; return -1; }
  if (op < mjw::RK_BEGIN || op > mjw::RK_END) { g_err = "mjw_rk4_op: op must be 0..3"; return -4; }
  return set_err((hipError_t)mjw::rk4_launch(m, d, (hipStream_t)stream, op, scale), "mjw_rk4_op");
}
int mjw_step_events(const mjw_model_t* m, const mjw_data_t* d, void* stream, void* ev_begin, void* ev_mid, void* ev_end) {
  g_ev[0] = (hipEvent_t)ev_begin;
  g_ev[1] = (hipEvent_t)ev_mid;
  g_ev[2] = (hipEvent_t)ev_end;
  int rc = step(m, d, stream, "mjw_step_events");
  g_ev[0] = g_ev[1] = g_ev[2] = nullptr;
  return rc;
}
int mjw_step_trace(const mjw_model_t* m, const mjw_data_t* d, void* stream, void** events, int nevents, int* kernel_ids,
                   int* nlaunch) {
  if (!events || nevents < 1 || !kernel_ids || !nlaunch) { g_err = "mjw_step_trace: need events[>=1], kernel_ids, nlaunch"; return -1; }
  mjw::LaunchTrace t{(hipEvent_t*)events, kernel_ids, nevents - 1, 0};
  (void)hipEventRecord((hipEvent_t)events[0], (hipStream_t)stream);
  mjw::g_trace = &t;
  int rc = step(m, d, stream, "mjw_step_trace");
  mjw::g_trace = nullptr;
  *nlaunch = t.n;
  return rc;
}
// names as rocprofv3 demangles them (numeric template arguments: SP_POS_A = 256, SP_COLL = 1024,
// SP_CON = 2048, ST_VEL = 2), so that traced launches and PMC summaries key on the same string
const char* mjw_kernel_name(int id) {
  static const char* misc[] = {"mjw::reset_counters_kernel", "mjw::ctrl_noise_kernel", "mjw::ccd_kernel", "mjw::sensor_acc_kernel",
                               "mjw::rk4_kernel", "mjw::sp::forward_kernel<256>", "mjw::sp::ccd_kernel",
                               "mjw::sp::forward_kernel<1024>", "mjw::sp::forward_kernel<2048>", "mjw::sp::forward_kernel<2>",
                               "mjw::sp::solve_kernel<0>", "mjw::sp::solve_kernel<1>", "mjw::sp::solve_kernel<2>", "mjw::sp::euler_kernel",
                               "mjw::ccd_hf_kernel", "mjw::sensor_coll_kernel", "mjw::sp::ccd_hf_kernel"};
  static thread_local char buf[64];
  if (id >= 0 && id < (int)(sizeof(misc) / sizeof(misc[0]))) return misc[id];
  if (id >= mjw::K_STEP && id < mjw::K_STEP + 8) {
    const int k = id - mjw::K_STEP;
    snprintf(buf, sizeof(buf), "mjw::step_kernel<79, %s, 7, %s, %d>", (k & 2) ? "true" : "false", (k & 1) ? "true" : "false", (k & 4) ? 16 : 28);
    return buf;
  }
  if (id >= mjw::K_DENSE && id < mjw::K_DENSE + 96) {
    const int k = (id - mjw::K_DENSE) & 31, nb[3] = {32, 16, 28};
    snprintf(buf, sizeof(buf), "mjw::dense_kernel<%d, %s, %s, %d>", k >> 2, (k & 1) ? "true" : "false", (k & 2) ? "true" : "false",
             nb[(id - mjw::K_DENSE) >> 5]);
    return buf;
  }
  if (id >= mjw::K_FWD && id < mjw::K_END) {
    snprintf(buf, sizeof(buf), "mjw::mjw_kernel<%d, %s, %s>", (id - mjw::K_FWD) >> 2, (id & 2) ? "true" : "false", (id & 1) ? "true" : "false");
    return buf;
  }
  return "unknown";
}
// one stage of every world (sub_kernel); the stages the step fuses, launched on their own for the reference's
// stage functions.  BODY transmissions accumulate over the position stage's contacts, so the transmission
// stage of a model with them is the caller's full position launch (stages.py).
int mjw_stage(const mjw_model_t* m, const mjw_data_t* d, int stage, void* stream) {
  using namespace mjw;
  if (!m || !d) { g_err = "mjw_stage: null model/data"; return -1; }
  if (m->is_sparse || m->nv > 64 || m->nbody > 4096) { g_err = "mjw_stage: dense-path models only"; return -2; }
  if (stage == SUB_TRANSMISSION && m->nbodytrn) { g_err = "mjw_stage: BODY transmissions need the position launch"; return -4; }
  if (d->nworld <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const Lay L = make_layout(*m, d->njmax, false);
  const size_t lds = (size_t)L.total * 4;
  if (lds > 160 * 1024) { g_err = "mjw_stage: per-world LDS working set exceeds 160 KiB"; return -3; }
  if (stage == SUB_MAKE_CONSTRAINT) {
    const int rc = set_err((hipError_t)pool_ranges_launch(d, s), "mjw_stage");
    if (rc) return rc;
  }
#define MJW_SUB_CASE(K)                                                                                                   \
  case K: {                                                                                                                \
    static std::once_flag once;                                                                                            \
    std::call_once(once, [] { (void)hipFuncSetAttribute((const void*)sub_kernel<K>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); }); \
    hipLaunchKernelGGL(sub_kernel<K>, dim3(d->nworld), dim3(64), lds, s, *m, *d, L, 0);                                    \
    break;                                                                                                                 \
  }
  switch (stage) {
    MJW_SUB_CASE(SUB_KINEMATICS)
    MJW_SUB_CASE(SUB_COM_POS)
    MJW_SUB_CASE(SUB_CAMLIGHT)
    MJW_SUB_CASE(SUB_TENDON)
    MJW_SUB_CASE(SUB_CRB)
    MJW_SUB_CASE(SUB_MAKE_CONSTRAINT)
    MJW_SUB_CASE(SUB_TRANSMISSION)
    MJW_SUB_CASE(SUB_COM_VEL)
    MJW_SUB_CASE(SUB_PASSIVE)
    MJW_SUB_CASE(SUB_RNE)
    default: g_err = "mjw_stage: unknown stage id"; return -4;
  }
#undef MJW_SUB_CASE
  return set_err(hipGetLastError(), "mjw_stage");
}

int mjw_forward(const mjw_model_t* m, const mjw_data_t* d, void* stream) {
  return run(m, d, stream, mjw::ST_POS | mjw::ST_VEL | mjw::ST_ACT | mjw::ST_ACC | mjw::ST_SOLVE, "mjw_forward");
}
int mjw_fwd_position(const mjw_model_t* m, const mjw_data_t* d, void* stream) {
  return run(m, d, stream, mjw::ST_POS, "mjw_fwd_position");
}
int mjw_contact_rows(const mjw_model_t* m, const mjw_data_t* d, void* stream) {
  if (m && d && !m->is_sparse && d->nworld > 0) {
    const int rc = set_err((hipError_t)mjw::pool_ranges_launch(d, (hipStream_t)stream), "mjw_contact_rows");
    if (rc) return rc;
  }
  return run(m, d, stream, mjw::ST_POS | mjw::ST_POOL, "mjw_contact_rows");
}
int mjw_fwd_velocity(const mjw_model_t* m, const mjw_data_t* d, void* stream) {
  return run(m, d, stream, mjw::ST_VEL, "mjw_fwd_velocity");
}
int mjw_fwd_actuation(const mjw_model_t* m, const mjw_data_t* d, void* stream) {
  return run(m, d, stream, mjw::ST_ACT, "mjw_fwd_actuation");
}
int mjw_fwd_acceleration(const mjw_model_t* m, const mjw_data_t* d, void* stream) {
  return run(m, d, stream, mjw::ST_ACC, "mjw_fwd_acceleration");
}
int mjw_solve(const mjw_model_t* m, const mjw_data_t* d, void* stream) {
  return run(m, d, stream, mjw::ST_SOLVE, "mjw_solve");
}
int mjw_euler(const mjw_model_t* m, const mjw_data_t* d, void* stream) {
  return run(m, d, stream, mjw::ST_EULER, "mjw_euler");
}

int mjw_actuator_map(const mjw_model_t* m, const mjw_data_t* d, void* stream) {
  if (!m || !d) { g_err = "mjw_actuator_map: null model/data"; return -1; }
  if (d->nworld <= 0) return 0;
  // layout-independent: the moment rows (rowadr / rownnz / colind) are the same on the sparse path
  hipLaunchKernelGGL(mjw::actuator_map_kernel, dim3(d->nworld), dim3(64), 0, (hipStream_t)stream, *m, *d);
  return set_err(hipGetLastError(), "mjw_actuator_map");
}

int mjw_nxn_broadphase(const mjw_model_t* m, const mjw_data_t* d, int* collision_pair, int* collision_pairid, int* collision_worldid,
                       void* stream) {
  const long n = (long)d->nworld * m->nxn;
  if (n <= 0) return 0;
  if (!collision_pair || !collision_pairid || !collision_worldid) return set_err(hipErrorInvalidValue, "mjw_nxn_broadphase: null context array");
  hipLaunchKernelGGL(mjw::nxn_broadphase_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *m, *d, collision_pair,
                     collision_pairid, collision_worldid);
  return set_err(hipGetLastError(), "mjw_nxn_broadphase");
}

int mjw_sap_broadphase(const mjw_model_t* m, const mjw_data_t* d, int* collision_pair, int* collision_pairid, int* collision_worldid,
                       void* stream) {
  if (d->nworld <= 0 || m->nxn <= 0) return 0;
  if (!collision_pair || !collision_pairid || !collision_worldid) return set_err(hipErrorInvalidValue, "mjw_sap_broadphase: null context array");
  if (m->ngeom > mjw::SAP_MAX_GEOM) {
    g_err = "mjw_sap_broadphase: more than " + std::to_string(mjw::SAP_MAX_GEOM) + " geoms (the LDS sort)";
    return -2;
  }
  int np2 = 1;
  while (np2 < m->ngeom) np2 <<= 1;
  const size_t lds = (size_t)(2 * np2 + m->ngeom) * 4;
  static std::once_flag once;
  std::call_once(once, [] {
    (void)hipFuncSetAttribute((const void*)mjw::sap_broadphase_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  });
  hipLaunchKernelGGL(mjw::sap_broadphase_kernel, dim3(d->nworld), dim3(256), lds, (hipStream_t)stream, *m, *d, collision_pair, collision_pairid,
                     collision_worldid);
  return set_err(hipGetLastError(), "mjw_sap_broadphase");
}

int mjw_primitive_narrowphase(const mjw_model_t* m, const mjw_data_t* d, const int* collision_pair, const int* collision_pairid,
                              const int* collision_worldid, unsigned long long typemask, void* stream) {
  if (d->naconmax <= 0) return 0;
  if (!collision_pair || !collision_pairid || !collision_worldid) return set_err(hipErrorInvalidValue, "mjw_primitive_narrowphase: null context array");
  hipLaunchKernelGGL(mjw::primitive_narrowphase_kernel, dim3((d->naconmax + 255) / 256), dim3(256), 0, (hipStream_t)stream, *m, *d, collision_pair,
                     collision_pairid, collision_worldid, typemask);
  return set_err(hipGetLastError(), "mjw_primitive_narrowphase");
}

int mjw_ctrl_noise(const mjw_model_t* m, const mjw_data_t* d, const float* center, int step, float std, float rate, void* stream) {
  int n = d->nworld * m->nu;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(mjw::ctrl_noise_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, *m, *d, center, step, std, rate);
  mjw::trace_launch((hipStream_t)stream, mjw::K_CTRL_NOISE);
  return set_err(hipGetLastError(), "mjw_ctrl_noise");
}

}  // extern "C"
