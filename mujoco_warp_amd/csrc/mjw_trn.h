// mjw_trn.h -- the site-based transmissions of the world-per-wavefront path (smooth.py:2150-2241
// SLIDERCRANK, 2274-2442 SITE) and the contact-driven BODY transmission of adhesion actuators
// (smooth.py:2260-2273, 2448-2602).
//
// A site transmission's moment row spans the dof chains of its sites' weld bodies: one lane per actuator
// walks them deepest dof first, as the reference does, and writes the row ascending.  The BODY moment is
// minus the mean, over the contacts touching the body, of the contact normal's Jacobian row.  The
// reference reads it back from the contact's constraint rows (the pyramid rows' weighted sum, or the
// normal row) or, for contacts outside the margin, from n . (J(pos, b2) - J(pos, b1)); all three equal
// n . (J(pos, b2) - J(pos, b1)), which the collision stage accumulates per actuator while the contact is
// staged (body_trn_contact) and the transmission stage scales (body_trn_finish).
#pragma once
#include "mjw_common.h"

namespace mjw {

// support.py:397-432 (jac_dof): column `dof` of the point Jacobian of `body`, zero unless the dof moves it
__device__ __forceinline__ void trn_jac_dof(const mjw_model_t& m, const float* subtree_com, const float* cdof, const float* pnt, int body,
                                            int dof, float* jp, float* jr) {
  const int db = m.dof_bodyid[dof];
  bool in_tree = db == 0;
  for (int b = body; b != 0 && !in_tree; b = m.body_parentid[b]) in_tree = b == db;
  if (!in_tree) {
    jp[0] = jp[1] = jp[2] = jr[0] = jr[1] = jr[2] = 0.0f;
    return;
  }
  const float* sc = subtree_com + 3 * m.body_rootid[body];
  const float off[3] = {pnt[0] - sc[0], pnt[1] - sc[1], pnt[2] - sc[2]};
  const float* cd = cdof + 6 * dof;
  float c[3];
  cross3(c, cd, off);
  for (int i = 0; i < 3; i++) { jp[i] = cd[3 + i] + c[i]; jr[i] = cd[i]; }
}

__device__ __forceinline__ int trn_last_dof(const mjw_model_t& m, int body) {
  return body > 0 ? m.body_dofadr[body] + m.body_dofnum[body] - 1 : -1;
}

// moment row length of a SITE / SLIDERCRANK / BODY actuator (io.py _mom_nnz counts the same on the host)
__device__ __forceinline__ int trn_site_nnz(const mjw_model_t& m, int a) {
  const int trn = m.actuator_trntype[a];
  if (trn == TRN_BODY) return m.nv;
  const int i1 = m.actuator_trnid[2 * a], i2 = m.actuator_trnid[2 * a + 1];
  int d1 = trn_last_dof(m, m.body_weldid[m.site_bodyid[i1]]);
  int d2 = i2 >= 0 ? trn_last_dof(m, m.body_weldid[m.site_bodyid[i2]]) : -1;
  int n = 0;
  while (d1 >= 0 || d2 >= 0) {
    const int da = max(d1, d2);
    if (trn == TRN_SITE && i2 >= 0 && d1 == da && d2 == da) break;
    n++;
    if (d1 == da) d1 = m.dof_parentid[d1];
    if (d2 == da) d2 = m.dof_parentid[d2];
  }
  return n;
}

// one SITE / SLIDERCRANK actuator (the calling lane's): length and moment row; mom / momdof: the
// actuator's LDS slots (nnz of them, ascending dofs); gm / gc: its global moment / colind row
__device__ __forceinline__ float trn_site(const mjw_model_t& m, int wid, int a, int nnz, const float* site_xpos, const float* site_xmat,
                                          const float* xquat, const float* subtree_com, const float* cdof, float* mom, int* momdof, float* gm,
                                          int* gc) {
  const float* gear = MR(actuator_gear) + 6 * a;
  const int trn = m.actuator_trntype[a], id = m.actuator_trnid[2 * a], id2 = m.actuator_trnid[2 * a + 1];
  const float* sx = site_xpos + 3 * id;
  float jp[3], jr[3], jp2[3], jr2[3];
  int ptr = nnz - 1;
  auto emit = [&](int da, float v) {
    mom[ptr] = v;
    momdof[ptr] = da;
    gm[ptr] = v;
    gc[ptr] = da;
    ptr--;
  };
  if (trn == TRN_SLIDERCRANK) {
    const float rod = MR(actuator_cranklength)[a];
    const float* sm = site_xmat + 9 * id2;
    const float* sx2 = site_xpos + 3 * id2;
    const float axis[3] = {sm[2], sm[5], sm[8]};
    const float vec[3] = {sx[0] - sx2[0], sx[1] - sx2[1], sx[2] - sx2[2]};
    const float av = dot3(vec, axis), det = av * av + rod * rod - dot3(vec, vec);
    const bool ok = det > 0.0f;
    const float sdet = ok ? sqrtf(det) : 0.0f;
    const float length = ok ? av - sdet : av;
    float dldv[3], dlda[3];
    const float sc = ok ? 1.0f - av / (sdet != 0.0f ? sdet : MJW_MINVAL) : 0.0f;
    for (int i = 0; i < 3; i++) {
      dldv[i] = ok ? axis[i] * sc + vec[i] / (sdet != 0.0f ? sdet : MJW_MINVAL) : axis[i];
      dlda[i] = ok ? vec[i] * sc : vec[i];
    }
    int d1 = trn_last_dof(m, m.body_weldid[m.site_bodyid[id]]), d2 = trn_last_dof(m, m.body_weldid[m.site_bodyid[id2]]);
    while (d1 >= 0 || d2 >= 0) {
      const int da = max(d1, d2);
      float jacA[3];
      trn_jac_dof(m, subtree_com, cdof, sx2, m.site_bodyid[id2], da, jp2, jr2);
      cross3(jacA, jr2, axis);
      trn_jac_dof(m, subtree_com, cdof, sx, m.site_bodyid[id], da, jp, jr);
      const float jac[3] = {jp[0] - jp2[0], jp[1] - jp2[1], jp[2] - jp2[2]};
      emit(da, (dot3(dlda, jacA) + dot3(dldv, jac)) * gear[0]);
      if (d1 == da) d1 = m.dof_parentid[d1];
      if (d2 == da) d2 = m.dof_parentid[d2];
    }
    return length * gear[0];
  }
  if (id2 < 0) {  // the wrench in the global frame, no length
    const float* sm = site_xmat + 9 * id;
    float wt[3], wr[3];
    matvec3(wt, sm, gear);
    matvec3(wr, sm, gear + 3);
    for (int da = trn_last_dof(m, m.body_weldid[m.site_bodyid[id]]); da >= 0; da = m.dof_parentid[da]) {
      trn_jac_dof(m, subtree_com, cdof, sx, m.site_bodyid[id], da, jp, jr);
      emit(da, dot3(jp, wt) + dot3(jr, wr));
    }
    return 0.0f;
  }
  const int body = m.site_bodyid[id], bref = m.site_bodyid[id2];
  const float* rx = site_xpos + 3 * id2;
  const float* rm = site_xmat + 9 * id2;
  const bool tr = gear[0] != 0.0f || gear[1] != 0.0f || gear[2] != 0.0f;
  const bool rot = gear[3] != 0.0f || gear[4] != 0.0f || gear[5] != 0.0f;
  float length = 0.0f, wt[3] = {0.0f, 0.0f, 0.0f}, wr[3] = {0.0f, 0.0f, 0.0f};
  if (tr) {
    const float dx[3] = {sx[0] - rx[0], sx[1] - rx[1], sx[2] - rx[2]};
    float vec[3];
    for (int i = 0; i < 3; i++) vec[i] = rm[i] * dx[0] + rm[3 + i] * dx[1] + rm[6 + i] * dx[2];
    length += dot3(vec, gear);
    matvec3(wt, rm, gear);
  }
  if (rot) {
    const float* squat = MR(site_quat);
    float q[4], qr[4], vec[3];
    mul_quat(q, squat + 4 * id, xquat + 4 * body);  // smooth.py:2375-2376 multiplies in this order
    mul_quat(qr, squat + 4 * id2, xquat + 4 * bref);
    quat_sub(vec, q, qr);
    length += dot3(vec, gear + 3);
    matvec3(wr, rm, gear + 3);
  }
  int d1 = trn_last_dof(m, m.body_weldid[body]), d2 = trn_last_dof(m, m.body_weldid[bref]);
  while (d1 >= 0 || d2 >= 0) {
    const int da = max(d1, d2);
    if (d1 == da && d2 == da) break;
    trn_jac_dof(m, subtree_com, cdof, sx, body, da, jp, jr);
    trn_jac_dof(m, subtree_com, cdof, rx, bref, da, jp2, jr2);
    float v = 0.0f;
    for (int i = 0; i < 3; i++) {
      if (tr) v += (jp[i] - jp2[i]) * wt[i];
      if (rot) v += (jr[i] - jr2[i]) * wr[i];
    }
    emit(da, v);
    if (d1 == da) d1 = m.dof_parentid[d1];
    if (d2 == da) d2 = m.dof_parentid[d2];
  }
  return length;
}

// BODY transmissions, before the collision stage: zero each actuator's accumulator row (its LDS moment
// slots) and contact count (its LDS nnz slot)
__device__ __forceinline__ void body_trn_init(const mjw_model_t& m, float* act_mom, int* act_nnz, int amax, int lane) {
  for (int a = 0; a < m.nu; a++) {
    if (m.actuator_trntype[a] != TRN_BODY) continue;
    for (int i = lane; i < amax; i += 64) act_mom[amax * a + i] = 0.0f;
    if (lane == 0) act_nnz[a] = 0;
  }
}

// one staged contact (geoms g1 / g2 of bodies cb1 / cb2 -- their weld bodies wb1 / wb2 and roots r1 / r2
// give the same Jacobian): lane i adds n . (J(pos, b2) - J(pos, b1)) at dof i to every BODY actuator on
// either body.  The caller loops over contacts in order, so each (actuator, dof) slot has one writer.
__device__ __forceinline__ void body_trn_contact(const mjw_model_t& m, const float* subtree_com, const float* cdof, const float* pos,
                                                 const float* n, int cb1, int cb2, float* act_mom, int* act_nnz, int amax, int lane) {
  for (int a = 0; a < m.nu; a++) {
    if (m.actuator_trntype[a] != TRN_BODY) continue;
    const int body = m.actuator_trnid[2 * a];
    if (cb1 != body && cb2 != body) continue;
    if (lane < m.nv) {
      float j1[3], j2[3], r[3];
      trn_jac_dof(m, subtree_com, cdof, pos, cb1, lane, j1, r);
      trn_jac_dof(m, subtree_com, cdof, pos, cb2, lane, j2, r);
      act_mom[amax * a + lane] += n[0] * (j2[0] - j1[0]) + n[1] * (j2[1] - j1[1]) + n[2] * (j2[2] - j1[2]);
    }
    if (lane == 0) act_nnz[a] += 1;
  }
}

}  // namespace mjw
