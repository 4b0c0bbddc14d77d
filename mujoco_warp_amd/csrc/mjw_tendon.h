// mjw_tendon.h -- fixed (joint) tendons on the world-per-wavefront path: length and sparse Jacobian
// (smooth.py:3085-3121), armature in qM (smooth.py:916-1000), velocity (forward.py:604-609), spring /
// damper (passive.py:183-252), friction and limit rows (constraint.py:1204-1313, 1547-1665), tendon
// transmissions (smooth.py:2244-2260) and the tendon actuator force range (forward.py:739-779).
//
// A fixed tendon's Jacobian is its wrap coefficients at the joints' dofs, the same in every world, so
// the helpers recompute lengths and coefficients from the model and the world's qpos / qvel in LDS
// instead of keeping per-stage copies; every routine is a no-op for models without tendons (ntendon = 0
// is a wave-uniform branch), which keeps the hot kernels' registers untouched.
#pragma once
#include "mjw_common.h"

namespace mjw {

// coefficient of tendon t at dof `dof` (the last wrap on that dof's joint, as _joint_tendon writes it)
__device__ __forceinline__ float ten_coef(const mjw_model_t& m, int wid, int t, int dof) {
  float c = 0.0f;
  const float* prm = MR(wrap_prm);
  for (int w = m.tendon_adr[t]; w < m.tendon_adr[t] + m.tendon_num[t]; w++)
    if (m.jnt_dofadr[m.wrap_objid[w]] == dof) c = prm[w];
  return c;
}

// tendon length sum coef * qpos (qpos: the world's qpos in LDS)
__device__ __forceinline__ float ten_len(const mjw_model_t& m, int wid, const float* qpos, int t) {
  float L = 0.0f;
  const float* prm = MR(wrap_prm);
  for (int w = m.tendon_adr[t]; w < m.tendon_adr[t] + m.tendon_num[t]; w++) L += prm[w] * qpos[m.jnt_qposadr[m.wrap_objid[w]]];
  return L;
}

// tendon velocity J qvel over the sparse row
__device__ __forceinline__ float ten_vel(const mjw_model_t& m, int wid, const float* qvel, int t) {
  float v = 0.0f;
  for (int k = 0; k < m.ten_J_rownnz[t]; k++) {
    const int dof = m.ten_J_colind[m.ten_J_rowadr[t] + k];
    v += ten_coef(m, wid, t, dof) * qvel[dof];
  }
  return v;
}

// position stage: ten_length, ten_J (Data contract)
__device__ __forceinline__ void tendon_pos(const mjw_model_t& m, const mjw_data_t& d, const float* qpos, int wid, int lane) {
  for (int t = lane; t < m.ntendon; t += 64) {
    d.ten_length[(long)wid * m.ntendon + t] = ten_len(m, wid, qpos, t);
    for (int k = 0; k < m.ten_J_rownnz[t]; k++) {
      const int e = m.ten_J_rowadr[t] + k;
      d.ten_J[(long)wid * m.nJten + e] = ten_coef(m, wid, t, m.ten_J_colind[e]);
    }
  }
}

// qM[i][j] += armature J_i J_j for j = i or an ancestor of i (the pattern of qM), M row stride nvs;
// one tendon at a time, lanes over its (k1, k2) entry pairs (distinct (i, j) within a tendon)
__device__ __forceinline__ void tendon_armature(const mjw_model_t& m, float* M, int nvs, int wid, int lane) {
  const float* arm = MR(tendon_armature);
  for (int t = 0; t < m.ntendon; t++) {
    if (arm[t] == 0.0f) continue;
    const int rn = m.ten_J_rownnz[t], ra = m.ten_J_rowadr[t];
    for (int p = lane; p < rn * rn; p += 64) {
      const int k1 = p / rn, k2 = p - k1 * rn;
      if (k2 > k1) continue;
      const int i = m.ten_J_colind[ra + k1], j = m.ten_J_colind[ra + k2];  // colind ascending: j <= i
      int a = i;
      while (a > j) a = m.dof_parentid[a];
      if (a != j) continue;
      const float v = arm[t] * ten_coef(m, wid, t, i) * ten_coef(m, wid, t, j);
      M[i * nvs + j] += v;
      if (i != j) M[j * nvs + i] += v;
    }
    __syncthreads();
  }
}

// velocity stage: ten_velocity and the spring / damper forces added into spring[] / damper[] (LDS, nv)
__device__ __forceinline__ void tendon_passive(const mjw_model_t& m, const mjw_data_t& d, const float* qpos, const float* qvel,
                                               float* spring, float* damper, int wid, int lane) {
  for (int t = lane; t < m.ntendon; t += 64) d.ten_velocity[(long)wid * m.ntendon + t] = ten_vel(m, wid, qvel, t);
  const int dsbl_spring = m.opt_disableflags & DSBL_SPRING, dsbl_damper = m.opt_disableflags & DSBL_DAMPER;
  const float* stiff = MR(tendon_stiffness);
  const float* damp = MR(tendon_damping);
  const float* ls = MR(tendon_lengthspring);
  for (int t = 0; t < m.ntendon; t++) {
    const bool hs = stiff[t] != 0.0f && !dsbl_spring, hd = damp[t] != 0.0f && !dsbl_damper;
    if (!hs && !hd) continue;
    const float L = ten_len(m, wid, qpos, t), v = ten_vel(m, wid, qvel, t);
    const float lo = ls[2 * t], hi = ls[2 * t + 1];
    const float fs = L > hi ? stiff[t] * (hi - L) : (L < lo ? stiff[t] * (lo - L) : 0.0f);
    const float fd = -damp[t] * v;
    for (int k = lane; k < m.ten_J_rownnz[t]; k += 64) {
      const int dof = m.ten_J_colind[m.ten_J_rowadr[t] + k];
      const float J = ten_coef(m, wid, t, dof);
      if (hs) spring[dof] += J * fs;
      if (hd) damper[dof] += J * fd;
    }
    __syncthreads();
  }
}

// forward.py:739-779: scale the forces of the actuators on a force-limited tendon so that their sum
// stays in tendon_actfrcrange (force[]: this world's actuator forces in LDS)
__device__ __forceinline__ void tendon_actuator_clamp(const mjw_model_t& m, float* force, int wid, int lane) {
  const float* rng = MR(tendon_actfrcrange);
  for (int t = 0; t < m.ntendon; t++) {
    if (!m.tendon_actfrclimited[t]) continue;
    float tot = 0.0f;
    for (int a = 0; a < m.nu; a++)
      if (m.actuator_trntype[a] == 3 && m.actuator_trnid[2 * a] == t) tot += force[a];
    __syncthreads();
    for (int a = lane; a < m.nu; a += 64) {
      if (m.actuator_trntype[a] != 3 || m.actuator_trnid[2 * a] != t) continue;
      if (tot < rng[2 * t]) force[a] *= rng[2 * t] / tot;
      else if (tot > rng[2 * t + 1]) force[a] *= rng[2 * t + 1] / tot;
    }
    __syncthreads();
  }
}

}  // namespace mjw
