// mjw_rk4.hip -- the classic 4th-order Runge-Kutta integrator (forward.py:357-492).
//
// RK4 re-runs `forward` at three perturbed states; the forward passes are the regular fused
// launches (mjw_step.hip / mjw_dense.hip), and the state bookkeeping between them is this kernel:
// one 64-lane wave per world, lanes over dofs / joints / activations, one launch per RK stage op.
// The scratch state (t0 copies and the weighted sums) lives in Data (qpos_t0 ... act_dot_rk, allocated by
// make_data), so the library still allocates nothing.

#include "mjw_common.h"

namespace mjw {


// forward.py:51-109 _next_position: qpos_out = qpos_in (+) dt * scale * qvel (quaternions integrated)
__device__ __forceinline__ void next_position(const mjw_model_t& m, int wid, int lane, const float* qpos_in, const float* qvel, float scale,
                                              float* qpos_out) {
  const float dt = MR(opt_timestep)[0];
  for (int j = lane; j < m.njnt; j += LPW) {
    const int qa = m.jnt_qposadr[j], da = m.jnt_dofadr[j], jt = m.jnt_type[j];
    if (jt == JNT_FREE) {
      float q[4], qn[4], w[3];
      for (int i = 0; i < 3; i++) qpos_out[qa + i] = qpos_in[qa + i] + dt * (qvel[da + i] * scale);
      for (int i = 0; i < 4; i++) q[i] = qpos_in[qa + 3 + i];
      for (int i = 0; i < 3; i++) w[i] = qvel[da + 3 + i] * scale;
      quat_integrate(qn, q, w, dt);
      for (int i = 0; i < 4; i++) qpos_out[qa + 3 + i] = qn[i];
    } else if (jt == JNT_BALL) {
      float q[4], qn[4], w[3];
      for (int i = 0; i < 4; i++) q[i] = qpos_in[qa + i];
      for (int i = 0; i < 3; i++) w[i] = qvel[da + i] * scale;
      quat_integrate(qn, q, w, dt);
      for (int i = 0; i < 4; i++) qpos_out[qa + i] = qn[i];
    } else {
      qpos_out[qa] = qpos_in[qa] + dt * qvel[da] * scale;
    }
  }
}

__global__ void __launch_bounds__(64) rk4_kernel(const mjw_model_t m, const mjw_data_t d, int op, float scale) {
  const int wid = blockIdx.x, lane = threadIdx.x & 63;
  if (wid >= d.nworld) return;
  const int nq = m.nq, nv = m.nv, na = m.na;
  const float dt = MR(opt_timestep)[0];
  float* qpos = d.qpos + (long)wid * nq;
  float* qvel = d.qvel + (long)wid * nv;
  const float* qacc = d.qacc + (long)wid * nv;
  float* act = d.act + (long)wid * na;
  float* act_dot = d.act_dot + (long)wid * na;
  float* qpos0 = d.qpos_t0 + (long)wid * nq;
  float* qvel0 = d.qvel_t0 + (long)wid * nv;
  float* qvel_rk = d.qvel_rk + (long)wid * nv;
  float* qacc_rk = d.qacc_rk + (long)wid * nv;
  float* act0 = d.act_t0 + (long)wid * na;
  float* act_dot_rk = d.act_dot_rk + (long)wid * na;
  if (op == RK_BEGIN) {  // forward.py:464-476: t0 copies, then accumulate B[0]
    for (int i = lane; i < nq; i += LPW) qpos0[i] = qpos[i];
    for (int i = lane; i < nv; i += LPW) {
      qvel0[i] = qvel[i];
      qvel_rk[i] = scale * qvel[i];
      qacc_rk[i] = scale * qacc[i];
    }
    for (int i = lane; i < na; i += LPW) {
      act0[i] = act[i];
      act_dot_rk[i] = scale * act_dot[i];
    }
  } else if (op == RK_PERTURB) {  // forward.py:357-399 _rk_perturb_state
    next_position(m, wid, lane, qpos0, qvel, scale, qpos);  // uses the current qvel: before it changes
    __syncthreads();
    for (int i = lane; i < nv; i += LPW) qvel[i] = qvel0[i] + scale * qacc[i] * dt;
    for (int u = lane; u < m.nu; u += LPW) {
      const int adr = m.actuator_actadr[u];
      for (int j = adr; adr >= 0 && j < adr + m.actuator_actnum[u]; j++) act[j] = next_act(dt, m.actuator_dyntype[u], MR(actuator_dynprm)[10 * u], MR(actuator_actrange) + 2 * u, act0[j], act_dot[j], scale, false);
    }
  } else if (op == RK_ACCUM) {  // forward.py:402-440 _rk_accumulate
    for (int i = lane; i < nv; i += LPW) {
      qvel_rk[i] += scale * qvel[i];
      qacc_rk[i] += scale * qacc[i];
    }
    for (int i = lane; i < na; i += LPW) act_dot_rk[i] += scale * act_dot[i];
  } else {  // forward.py:484-492 restore t0, then _advance(m, d, qacc_rk, qvel_rk) :213-274
    for (int i = lane; i < na; i += LPW) { act[i] = act0[i]; act_dot[i] = act_dot_rk[i]; }
    __syncthreads();
    for (int u = lane; u < m.nu; u += LPW) {
      const int adr = m.actuator_actadr[u];
      for (int j = adr; adr >= 0 && j < adr + m.actuator_actnum[u]; j++)
        act[j] = next_act(dt, m.actuator_dyntype[u], MR(actuator_dynprm)[10 * u], MR(actuator_actrange) + 2 * u, act[j], act_dot[j], 1.0f,
                          m.actuator_actlimited[u] != 0);
    }
    for (int i = lane; i < nv; i += LPW) {
      qvel[i] = qvel0[i] + qacc_rk[i] * dt;
      d.qacc_warmstart[(long)wid * nv + i] = qacc[i];
    }
    next_position(m, wid, lane, qpos0, qvel_rk, 1.0f, qpos);
    if (lane == 0) d.time[wid] += dt;
  }
}

int rk4_launch(const mjw_model_t* m, const mjw_data_t* d, hipStream_t s, int op, float scale) {
  if (d->nworld <= 0) return 0;
  hipLaunchKernelGGL(rk4_kernel, dim3(d->nworld), dim3(64), 0, s, *m, *d, op, scale);
  trace_launch(s, K_RK4);
  return (int)hipGetLastError();
}

}  // namespace mjw
