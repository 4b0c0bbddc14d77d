// mjw_sensor.h -- sensor evaluation shared by the forward kernel (position / velocity sensors,
// mjw_step.hip) and the post-solve kernel (rne_postconstraint + acceleration sensors,
// mjw_sensor.hip).  Restates mujoco_warp/_src/sensor.py for the supported sensor types; the
// caller passes where each frame quantity lives (LDS in the forward kernel, HBM afterwards).
#pragma once

#include "mjw_common.h"

namespace mjw {

// per-world frame sources (each a per-world base pointer)
struct Frames {
  const float *xpos, *xquat, *xmat, *xipos, *ximat, *gxpos, *gxmat, *cxpos, *cxmat, *subtree_com, *cvel;
};

// site pose from the body pose (smooth.py:205-224, same operations as kinematics)
__device__ __forceinline__ void site_pose(const mjw_model_t& m, int wid, const Frames& F, int id, float* pos, float* mat) {
  const float* site_pos = MR(site_pos);
  const float* site_quat = MR(site_quat);
  int b = m.site_bodyid[id];
  float q[4] = {F.xquat[4 * b], F.xquat[4 * b + 1], F.xquat[4 * b + 2], F.xquat[4 * b + 3]};
  float t[3], sq[4];
  rot_vec_quat(t, site_pos + 3 * id, q);
  mul_quat(sq, q, site_quat + 4 * id);
  quat_to_mat(mat, sq);
  for (int i = 0; i < 3; i++) pos[i] = F.xpos[3 * b + i] + t[i];
}

// object frame position / rotation / body (sensor.py:282-340, 1011-1050)
__device__ __forceinline__ int obj_frame(const mjw_model_t& m, int wid, const Frames& F, int type, int id, float* pos, float* mat) {
  int body = 0;
  const float *p = nullptr, *R = nullptr;
  if (type == OBJ_BODY) { p = F.xipos + 3 * id; R = F.ximat + 9 * id; body = id; }
  else if (type == OBJ_XBODY) { p = F.xpos + 3 * id; R = F.xmat + 9 * id; body = id; }
  else if (type == OBJ_GEOM) { p = F.gxpos + 3 * id; R = F.gxmat + 9 * id; body = m.geom_bodyid[id]; }
  else if (type == OBJ_CAMERA) { p = F.cxpos + 3 * id; R = F.cxmat + 9 * id; body = m.cam_bodyid[id]; }
  if (type == OBJ_SITE) {
    site_pose(m, wid, F, id, pos, mat);
    return m.site_bodyid[id];
  }
  if (p) {
    for (int i = 0; i < 3; i++) pos[i] = p[i];
    for (int i = 0; i < 9; i++) mat[i] = R[i];
  } else {
    for (int i = 0; i < 3; i++) pos[i] = 0.0f;
    for (int i = 0; i < 9; i++) mat[i] = (i % 4 == 0) ? 1.0f : 0.0f;
  }
  return body;
}

__device__ __forceinline__ void mat_t_vec(float* r, const float* M, const float* v) {
  for (int i = 0; i < 3; i++) r[i] = M[i] * v[0] + M[3 + i] * v[1] + M[6 + i] * v[2];
}

// sensor.py:54-110 _write_scalar / _write_vector
__device__ __forceinline__ void sensor_write(const mjw_model_t& m, const mjw_data_t& d, int wid, int s, const float* v, int dim) {
  const float cutoff = MR(sensor_cutoff)[s];
  const int dt = m.sensor_datatype[s];
  float* out = d.sensordata + (long)wid * m.nsensordata + m.sensor_adr[s];
  for (int i = 0; i < dim; i++) {
    float x = v[i];
    if (cutoff > 0.0f && dt == DATATYPE_REAL) x = clampf(x, -cutoff, cutoff);
    else if (cutoff > 0.0f && dt == DATATYPE_POSITIVE) x = fminf(x, cutoff);
    out[i] = x;
  }
}

// sensor.py:394-446 _frame_quat
__device__ __forceinline__ void frame_quat(const mjw_model_t& m, int wid, const Frames& F, int type, int id, float* q) {
  q[0] = 1.0f; q[1] = q[2] = q[3] = 0.0f;
  const float* xq = F.xquat;
  if (type == OBJ_BODY) mul_quat(q, xq + 4 * id, MR(body_iquat) + 4 * id);
  else if (type == OBJ_XBODY) for (int i = 0; i < 4; i++) q[i] = xq[4 * id + i];
  else if (type == OBJ_GEOM) mul_quat(q, xq + 4 * m.geom_bodyid[id], MR(geom_quat) + 4 * id);
  else if (type == OBJ_SITE) mul_quat(q, xq + 4 * m.site_bodyid[id], MR(site_quat) + 4 * id);
  else if (type == OBJ_CAMERA) mul_quat(q, xq + 4 * m.cam_bodyid[id], MR(cam_quat) + 4 * id);
}

// sensor.py:1011-1050 _cvel_offset
__device__ __forceinline__ const float* cvel_offset(const mjw_model_t& m, int wid, const Frames& F, int type, int id, float* off) {
  float p[3], R[9];
  int b = obj_frame(m, wid, F, type, id, p, R);
  const float* com = F.subtree_com + 3 * m.body_rootid[b];
  for (int i = 0; i < 3; i++) off[i] = p[i] - com[i];
  return F.cvel + 6 * b;
}

// one position- or velocity-stage sensor (sensor.py:459-706 / 1251-1373, supported types)
__device__ void sensor_posvel_one(const mjw_model_t& m, const mjw_data_t& d, int wid, const Frames& F, int s, const float* qpos,
                                  const float* qvel, const float* act_len, const float* act_vel, float time) {
  const int t = m.sensor_type[s], id = m.sensor_objid[s], ot = m.sensor_objtype[s];
  const int rid = m.sensor_refid[s], rt = m.sensor_reftype[s];
  float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  int dim = 3;
  if (t == SENS_MAGNETOMETER) {  // sensor.py:114-125
    float p[3], R[9];
    site_pose(m, wid, F, id, p, R);
    mat_t_vec(v, R, MR(opt_magnetic));
  } else if (t == SENS_JOINTPOS) {
    v[0] = qpos[m.jnt_qposadr[id]]; dim = 1;
  } else if (t == SENS_ACTUATORPOS) {
    v[0] = act_len[id]; dim = 1;
  } else if (t == SENS_BALLQUAT) {  // sensor.py:232-240
    for (int i = 0; i < 4; i++) v[i] = qpos[m.jnt_qposadr[id] + i];
    normalize4(v);
    dim = 4;
  } else if (t == SENS_FRAMEPOS) {  // sensor.py:282-338
    float p[3], R[9];
    obj_frame(m, wid, F, ot, id, p, R);
    if (rid == -1) {
      for (int i = 0; i < 3; i++) v[i] = p[i];
    } else {
      // reference branch order: the XBODY test reads objtype (sensor.py:323-326)
      int rt2 = rt == OBJ_BODY ? OBJ_BODY : (ot == OBJ_XBODY ? OBJ_XBODY : ((rt == OBJ_GEOM || rt == OBJ_SITE || rt == OBJ_CAMERA) ? rt : OBJ_UNKNOWN));
      float pr[3], Rr[9], dif[3];
      obj_frame(m, wid, F, rt2, rid, pr, Rr);
      for (int i = 0; i < 3; i++) dif[i] = p[i] - pr[i];
      mat_t_vec(v, Rr, dif);
    }
  } else if (t == SENS_FRAMEXAXIS || t == SENS_FRAMEYAXIS || t == SENS_FRAMEZAXIS) {  // sensor.py:341-391
    const int ax = t - SENS_FRAMEXAXIS;
    float p[3], R[9];
    obj_frame(m, wid, F, ot, id, p, R);
    float a[3] = {R[ax], R[3 + ax], R[6 + ax]};
    if (rid == -1) {
      for (int i = 0; i < 3; i++) v[i] = a[i];
    } else {
      float pr[3], Rr[9];
      obj_frame(m, wid, F, rt, rid, pr, Rr);
      mat_t_vec(v, Rr, a);
    }
  } else if (t == SENS_FRAMEQUAT) {  // sensor.py:394-446
    float q[4];
    frame_quat(m, wid, F, ot, id, q);
    if (rid == -1) {
      for (int i = 0; i < 4; i++) v[i] = q[i];
    } else {
      float qr[4], qi[4];
      frame_quat(m, wid, F, rt, rid, qr);
      qi[0] = qr[0]; qi[1] = -qr[1]; qi[2] = -qr[2]; qi[3] = -qr[3];
      mul_quat(v, qi, q);
    }
    dim = 4;
  } else if (t == SENS_SUBTREECOM) {
    for (int i = 0; i < 3; i++) v[i] = F.subtree_com[3 * id + i];
  } else if (t == SENS_CLOCK) {
    v[0] = time; dim = 1;
  } else if (t == SENS_GYRO || t == SENS_VELOCIMETER) {  // sensor.py:909-949
    float p[3], R[9];
    site_pose(m, wid, F, id, p, R);
    const int b = m.site_bodyid[id];
    const float* cv = F.cvel + 6 * b;
    if (t == SENS_GYRO) {
      mat_t_vec(v, R, cv);
    } else {
      const float* com = F.subtree_com + 3 * m.body_rootid[b];
      float dif[3], c[3], lin[3];
      for (int i = 0; i < 3; i++) dif[i] = p[i] - com[i];
      cross3(c, dif, cv);
      for (int i = 0; i < 3; i++) lin[i] = cv[3 + i] - c[i];
      mat_t_vec(v, R, lin);
    }
  } else if (t == SENS_JOINTVEL) {
    v[0] = qvel[m.jnt_dofadr[id]]; dim = 1;
  } else if (t == SENS_ACTUATORVEL) {
    v[0] = act_vel[id]; dim = 1;
  } else if (t == SENS_BALLANGVEL) {
    for (int i = 0; i < 3; i++) v[i] = qvel[m.jnt_dofadr[id] + i];
  } else if (t == SENS_FRAMELINVEL) {  // sensor.py:1053-1156
    float p[3], R[9], pr[3], Rr[9], off[3], offr[3], c[3], xl[3];
    obj_frame(m, wid, F, ot, id, p, R);
    obj_frame(m, wid, F, rt, rid, pr, Rr);
    const float* cv = cvel_offset(m, wid, F, ot, id, off);
    const float* cvr = cvel_offset(m, wid, F, rt, rid, offr);
    cross3(c, off, cv);
    for (int i = 0; i < 3; i++) xl[i] = cv[3 + i] - c[i];
    if (rid > -1) {
      float cr[3], rvec[3], rc[3], rel[3];
      cross3(cr, offr, cvr);
      for (int i = 0; i < 3; i++) rvec[i] = p[i] - pr[i];
      cross3(rc, rvec, cvr);
      for (int i = 0; i < 3; i++) rel[i] = xl[i] - (cvr[3 + i] - cr[i]) + rc[i];
      mat_t_vec(v, Rr, rel);
    } else {
      for (int i = 0; i < 3; i++) v[i] = xl[i];
    }
  } else if (t == SENS_FRAMEANGVEL) {  // sensor.py:1159-1238
    float off[3];
    const float* cv = cvel_offset(m, wid, F, ot, id, off);
    if (rid > -1) {
      float pr[3], Rr[9];
      obj_frame(m, wid, F, rt, rid, pr, Rr);
      const float* cvr = cvel_offset(m, wid, F, rt, rid, off);
      float dw[3] = {cv[0] - cvr[0], cv[1] - cvr[1], cv[2] - cvr[2]};
      mat_t_vec(v, Rr, dw);
    } else {
      for (int i = 0; i < 3; i++) v[i] = cv[i];
    }
  } else {
    return;
  }
  sensor_write(m, d, wid, s, v, dim);
}

}  // namespace mjw
