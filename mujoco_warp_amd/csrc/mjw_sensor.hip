// mjw_sensor.hip -- post-solve sensor kernel: sensor_pos, sensor_vel, rne_postconstraint and
// sensor_acc (forward.py:981-998) in one launch.
//
// Runs between the solver and the integrator, only for models with sensors, so the forward kernel
// carries no sensor code (its register budget is untouched).  None of the position / velocity
// quantities change between fwd_position and the integrator, so evaluating those sensors here
// gives the values the reference computes right after each stage.  One 64-lane wavefront per
// world: lanes map to bodies for the tree passes and to sensors for the evaluation.  Inputs come
// from HBM (written by the forward and dense kernels of the same step: qpos / qvel / time before
// integration, qacc, cdof, cdof_dot, cvel, cinert, subtree_com, frames, contacts and efc forces);
// cacc / cfrc_int / cfrc_ext / sensordata are written back.  Restates smooth.py:1276-1499
// (rne_postconstraint) and sensor.py:459-706, 1251-1373, 1451-1700, 2447-2680.

#include "mjw_sensor.h"

namespace mjw {

struct SLay {
  int cacc, cfrc, cext, cvel, cinert, com, cdof, cdofdot, qvel, qacc, ccd, scc, tac, total;
};

__host__ inline SLay make_slayout(const mjw_model_t& m) {
  SLay L;
  int o = 0;
  auto take = [&](int n) { int r = o; o += (n + 3) & ~3; return r; };
  const int nb = m.nbody, nv = m.nv;
  L.cacc = take(nb * 6); L.cfrc = take(nb * 6); L.cext = take(nb * 6); L.cvel = take(nb * 6); L.cinert = take(nb * 10);
  L.com = take(nb * 3); L.cdof = take(nv * 6); L.cdofdot = take(nv * 6); L.qvel = take(nv); L.qacc = take(nv);
  // collision sensors on convex pairs: the lockstep GJK / EPA workspace and the per-record results
  L.tac = m.nsensortaxel > 0 ? take(64) : -1;  // tactile: a weld body's contact partners (tactile_partners)
  L.ccd = L.scc = -1;
  if (m.nsensorccd > 0) {
    L.ccd = take(ccd_layout(m.ccd_epa_iterations, m.nhfield > 0, m.nmaxpolygon, m.nmaxmeshdeg).total);
    L.scc = take(SCC_WORDS * m.nsensorcollision);
  }
  L.total = o;
  return L;
}

// stages: bit 0 position, bit 1 velocity, bit 2 acceleration sensors (+ rne_postconstraint).  COLL: the
// instantiation with the collision sensors (primitive narrowphase + the lockstep GJK / EPA), launched as
// sensor_coll_kernel for models that have them; compiled into every model's kernel they pushed it to
// 256 VGPRs with 3.2 KB of scratch per lane (apollo's IMU-only sensor kernel 0.306 ms)
template <bool COLL>
__device__ __forceinline__ void sensor_body(const mjw_model_t& m, const mjw_data_t& d, const SLay& L, int stages, int w0) {
  extern __shared__ __attribute__((aligned(16))) float s[];
  const int wid = w0 + (int)blockIdx.x, lane = threadIdx.x & 63;
  if (wid >= d.nworld) return;
  const int nb = m.nbody, nv = m.nv;
  const long wb = (long)wid * nb;
  for (int e = lane; e < nb * 6; e += LPW) s[L.cvel + e] = d.cvel[wb * 6 + e];
  for (int e = lane; e < nb * 10; e += LPW) s[L.cinert + e] = d.cinert[wb * 10 + e];
  for (int e = lane; e < nb * 3; e += LPW) s[L.com + e] = d.subtree_com[wb * 3 + e];
  for (int e = lane; e < nv * 6; e += LPW) {
    s[L.cdof + e] = d.cdof[(long)wid * nv * 6 + e];
    s[L.cdofdot + e] = d.cdof_dot[(long)wid * nv * 6 + e];
  }
  for (int i = lane; i < nv; i += LPW) {
    s[L.qvel + i] = d.qvel[(long)wid * nv + i];
    s[L.qacc + i] = d.qacc[(long)wid * nv + i];
  }
  __syncthreads();
  float* cacc = s + L.cacc;
  float* cfrc = s + L.cfrc;
  float* cext = s + L.cext;
  const float* cvel = s + L.cvel;
  if ((stages & 4) && m.sensor_rne_postconstraint) {
    // cfrc_ext = xfrc_applied moved to the subtree com (smooth.py:1278-1295)
    const float* xipos = d.xipos + wb * 3;
    for (int b = lane; b < nb; b += LPW) {
      float f[6] = {0, 0, 0, 0, 0, 0};
      if (b > 0) {
        const float* xf = d.xfrc_applied + (wb + b) * 6;
        const float* com = s + L.com + 3 * m.body_rootid[b];
        float off[3], c[3];
        for (int i = 0; i < 3; i++) off[i] = com[i] - xipos[3 * b + i];
        cross3(c, off, xf);
        for (int i = 0; i < 3; i++) { f[i] = xf[3 + i] - c[i]; f[3 + i] = xf[i]; }
      }
      for (int i = 0; i < 6; i++) cext[6 * b + i] = f[i];
    }
    __syncthreads();
    const int nefc = min(d.nefc[wid], d.njmax);
    const long wr = (long)wid * d.njmax;
    // cfrc_ext += connect / weld forces (smooth.py:1296-1430): their rows lead the efc block
    // (all connects, then all welds), lane = body
    if (m.neq_cw > 0) {
      const int ne = min(d.ne[wid], nefc);
      const float* xpos = d.xpos + wb * 3;
      const float* xmat = d.xmat + wb * 9;
      int r = 0;
      while (r < ne) {
        const int id = d.efc_id[wr + r];
        const int et = m.eq_type[id];
        if (et != EQ_CONNECT && et != EQ_WELD) break;  // joint equality rows follow
        const bool weld = et == EQ_WELD;
        float frc[3], trq[3] = {0, 0, 0};
        for (int i = 0; i < 3; i++) frc[i] = d.efc_force[wr + r + i];
        if (weld)
          for (int i = 0; i < 3; i++) trq[i] = d.efc_force[wr + r + 3 + i];
        const bool body_sem = m.eq_objtype[id] == OBJ_BODY;
        const int o1 = m.eq_obj1id[id], o2 = m.eq_obj2id[id];
        const int b1 = body_sem ? o1 : m.site_bodyid[o1], b2 = body_sem ? o2 : m.site_bodyid[o2];
        const float* data = MR(eq_data) + 11 * id;
        for (int b = lane; b < nb; b += LPW) {
          for (int k = 0; k < 2; k++) {
            const int bk = k == 0 ? b1 : b2;
            if (b == 0 || b != bk) continue;
            const float* off = body_sem ? (data + ((k == 0) != weld ? 0 : 3)) : MR(site_pos) + 3 * (k == 0 ? o1 : o2);
            float pos[3], dif[3], c[3];
            matvec3(pos, xmat + 9 * b, off);
            for (int i = 0; i < 3; i++) dif[i] = s[L.com + 3 * m.body_rootid[b] + i] - (pos[i] + xpos[3 * b + i]);
            cross3(c, dif, frc);
            const float sg = k == 0 ? 1.0f : -1.0f;
            for (int i = 0; i < 3; i++) {
              cext[6 * b + i] += sg * (trq[i] - c[i]);
              cext[6 * b + 3 + i] += sg * frc[i];
            }
          }
        }
        r += weld ? 6 : 3;
      }
      __syncthreads();
    }
    // cfrc_ext += contact forces (smooth.py:1447-1495, support.py:241-308); contacts visited in
    // constraint-row order (each contact at its first row), lane = body
    for (int r = 0; r < nefc; r++) {
      const int type = d.efc_type[wr + r];
      if (type != CNSTR_CONTACT_FRICTIONLESS && type != CNSTR_CONTACT_PYRAMIDAL && type != CNSTR_CONTACT_ELLIPTIC) continue;
      const int cid = d.efc_id[wr + r];
      if (cid < 0 || cid >= d.naconmax || d.contact_efc_address[(long)cid * m.nmaxpyramid] != r) continue;
      const int id1 = m.geom_bodyid[d.contact_geom[2L * cid]], id2 = m.geom_bodyid[d.contact_geom[2L * cid + 1]];
      if (id1 == 0 && id2 == 0) continue;
      const int condim = d.contact_dim[cid];
      float f[6] = {0, 0, 0, 0, 0, 0};
      if (condim == 1) {
        f[0] = d.efc_force[wr + r];
      } else if (type == CNSTR_CONTACT_ELLIPTIC) {
        // elliptic rows are the contact-frame force components (support.py:296-299)
        for (int i = 0; i < condim; i++) {
          const int a = d.contact_efc_address[(long)cid * m.nmaxpyramid + i];
          f[i] = (a >= 0 && a < d.njmax) ? d.efc_force[wr + a] : 0.0f;
        }
      } else {
        for (int i = 0; i < condim - 1; i++) {
          int a = 2 * i + r;
          float d1 = a < d.njmax ? d.efc_force[wr + a] : 0.0f, d2 = a + 1 < d.njmax ? d.efc_force[wr + a + 1] : 0.0f;
          f[0] += d1 + d2;
          f[i + 1] = (d1 - d2) * d.contact_friction[5L * cid + i];
        }
      }
      const float* F = d.contact_frame + 9L * cid;
      float fw[6];
      for (int i = 0; i < 3; i++) {
        fw[i] = f[0] * F[i] + f[1] * F[3 + i] + f[2] * F[6 + i];
        fw[3 + i] = f[3] * F[i] + f[4] * F[3 + i] + f[5] * F[6 + i];
      }
      const float* pos = d.contact_pos + 3L * cid;
      for (int b = lane; b < nb; b += LPW) {
        if (b == 0 || (b != id1 && b != id2)) continue;
        const float* com = s + L.com + 3 * m.body_rootid[b];
        float off[3], c[3];
        for (int i = 0; i < 3; i++) off[i] = com[i] - pos[i];
        cross3(c, off, fw);
        float t[6];
        for (int i = 0; i < 3; i++) { t[i] = fw[3 + i] - c[i]; t[3 + i] = fw[i]; }
        if (b == id1)
          for (int i = 0; i < 6; i++) cext[6 * b + i] -= t[i];
        if (b == id2)
          for (int i = 0; i < 6; i++) cext[6 * b + i] += t[i];
      }
    }
    // cacc with qacc (smooth.py:1112-1170, flg_acc): body-local increments, then a level pass
    for (int b = lane; b < nb; b += LPW) {
      float acc[6] = {0, 0, 0, 0, 0, 0};
      if (b == 0) {
        const float* grav = MR(opt_gravity);
        if (!(m.opt_disableflags & DSBL_GRAVITY))
          for (int i = 0; i < 3; i++) acc[3 + i] = -grav[i];
      } else {
        const int adr = m.body_dofadr[b], num = m.body_dofnum[b];
        for (int k = adr; k < adr + num; k++)
          for (int i = 0; i < 6; i++) acc[i] += s[L.cdofdot + 6 * k + i] * s[L.qvel + k] + s[L.cdof + 6 * k + i] * s[L.qacc + k];
      }
      for (int i = 0; i < 6; i++) cacc[6 * b + i] = acc[i];
    }
    __syncthreads();
    for (int b0 = 0; b0 < nb; b0 += LPW) {
      const int b = b0 + lane;
      const bool ok = b > 0 && b < nb;
      const int par = ok ? m.body_parentid[b] : 0, lv = ok ? m.body_level[b] : 0;
      for (int lvl = 1; lvl < m.nlevel; lvl++) {
        if (ok && lv == lvl)
          for (int i = 0; i < 6; i++) cacc[6 * b + i] += cacc[6 * par + i];
        __syncthreads();
      }
    }
    // cfrc_int = cinert cacc + cvel x* (cinert cvel) - cfrc_ext, then subtree sums (smooth.py:1175-1230)
    for (int b = lane; b < nb; b += LPW) {
      float f[6] = {0, 0, 0, 0, 0, 0};
      if (b > 0) {
        float f1[6], iv[6], f2[6];
        inert_vec(f1, s + L.cinert + 10 * b, cacc + 6 * b);
        inert_vec(iv, s + L.cinert + 10 * b, cvel + 6 * b);
        motion_cross_force(f2, cvel + 6 * b, iv);
        for (int i = 0; i < 6; i++) f[i] = f1[i] + f2[i] - cext[6 * b + i];
      }
      for (int i = 0; i < 6; i++) cfrc[6 * b + i] = f[i];
    }
    __syncthreads();
    for (int b = lane; b < nb; b += LPW) {
      float acc[6] = {0, 0, 0, 0, 0, 0};
      const int end = m.body_subtree_end[b];
      for (int j = (b == 0 ? 1 : b); j < end; j++)
        for (int i = 0; i < 6; i++) acc[i] += cfrc[6 * j + i];
      for (int i = 0; i < 6; i++) {
        d.cfrc_int[(wb + b) * 6 + i] = acc[i];
        d.cacc[(wb + b) * 6 + i] = cacc[6 * b + i];
        d.cfrc_ext[(wb + b) * 6 + i] = cext[6 * b + i];
      }
    }
    __syncthreads();
    // subtree sums back into cfrc (each lane reads back only the bodies it wrote above)
    for (int b = lane; b < nb; b += LPW)
      for (int i = 0; i < 6; i++) cfrc[6 * b + i] = d.cfrc_int[(wb + b) * 6 + i];
    __syncthreads();
  } else {
    for (int e = lane; e < nb * 6; e += LPW) { cacc[e] = d.cacc[wb * 6 + e]; cfrc[e] = d.cfrc_int[wb * 6 + e]; }
    __syncthreads();
  }
  Frames F;
  F.xpos = d.xpos + wb * 3; F.xquat = d.xquat + wb * 4; F.xmat = d.xmat + wb * 9; F.xipos = d.xipos + wb * 3;
  F.ximat = d.ximat + wb * 9; F.gxpos = d.geom_xpos + (long)wid * m.ngeom * 3; F.gxmat = d.geom_xmat + (long)wid * m.ngeom * 9;
  F.cxpos = d.cam_xpos + (long)wid * m.ncam * 3; F.cxmat = d.cam_xmat + (long)wid * m.ncam * 9;
  F.subtree_com = s + L.com; F.cvel = cvel;
  F.scc = L.scc >= 0 ? s + L.scc : nullptr;
  if (COLL && (stages & 1) && L.ccd >= 0) sensor_convex_records(m, F, wid, s + L.ccd, s + L.scc);
  // smooth.py:3044-3084 subtree_vel for the subtree velocity / momentum sensors (sensor.py:1383-1384)
  if (stages & 2) {
    bool sub = false;
    for (int k = 0; k < m.nsensor; k++) sub |= m.sensor_type[k] == SENS_SUBTREELINVEL || m.sensor_type[k] == SENS_SUBTREEANGMOM;
    if (sub) {
      if (lane == 0) subtree_vel(m, d, wid, cvel, s + L.com);
      __syncthreads();
    }
  }
  // position / velocity sensors (sensor.py:459-706, 1251-1373), lane = sensor
  const float time = d.time[wid];
  for (int k = lane; k < m.nsensor; k += LPW) {
    const int st = m.sensor_needstage[k];
    if ((st == STAGE_POS && (stages & 1)) || (st == STAGE_VEL && (stages & 2)))
      sensor_posvel_one<COLL>(m, d, wid, F, k, d.qpos + (long)wid * m.nq, s + L.qvel, d.actuator_length + (long)wid * m.nu,
                        d.actuator_velocity + (long)wid * m.nu, time);
  }
  // acceleration sensors (sensor.py:1697-1997, supported types), lane = sensor
  for (int k = lane; k < m.nsensor && (stages & 4); k += LPW) {
    if (m.sensor_needstage[k] != STAGE_ACC) continue;
    const int t = m.sensor_type[k], id = m.sensor_objid[k], ot = m.sensor_objtype[k];
    float v[3] = {0, 0, 0};
    int dim = 3;
    if (t == SENS_ACCELEROMETER || t == SENS_FRAMELINACC) {  // sensor.py:1451-1480, 1619-1667
      float p[3], R[9];
      const int b = obj_frame(m, wid, F, t == SENS_ACCELEROMETER ? OBJ_SITE : ot, id, p, R);
      const float* cv = cvel + 6 * b;
      const float* ca = cacc + 6 * b;
      const float* com = F.subtree_com + 3 * m.body_rootid[b];
      float dif[3], c1[3], c2[3], lin[3], acc[3], corr[3];
      for (int i = 0; i < 3; i++) dif[i] = p[i] - com[i];
      cross3(c1, dif, cv);
      cross3(c2, dif, ca);
      for (int i = 0; i < 3; i++) { lin[i] = cv[3 + i] - c1[i]; acc[i] = ca[3 + i] - c2[i]; }
      if (t == SENS_ACCELEROMETER) {
        float ang_l[3], lin_l[3], acc_l[3];
        mat_t_vec(ang_l, R, cv);
        mat_t_vec(lin_l, R, lin);
        mat_t_vec(acc_l, R, acc);
        cross3(corr, ang_l, lin_l);
        for (int i = 0; i < 3; i++) v[i] = acc_l[i] + corr[i];
      } else {
        cross3(corr, cv, lin);
        for (int i = 0; i < 3; i++) v[i] = acc[i] + corr[i];
      }
    } else if (t == SENS_FORCE || t == SENS_TORQUE) {  // sensor.py:1483-1518
      float p[3], R[9];
      site_pose(m, wid, F, id, p, R);
      const int b = m.site_bodyid[id];
      const float* cf = cfrc + 6 * b;
      if (t == SENS_FORCE) {
        mat_t_vec(v, R, cf + 3);
      } else {
        const float* com = F.subtree_com + 3 * m.body_rootid[b];
        float dif[3], c[3], tq[3];
        for (int i = 0; i < 3; i++) dif[i] = p[i] - com[i];
        cross3(c, dif, cf + 3);
        for (int i = 0; i < 3; i++) tq[i] = cf[i] - c[i];
        mat_t_vec(v, R, tq);
      }
    } else if (t == SENS_ACTUATORFRC) {
      v[0] = d.actuator_force[(long)wid * m.nu + id]; dim = 1;
    } else if (t == SENS_JOINTACTFRC) {
      v[0] = d.qfrc_actuator[(long)wid * nv + m.jnt_dofadr[id]]; dim = 1;
    } else if (t == SENS_FRAMEANGACC) {  // sensor.py:1670-1694
      float p[3], R[9];
      const int b = obj_frame(m, wid, F, ot == OBJ_BODY ? OBJ_XBODY : ot, id, p, R);
      for (int i = 0; i < 3; i++) v[i] = cacc[6 * b + i];
    } else if (t == SENS_TENDONACTFRC) {  // sensor.py:1538-1577
      for (int a = 0; a < m.nu; a++)
        if (m.actuator_trntype[a] == TRN_TENDON && m.actuator_trnid[2 * a] == id) v[0] += d.actuator_force[(long)wid * m.nu + a];
      dim = 1;
    } else if (t == SENS_JOINTLIMITFRC || t == SENS_TENDONLIMITFRC) {  // sensor.py:1580-1615
      const int r = limit_row(d, wid, id);
      v[0] = r < 0 ? 0.0f : d.efc_force[(long)wid * d.njmax + r];
      dim = 1;
    } else if (t == SENS_CONTACT) {  // sensor.py:1750-1940
      contact_sensor(m, d, wid, F, k);
      continue;
    } else if (t == SENS_TOUCH) {  // sensor.py:2001-2076
      float p[3], R[9];
      site_pose(m, wid, F, id, p, R);
      v[0] = touch_sensor(m, d, wid, id, p, R);
      dim = 1;
    } else {
      continue;
    }
    sensor_write(m, d, wid, k, v, dim);
  }
  // tactile sensors (sensor.py:2085-2252): one sensor at a time, lane = taxel
  if ((stages & 4) && m.nsensortaxel > 0)
    for (int k = 0; k < m.nsensor; k++)
      if (m.sensor_type[k] == SENS_TACTILE) tactile_sensor(m, d, wid, F, k, lane, reinterpret_cast<int*>(s) + L.tac);
}

__global__ void __launch_bounds__(64) sensor_acc_kernel(const mjw_model_t m, const mjw_data_t d, const SLay L, int stages, int w0) {
  sensor_body<false>(m, d, L, stages, w0);
}
__global__ void __launch_bounds__(64) sensor_coll_kernel(const mjw_model_t m, const mjw_data_t d, const SLay L, int stages, int w0) {
  sensor_body<true>(m, d, L, stages, w0);
}

int sensor_launch(const mjw_model_t* m, const mjw_data_t* d, hipStream_t s, int stages, int w0, int count) {
  if (count < 0) count = d->nworld - w0;
  if (count <= 0 || m->nsensor == 0 || (m->opt_disableflags & DSBL_SENSOR) || !stages) return 0;
  SLay L = make_slayout(*m);
  size_t lds = (size_t)L.total * 4;
  if (lds > 64 * 1024) return (int)hipErrorInvalidValue;
  // contact and tactile sensors walk each world's contacts in the pool: its slot range first (the sparse
  // path's collision kernel records it itself)
  if (!m->is_sparse && (stages & 4) && (m->nsensorcontact > 0 || m->nsensortaxel > 0)) {
    const int rc = pool_ranges_launch(d, s);
    if (rc) return rc;
  }
  if (m->nsensorcollision > 0) {
    hipLaunchKernelGGL(sensor_coll_kernel, dim3(count), dim3(64), lds, s, *m, *d, L, stages, w0);
    trace_launch(s, K_SENSOR_COLL);
  } else {
    hipLaunchKernelGGL(sensor_acc_kernel, dim3(count), dim3(64), lds, s, *m, *d, L, stages, w0);
    trace_launch(s, K_SENSOR);
  }
  return (int)hipGetLastError();
}

}  // namespace mjw

extern "C" int mjw_sensor(const mjw_model_t* m, const mjw_data_t* d, int stages, void* stream) {
  if (!m || !d) return -1;
  return mjw::sensor_launch(m, d, (hipStream_t)stream, stages & 7);
}
