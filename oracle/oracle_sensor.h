/* Sensors beyond the frame / IMU set, for the CPU oracle (test infrastructure only -- never the product path).
 *
 * touch (sensor.py:2001-2076, with ray.py:105-450's ray-geom intersections for the site zone), tendon
 * position / velocity / actuator force (sensor.py:222, 957, 1538-1577), joint and tendon limit position /
 * velocity / force (sensor.py:243-278, 972-1007, 1580-1615), subtree linear velocity and angular momentum
 * (smooth.py:2932-3084), potential and kinetic energy (sensor.py:2700-2940).  Included by oracle.c after its
 * sensor helpers. */

enum {
  SENS_TOUCH = 0, SENS_TENDONPOS = 11, SENS_TENDONVEL = 12, SENS_TENDONACTFRC = 17, SENS_JOINTLIMITPOS = 20,
  SENS_JOINTLIMITVEL = 21, SENS_JOINTLIMITFRC = 22, SENS_TENDONLIMITPOS = 23, SENS_TENDONLIMITVEL = 24,
  SENS_TENDONLIMITFRC = 25, SENS_SUBTREELINVEL = 36, SENS_SUBTREEANGMOM = 37, SENS_E_POTENTIAL = 43, SENS_E_KINETIC = 44
};

/* ray.py:105-125: smallest non-negative root of a x^2 + 2 b x + c = 0 (else -1); both roots in x */
static real ray_quad(real a, real b, real c, real* x) {
  real det = b * b - a * c;
  x[0] = x[1] = -1;
  if (det < MINVAL) return -1;
  det = sqrt(det);
  const real den = safe_div(1.0, a);
  x[0] = (-b - det) * den;
  x[1] = (-b + det) * den;
  if (x[0] >= 0) return x[0];
  if (x[1] >= 0) return x[1];
  return -1;
}

static real ray_sphere(const real* pos, real r2, const real* pnt, const real* vec) {
  real dif[3] = {pnt[0] - pos[0], pnt[1] - pos[1], pnt[2] - pos[2]}, x[2];
  return ray_quad(dot3(vec, vec), dot3(vec, dif), dot3(dif, dif) - r2, x);
}

/* ray.py:187-450 (plane, capsule, ellipsoid, cylinder, box; distances only): lp / lv = ray in the local frame */
static real ray_geom_local(int type, const real* size, const real* lp, const real* lv) {
  real x[2];
  if (type == GEOM_PLANE) {
    if (lv[2] > -MINVAL) return -1;
    const real t = -lp[2] / lv[2];
    if (t < 0) return -1;
    const real p0 = lp[0] + t * lv[0], p1 = lp[1] + t * lv[1];
    return ((size[0] <= 0 || fabs(p0) <= size[0]) && (size[1] <= 0 || fabs(p1) <= size[1])) ? t : -1;
  }
  if (type == GEOM_SPHERE) {
    const real z[3] = {0, 0, 0};
    return ray_sphere(z, size[0] * size[0], lp, lv);
  }
  if (type == GEOM_CAPSULE) {
    const real z[3] = {0, 0, 0}, ssz = size[0] + size[1];
    if (ray_sphere(z, ssz * ssz, lp, lv) < 0) return -1;
    real best = -1;
    const real sq = size[0] * size[0];
    real a = lv[0] * lv[0] + lv[1] * lv[1], b = lv[0] * lp[0] + lv[1] * lp[1], c = lp[0] * lp[0] + lp[1] * lp[1] - sq;
    const real sol = ray_quad(a, b, c, x);
    if (sol >= 0 && fabs(lp[2] + sol * lv[2]) <= size[1]) best = sol;
    a += lv[2] * lv[2];
    for (int side = 1; side >= -1; side -= 2) {
      const real ld[3] = {lp[0], lp[1], lp[2] - side * size[1]};
      ray_quad(a, dot3(lv, ld), dot3(ld, ld) - sq, x);
      for (int i = 0; i < 2; i++)
        if (x[i] >= 0 && (side > 0 ? lp[2] + x[i] * lv[2] >= size[1] : lp[2] + x[i] * lv[2] <= -size[1]))
          if (best < 0 || x[i] < best) best = x[i];
    }
    return best;
  }
  if (type == GEOM_ELLIPSOID) {
    const real s[3] = {safe_div(1.0, size[0] * size[0]), safe_div(1.0, size[1] * size[1]), safe_div(1.0, size[2] * size[2])};
    const real sv[3] = {s[0] * lv[0], s[1] * lv[1], s[2] * lv[2]}, sp[3] = {s[0] * lp[0], s[1] * lp[1], s[2] * lp[2]};
    return ray_quad(dot3(sv, lv), dot3(sv, lp), dot3(sp, lp) - 1, x);
  }
  if (type == GEOM_CYLINDER) {
    const real z[3] = {0, 0, 0};
    if (ray_sphere(z, size[0] * size[0] + size[1] * size[1], lp, lv) < 0) return -1;
    real best = -1;
    if (fabs(lv[2]) > MINVAL)
      for (int side = -1; side <= 1; side += 2) {
        const real sol = (side * size[1] - lp[2]) / lv[2];
        if (sol >= 0) {
          const real p0 = lp[0] + sol * lv[0], p1 = lp[1] + sol * lv[1];
          if (p0 * p0 + p1 * p1 <= size[0] * size[0] && (best < 0 || sol < best)) best = sol;
        }
      }
    const real sol = ray_quad(lv[0] * lv[0] + lv[1] * lv[1], lv[0] * lp[0] + lv[1] * lp[1], lp[0] * lp[0] + lp[1] * lp[1] - size[0] * size[0], x);
    if (sol >= 0 && fabs(lp[2] + sol * lv[2]) <= size[1] && (best < 0 || sol < best)) best = sol;
    return best;
  }
  if (type == GEOM_BOX) {
    const real z[3] = {0, 0, 0};
    if (ray_sphere(z, dot3(size, size), lp, lv) < 0) return -1;
    static const int iface[3][2] = {{1, 2}, {0, 2}, {0, 1}};
    real best = -1;
    for (int i = 0; i < 3; i++) {
      if (fabs(lv[i]) <= MINVAL) continue;
      for (int side = -1; side <= 1; side += 2) {
        const real sol = (side * size[i] - lp[i]) / lv[i];
        if (sol < 0) continue;
        const real p0 = lp[iface[i][0]] + sol * lv[iface[i][0]], p1 = lp[iface[i][1]] + sol * lv[iface[i][1]];
        if (fabs(p0) <= size[iface[i][0]] && fabs(p1) <= size[iface[i][1]] && (best < 0 || sol < best)) best = sol;
      }
    }
    return best;
  }
  return -1;
}

/* ray.py:32-49 + 799-820: the ray in the geom frame (pos, row-major mat) */
static real ray_geom(const real* pos, const real* mat, const real* size, const real* pnt, const real* vec, int type) {
  if (type == GEOM_SPHERE) return ray_sphere(pos, size[0] * size[0], pnt, vec);
  real dif[3] = {pnt[0] - pos[0], pnt[1] - pos[1], pnt[2] - pos[2]}, lp[3], lv[3];
  mat_t_vec(lp, mat, dif);
  mat_t_vec(lv, mat, vec);
  return ray_geom_local(type, size, lp, lv);
}

/* the efc row of the limit on joint / tendon `id` (sensor.py:243-278: any LIMIT row with that id) or -1 */
static int limit_row(const orc_data* d, int id) {
  const int lo = d->ne[0] + d->nf[0], hi = lo + d->nl[0];
  int r = -1;
  for (int e = lo; e < hi && e < d->njmax; e++)
    if (d->efc_id[e] == id && (d->efc_type[e] == CNSTR_LIMIT_JOINT || d->efc_type[e] == CNSTR_LIMIT_TENDON)) r = e;
  return r;
}

/* sensor.py:2700-2890 energy_pos: -sum m g . xipos, joint and tendon springs */
static real energy_potential(const orc_model* m, const orc_data* d) {
  real e = 0;
  if (!(m->opt_disableflags & DSBL_GRAVITY))
    for (int b = 1; b < m->nbody; b++) e -= m->body_mass[b] * dot3(m->opt_gravity, d->xipos + 3 * b);
  if (m->opt_disableflags & DSBL_SPRING) return e;
  for (int j = 0; j < m->njnt; j++) {
    const real k = m->jnt_stiffness[j];
    if (k == 0) continue;
    const int a = m->jnt_qposadr[j], t = m->jnt_type[j];
    const real* qs = m->qpos_spring;
    if (t == JNT_FREE || t == JNT_BALL) {
      real dif0 = 0;
      int q0 = a;
      if (t == JNT_FREE) {
        for (int i = 0; i < 3; i++) dif0 += (d->qpos[a + i] - qs[a + i]) * (d->qpos[a + i] - qs[a + i]);
        q0 = a + 3;
      }
      real q[4] = {d->qpos[q0], d->qpos[q0 + 1], d->qpos[q0 + 2], d->qpos[q0 + 3]}, dif[3];
      normalize4(q);
      quat_sub(dif, q, qs + q0);
      e += 0.5 * k * (dif0 + dot3(dif, dif));
    } else {
      const real dq = d->qpos[a] - qs[a];
      e += 0.5 * k * dq * dq;
    }
  }
  for (int t = 0; t < m->ntendon; t++) {
    const real k = m->tendon_stiffness[t];
    if (k == 0) continue;
    const real L = d->ten_length[t], lo = m->tendon_lengthspring[2 * t], hi = m->tendon_lengthspring[2 * t + 1];
    const real disp = L > hi ? hi - L : (L < lo ? lo - L : 0);
    e += 0.5 * k * disp * disp;
  }
  return e;
}

/* sensor.py:2893-2940 energy_vel: 0.5 qvel' M qvel */
static real energy_kinetic(const orc_model* m, const orc_data* d) {
  real e = 0;
  for (int i = 0; i < m->nv; i++)
    for (int j = 0; j < m->nv; j++) e += d->qvel[i] * d->qM[(size_t)i * m->nv + j] * d->qvel[j];
  return 0.5 * e;
}

/* smooth.py:2932-3084 subtree_vel: subtree linear velocity and angular momentum about the subtree com */
static void subtree_vel(const orc_model* m, orc_data* d) {
  const int nb = m->nbody;
  real* bvel = (real*)malloc(6 * nb * sizeof(real));
  for (int b = 0; b < nb; b++) {
    const real* cv = d->cvel + 6 * b;
    const real* sc = d->subtree_com + 3 * m->body_rootid[b];
    real dif[3] = {d->xipos[3 * b] - sc[0], d->xipos[3 * b + 1] - sc[1], d->xipos[3 * b + 2] - sc[2]}, c[3], lin[3], dv[3];
    cross3(c, dif, cv);
    for (int i = 0; i < 3; i++) lin[i] = cv[3 + i] - c[i];
    for (int i = 0; i < 3; i++) d->subtree_linvel[3 * b + i] = m->body_mass[b] * lin[i];
    mat_t_vec(dv, d->ximat + 9 * b, cv);
    for (int i = 0; i < 3; i++) dv[i] *= m->body_inertia[3 * b + i];
    r_vec(d->subtree_angmom + 3 * b, d->ximat + 9 * b, dv);
    for (int i = 0; i < 3; i++) { bvel[6 * b + i] = cv[i]; bvel[6 * b + 3 + i] = lin[i]; }
  }
  /* deepest bodies first: bodies are in DFS pre-order, so reverse index order visits children first */
  for (int b = nb - 1; b >= 0; b--) {
    if (b > 0)
      for (int i = 0; i < 3; i++) d->subtree_linvel[3 * m->body_parentid[b] + i] += d->subtree_linvel[3 * b + i];
    for (int i = 0; i < 3; i++) d->subtree_linvel[3 * b + i] /= maxr(MINVAL, m->body_subtreemass[b]);
  }
  for (int b = nb - 1; b > 0; b--) {
    const int p = m->body_parentid[b];
    const real *com = d->subtree_com + 3 * b, *comp = d->subtree_com + 3 * p;
    const real *lv = d->subtree_linvel + 3 * b, *lvp = d->subtree_linvel + 3 * p;
    real dx[3], dp[3], dL[3];
    for (int i = 0; i < 3; i++) { dx[i] = d->xipos[3 * b + i] - com[i]; dp[i] = (bvel[6 * b + 3 + i] - lv[i]) * m->body_mass[b]; }
    cross3(dL, dx, dp);
    for (int i = 0; i < 3; i++) d->subtree_angmom[3 * b + i] += dL[i];
    for (int i = 0; i < 3; i++) d->subtree_angmom[3 * p + i] += d->subtree_angmom[3 * b + i];
    for (int i = 0; i < 3; i++) { dx[i] = com[i] - comp[i]; dp[i] = (lv[i] - lvp[i]) * m->body_subtreemass[b]; }
    cross3(dL, dx, dp);
    for (int i = 0; i < 3; i++) d->subtree_angmom[3 * p + i] += dL[i];
  }
  free(bvel);
}

/* sensor.py:2001-2076 touch: normal forces of the contacts on the site's body whose ray along the normal (from
 * the contact, away from the body) meets the site's zone */
static real touch_sensor(const orc_model* m, const orc_data* d, int site) {
  const int body = m->site_bodyid[site];
  real total = 0;
  for (int c = 0; c < d->ncon[0]; c++) {
    const int g1 = d->con_geom[2 * c], g2 = d->con_geom[2 * c + 1];
    if (g1 < 0 || g2 < 0) continue;
    const int b1 = m->geom_bodyid[g1], b2 = m->geom_bodyid[g2];
    const int* adr = d->con_efc_address + 10 * c;
    if (adr[0] < 0 || (body != b1 && body != b2)) continue;
    real f = d->efc_force[adr[0]];
    if (m->opt_cone == 0)
      for (int i = 1; i < 2 * (d->con_dim[c] - 1); i++) f += d->efc_force[adr[i]];
    if (f <= 0) continue;
    const real* n = d->con_frame + 9 * c;
    real ray[3] = {n[0] * f, n[1] * f, n[2] * f}, dir[3];
    normalize_with_norm(dir, ray);
    if (body == b2)
      for (int i = 0; i < 3; i++) dir[i] = -dir[i];
    if (ray_geom(d->site_xpos + 3 * site, d->site_xmat + 9 * site, m->site_size + 3 * site, d->con_pos + 3 * c, dir, m->site_type[site]) >= 0)
      total += f;
  }
  return total;
}

/* the sensors above for one stage (1 position, 2 velocity, 3 acceleration) */
static void sensor_extra(const orc_model* m, orc_data* d, int stage) {
  int subtree = 0;
  for (int s = 0; s < m->nsensor; s++)
    subtree |= m->sensor_type[s] == SENS_SUBTREELINVEL || m->sensor_type[s] == SENS_SUBTREEANGMOM;
  if (stage == STAGE_VEL && subtree) subtree_vel(m, d);
  for (int s = 0; s < m->nsensor; s++) {
    if (m->sensor_needstage[s] != stage) continue;
    const int t = m->sensor_type[s], id = m->sensor_objid[s];
    real v[3] = {0, 0, 0};
    int dim = 1, r;
    switch (t) {
      case SENS_TENDONPOS: v[0] = d->ten_length[id]; break;
      case SENS_TENDONVEL: v[0] = d->ten_velocity[id]; break;
      case SENS_JOINTLIMITPOS: case SENS_TENDONLIMITPOS:
        if ((r = limit_row(d, id)) >= 0) v[0] = d->efc_pos[r] - d->efc_margin[r];
        break;
      case SENS_JOINTLIMITVEL: case SENS_TENDONLIMITVEL:
        if ((r = limit_row(d, id)) >= 0) v[0] = d->efc_vel[r];
        break;
      case SENS_JOINTLIMITFRC: case SENS_TENDONLIMITFRC:
        if ((r = limit_row(d, id)) >= 0) v[0] = d->efc_force[r];
        break;
      case SENS_TENDONACTFRC:
        for (int a = 0; a < m->nu; a++)
          if (m->actuator_trntype[a] == TRN_TENDON && m->actuator_trnid[2 * a] == id) v[0] += d->actuator_force[a];
        break;
      case SENS_TOUCH: v[0] = touch_sensor(m, d, id); break;
      case SENS_SUBTREELINVEL: memcpy(v, d->subtree_linvel + 3 * id, sizeof(v)); dim = 3; break;
      case SENS_SUBTREEANGMOM: memcpy(v, d->subtree_angmom + 3 * id, sizeof(v)); dim = 3; break;
      case SENS_E_POTENTIAL: v[0] = energy_potential(m, d); break;
      case SENS_E_KINETIC: v[0] = energy_kinetic(m, d); break;
      default: continue;
    }
    sensor_write(m, d, s, v, dim);
  }
}
