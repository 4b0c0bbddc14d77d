/* Sensors beyond the frame / IMU set, for the CPU oracle (test infrastructure only -- never the product path).
 *
 * touch (sensor.py:2001-2076, with ray.py:105-450's ray-geom intersections for the site zone), tendon
 * position / velocity / actuator force (sensor.py:222, 957, 1538-1577), joint and tendon limit position /
 * velocity / force (sensor.py:243-278, 972-1007, 1580-1615), subtree linear velocity and angular momentum
 * (smooth.py:2932-3084), potential and kinetic energy (sensor.py:2700-2940), the collision sensors distance /
 * normal / fromto over primitive and convex geom pairs (sensor.py:604-680, 710-757; collision_convex.py:763-852) and insidesite (sensor.py:681-697,
 * util_misc.py:603-632).  Included by oracle.c after its sensor helpers. */

enum {
  SENS_TOUCH = 0, SENS_TENDONPOS = 11, SENS_TENDONVEL = 12, SENS_TENDONACTFRC = 17, SENS_JOINTLIMITPOS = 20,
  SENS_JOINTLIMITVEL = 21, SENS_JOINTLIMITFRC = 22, SENS_TENDONLIMITPOS = 23, SENS_TENDONLIMITVEL = 24,
  SENS_TENDONLIMITFRC = 25, SENS_SUBTREELINVEL = 36, SENS_SUBTREEANGMOM = 37, SENS_E_POTENTIAL = 43, SENS_E_KINETIC = 44,
  SENS_INSIDESITE = 38, SENS_GEOMDIST = 39, SENS_GEOMNORMAL = 40, SENS_GEOMFROMTO = 41, SENS_CONTACT = 42, SENS_TACTILE = 46
};

/* ---- collision sensors: the smallest-distance contact over the sensor's geom pairs ---- */
typedef struct {
  real dist, p1[3], p2[3];
  int flip;
} coll_best;

/* sensor.py:744-757: contact points pos -+ dist / 2 along the contact normal */
static void coll_offer(coll_best* b, real dist, const real* pos, const real* nrm, int flip) {
  if (!(dist < b->dist)) return;
  b->dist = dist;
  b->flip = flip;
  for (int i = 0; i < 3; i++) {
    b->p1[i] = pos[i] - 0.5 * dist * nrm[i];
    b->p2[i] = pos[i] + 0.5 * dist * nrm[i];
  }
}

/* every contact collision_primitive.py writes for the type-sorted pair (g1, g2), inside or outside the margin
 * (write_contact keeps sensor contacts, collision_core.py:199-213) */
static void coll_pair(const orc_model* m, const orc_data* d, int g1, int g2, int flip, coll_best* b) {
  int pairid = -1;
  for (int p = 0; p < m->nxn; p++) {
    int a = m->nxn_geom_pair[2 * p], c = m->nxn_geom_pair[2 * p + 1];
    if ((a == g1 && c == g2) || (a == g2 && c == g1)) { pairid = m->nxn_pairid[2 * p] > -1 ? m->nxn_pairid[2 * p] : -1; break; }
  }
  real margin = pairid > -1 ? m->pair_margin[pairid] : m->geom_margin[g1] + m->geom_margin[g2];
  int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
  const real *p1 = d->geom_xpos + 3 * g1, *p2 = d->geom_xpos + 3 * g2;
  const real *r1 = d->geom_xmat + 9 * g1, *r2 = d->geom_xmat + 9 * g2;
  const real *s1 = m->geom_size + 3 * g1, *s2 = m->geom_size + 3 * g2;
  real n1[3] = {r1[2], r1[5], r1[8]}, n2[3] = {r2[2], r2[5], r2[8]}, nrm[3], pos[3], dist;
  if (t1 == GEOM_HFIELD) {
    /* collision_convex.py:158-697 for a sensor pair: every kept prism contact, its own normal, unflipped */
    ccd_geom cg2;
    memset(&cg2, 0, sizeof(cg2));
    cg2.type = t2;
    memcpy(cg2.pos, p2, sizeof(cg2.pos)); memcpy(cg2.rot, r2, sizeof(cg2.rot)); memcpy(cg2.size, s2, sizeof(cg2.size));
    cg2.vert = t2 == GEOM_MESH ? m->mesh_vert + 3 * m->mesh_vertadr[m->geom_dataid[g2]] : NULL;
    cg2.nvert = t2 == GEOM_MESH ? m->mesh_vertnum[m->geom_dataid[g2]] : 0;
    int hid = m->geom_dataid[g1];
    real hd[4], hp[4][3], hn[4][3];
    int n = hfield_pair(p1, r1, m->hfield_size + 4 * hid, m->hfield_nrow[hid], m->hfield_ncol[hid], m->hfield_data + m->hfield_adr[hid],
                        &cg2, m->geom_rbound[g2], m->geom_margin[g1] + m->geom_margin[g2], margin, m->opt_ccd_tolerance,
                        m->opt_ccd_iterations, m->ccd_epa_iterations, hd, hp, hn);
    for (int k = 0; k < n; k++) {
      real fr[9];
      make_frame(fr, hn[k]);
      coll_offer(b, hd[k], hp[k], fr, flip);
    }
    return;
  }
  if (convex_pair(t1, t2)) {
    /* collision_convex.py:763-852 for a sensor pair: GJK / EPA with cutoff 1e32 (separated pairs keep their
     * distance), dist += margin, the first point, and the frame flipped (:849-852) */
    ccd_geom cg1, cg2;
    memset(&cg1, 0, sizeof(cg1));
    memset(&cg2, 0, sizeof(cg2));
    cg1.type = t1; cg2.type = t2;
    memcpy(cg1.pos, p1, sizeof(cg1.pos)); memcpy(cg1.rot, r1, sizeof(cg1.rot)); memcpy(cg1.size, s1, sizeof(cg1.size));
    memcpy(cg2.pos, p2, sizeof(cg2.pos)); memcpy(cg2.rot, r2, sizeof(cg2.rot)); memcpy(cg2.size, s2, sizeof(cg2.size));
    if (t1 == GEOM_MESH) ccd_geom_mesh(m, m->geom_dataid[g1], &cg1);
    if (t2 == GEOM_MESH) ccd_geom_mesh(m, m->geom_dataid[g2], &cg2);
    ccd_multiccd = (m->opt_enableflags & ENBL_MULTICCD) != 0;
    real cdist, cnrm[3], cpts[4][3];
    int nc = ccd_pair_cut(&cg1, &cg2, m->opt_ccd_tolerance, m->opt_ccd_iterations, m->ccd_epa_iterations, margin, 1e32, &cdist, cnrm, cpts);
    if (nc > 0) {
      normalize3(cnrm);
      for (int i = 0; i < 3; i++) cnrm[i] = -cnrm[i];
      coll_offer(b, cdist, cpts[0], cnrm, flip);
    }
    return;
  }
  contacts2 c;
  c.n = 0;
  if (t1 == GEOM_PLANE && t2 == GEOM_BOX) {
    for (int k = 0; k < 8; k++) { plane_box_corner(k, n1, p1, p2, r2, s2, &dist, pos); coll_offer(b, dist, pos, n1, flip); }
    return;
  }
  if (t1 == GEOM_PLANE && t2 == GEOM_CYLINDER) {
    for (int k = 0; k < 4; k++) { plane_cylinder_k(k, n1, p1, p2, n2, s2[0], s2[1], &dist, pos); coll_offer(b, dist, pos, n1, flip); }
    return;
  }
  if (t1 == GEOM_PLANE && t2 == GEOM_SPHERE) {
    c.dist[0] = plane_sphere(c.pos[0], n1, p1, p2, s2[0]); make_frame(c.frame[0], n1); c.n = 1;
  } else if (t1 == GEOM_PLANE && t2 == GEOM_CAPSULE) {
    plane_capsule(&c, n1, p1, p2, n2, s2[0], s2[1]);
  } else if (t1 == GEOM_PLANE && t2 == GEOM_ELLIPSOID) {
    c.dist[0] = plane_ellipsoid(c.pos[0], n1, p1, p2, r2, s2); make_frame(c.frame[0], n1); c.n = 1;
  } else if (t1 == GEOM_SPHERE && t2 == GEOM_SPHERE) {
    c.dist[0] = sphere_sphere(c.pos[0], nrm, p1, s1[0], p2, s2[0]); make_frame(c.frame[0], nrm); c.n = 1;
  } else if (t1 == GEOM_SPHERE && t2 == GEOM_CAPSULE) {
    c.dist[0] = sphere_capsule(c.pos[0], nrm, p1, s1[0], p2, n2, s2[0], s2[1]); make_frame(c.frame[0], nrm); c.n = 1;
  } else if (t1 == GEOM_SPHERE && t2 == GEOM_CYLINDER) {
    c.dist[0] = sphere_cylinder(c.pos[0], nrm, p1, s1[0], p2, n2, s2[0], s2[1]); make_frame(c.frame[0], nrm); c.n = 1;
  } else if (t1 == GEOM_SPHERE && t2 == GEOM_BOX) {
    c.dist[0] = sphere_box(c.pos[0], nrm, p1, s1[0], p2, r2, s2); make_frame(c.frame[0], nrm); c.n = 1;
  } else if (t1 == GEOM_CAPSULE && t2 == GEOM_CAPSULE) {
    capsule_capsule(&c, p1, n1, s1[0], s1[1], p2, n2, s2[0], s2[1], margin);
  } else if (t1 == GEOM_CAPSULE && t2 == GEOM_BOX) {
    capsule_box(&c, p1, n1, s1[0], s1[1], p2, r2, s2);
  }
  for (int i = 0; i < c.n && i < 2; i++) coll_offer(b, c.dist[i], c.pos[i], c.frame[i], flip);
}

/* sensor.py:604-680: GEOMDIST / GEOMNORMAL / GEOMFROMTO; obj (a geom, or a body's geoms) against ref, pairs
 * in type-then-index order with flip = the pair runs (ref, obj) */
static void collision_sensor(const orc_model* m, orc_data* d, int s) {
  const int t = m->sensor_type[s];
  const real cutoff = m->sensor_cutoff[s];
  coll_best b = {cutoff, {0, 0, 0}, {0, 0, 0}, 0};
  int ids[2], nums[2];
  const int types[2] = {m->sensor_objtype[s], m->sensor_reftype[s]}, objs[2] = {m->sensor_objid[s], m->sensor_refid[s]};
  for (int k = 0; k < 2; k++) {
    if (types[k] == OBJ_BODY) { ids[k] = m->body_geomadr[objs[k]]; nums[k] = m->body_geomnum[objs[k]]; }
    else { ids[k] = objs[k]; nums[k] = 1; }
  }
  for (int a = ids[0]; a < ids[0] + nums[0]; a++)
    for (int c = ids[1]; c < ids[1] + nums[1]; c++) {
      int ta = m->geom_type[a], tc = m->geom_type[c];
      int flip = ta > tc || (ta == tc && a > c);
      coll_pair(m, d, flip ? c : a, flip ? a : c, flip, &b);
    }
  real v[6] = {0, 0, 0, 0, 0, 0};
  int dim = 1;
  if (t == SENS_GEOMDIST) {
    v[0] = b.dist;
  } else if (t == SENS_GEOMNORMAL) {
    dim = 3;
    if (b.dist <= cutoff) {
      real nn[3] = {b.p2[0] - b.p1[0], b.p2[1] - b.p1[1], b.p2[2] - b.p1[2]};
      normalize3(nn);
      for (int i = 0; i < 3; i++) v[i] = b.flip ? -nn[i] : nn[i];
    }
  } else {
    dim = 6;
    if (b.dist <= cutoff)
      for (int i = 0; i < 3; i++) { v[i] = b.flip ? b.p2[i] : b.p1[i]; v[3 + i] = b.flip ? b.p1[i] : b.p2[i]; }
  }
  sensor_write(m, d, s, v, dim);
}

/* util_misc.py:603-632 inside_geom */
static int inside_geom(const real* pos, const real* mat, const real* size, int type, const real* pt) {
  real vec[3] = {pt[0] - pos[0], pt[1] - pos[1], pt[2] - pos[2]}, pl[3];
  if (type == GEOM_SPHERE) return dot3(vec, vec) < size[0] * size[0];
  mat_t_vec(pl, mat, vec);
  if (type == GEOM_CAPSULE) {
    real z = pl[2], zc = z < -size[1] ? -size[1] : (z > size[1] ? size[1] : z), zd = z - zc;
    return pl[0] * pl[0] + pl[1] * pl[1] + zd * zd < size[0] * size[0];
  }
  if (type == GEOM_ELLIPSOID) {
    real q[3] = {pl[0] / size[0], pl[1] / size[1], pl[2] / size[2]};
    return dot3(q, q) < 1;
  }
  if (type == GEOM_CYLINDER) return fabs(pl[2]) < size[1] && pl[0] * pl[0] + pl[1] * pl[1] < size[0] * size[0];
  if (type == GEOM_BOX) return fabs(pl[0]) < size[0] && fabs(pl[1]) < size[1] && fabs(pl[2]) < size[2];
  if (type == GEOM_PLANE) return pl[2] < 0;
  return 0;
}

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

/* ---- contact sensor (sensor.py:1750-1940 output, 2258-2430 matching) ---- */
/* support.py:241-308: the contact's 6D force in its own frame */
static void contact_force_local(const orc_model* m, const orc_data* d, int c, real* f) {
  for (int i = 0; i < 6; i++) f[i] = 0;
  const int condim = d->con_dim[c], adr = d->con_efc_address[10 * c];
  if (adr < 0) return;
  if (m->opt_cone == 0) {
    if (condim == 1) { f[0] = d->efc_force[adr]; return; }
    for (int i = 0; i < condim - 1; i++) {
      const int a = 2 * i + adr;
      const real d1 = a < d->njmax ? d->efc_force[a] : 0, d2 = a + 1 < d->njmax ? d->efc_force[a + 1] : 0;
      f[0] += d1 + d2;
      f[i + 1] = (d1 - d2) * d->con_friction[5 * c + i];
    }
  } else {
    for (int i = 0; i < condim; i++) {
      const int a = d->con_efc_address[10 * c + i];
      if (a >= 0 && a < d->njmax) f[i] = d->efc_force[a];
    }
  }
}

/* sensor.py:2258-2272 _check_match */
static int contact_obj_match(const orc_model* m, int body, int geom, int type, int id) {
  if (type == OBJ_UNKNOWN || type == OBJ_SITE) return 1; /* no object / the site zone was tested already */
  if (type == OBJ_GEOM) return id == geom;
  if (type == OBJ_BODY) return id == body;
  if (type == OBJ_XBODY) {
    while (body > id) body = m->body_parentid[body];
    return body == id;
  }
  return 0;
}

/* sensor.py:2330-2375: direction (+-1) of a matched contact, 0 when it does not match */
static real contact_match(const orc_model* m, const orc_data* d, int s, int c) {
  const int ot = m->sensor_objtype[s], oid = m->sensor_objid[s], rt = m->sensor_reftype[s], rid = m->sensor_refid[s];
  if (ot == OBJ_SITE &&
      !inside_geom(d->site_xpos + 3 * oid, d->site_xmat + 9 * oid, m->site_size + 3 * oid, m->site_type[oid], d->con_pos + 3 * c))
    return 0;
  if (ot == OBJ_UNKNOWN && rt == OBJ_UNKNOWN) return 1;
  const int g1 = d->con_geom[2 * c], g2 = d->con_geom[2 * c + 1];
  const int b1 = m->geom_bodyid[g1], b2 = m->geom_bodyid[g2];
  const int m11 = contact_obj_match(m, b1, g1, ot, oid), m12 = contact_obj_match(m, b2, g2, ot, oid);
  const int m21 = contact_obj_match(m, b1, g1, rt, rid), m22 = contact_obj_match(m, b2, g2, rt, rid);
  if ((!m11 && !m12) || (!m21 && !m22)) return 0;
  if (ot != OBJ_UNKNOWN && rt != OBJ_UNKNOWN) {
    const int reg = m11 && m22, rev = m12 && m21;
    if (!reg && !rev) return 0;
    return (rev && !reg) ? -1 : 1;
  }
  if (ot != OBJ_UNKNOWN) return m11 ? 1 : -1;
  return m22 ? 1 : -1;
}

/* one contact sensor: matches in the world's contact order (MuJoCo's mj_sensorAcc order), at most
 * contact_sensor_maxmatch of them; mindist / maxforce sort the matches stably by their criteria (insertion
 * sort of the match list); netforce sums about the force-weighted centroid */
/* collision_sdf.py:148-183: signed distances of the primitive SDFs in the geom frame (plane, sphere,
 * box with the radial field inside, ellipsoid); other types have none there (0: no pressure) */
static real tactile_sdf(int type, const real* p, const real* size) {
  if (type == GEOM_PLANE) return p[2];
  if (type == GEOM_SPHERE) return sqrt(dot3(p, p)) - size[0];
  if (type == GEOM_BOX) {
    real a[3];
    for (int i = 0; i < 3; i++) a[i] = fabs(p[i]) - size[i];
    if (a[0] >= 0 || a[1] >= 0 || a[2] >= 0) {
      real b[3], mx = a[0];
      for (int i = 0; i < 3; i++) b[i] = a[i] > 0 ? a[i] : 0;
      if (a[1] > mx) mx = a[1];
      if (a[2] > mx) mx = a[2];
      return sqrt(dot3(b, b)) + (mx < 0 ? mx : 0);
    }
    real f[3];
    for (int i = 0; i < 3; i++) f[i] = -size[i] / a[i];
    const real fn = sqrt(dot3(f, f));
    /* radial field b = +-normalize(-size / a) (collision_sdf.py:148-154): |b| = 1, t = -a / |b| */
    real tmin = 1e30;
    for (int i = 0; i < 3; i++) {
      const real t = -a[i] / fabs(f[i] / fn);
      if (t < tmin) tmin = t;
    }
    return -tmin;
  }
  if (type == GEOM_ELLIPSOID) {
    real sp[3], s2[3];
    for (int i = 0; i < 3; i++) { sp[i] = p[i] / size[i]; s2[i] = p[i] / (size[i] * size[i]); }
    const real k0 = sqrt(dot3(sp, sp)), k1 = sqrt(dot3(s2, s2));
    return k0 * (k0 - 1) / (k1 != 0 ? k1 : (real)1e-12);
  }
  return 0;
}

/* sensor.py:2085-2250 tactile: for each vertex (taxel) of the sensor's mesh, placed with the sensor
 * geom's frame, the geoms in contact with that geom's weld body (first MJ_MAXCONPAIR = 50 entries of
 * the per-weld list, duplicates once) add pressure depth / max(0.05 - depth, MINVAL) for a negative
 * SDF depth (slip components 0: no tangent frames).  Every contact of the world counts, with constraint
 * rows or not (sensor.py:2097-2118 takes all of nacon: the margin-gap zone, rows cut by njmax).  Other geoms
 * than plane / sphere / box / ellipsoid (mesh ray SDF, SDF plugins) give no pressure here. */
static void tactile_sensor(const orc_model* m, orc_data* d, int s) {
  const int mesh = m->sensor_objid[s], geom = m->sensor_refid[s];
  const int nvt = m->mesh_vertnum[mesh];
  real* out = d->sensordata + m->sensor_adr[s];
  for (int i = 0; i < 3 * nvt; i++) out[i] = 0;
  const int pw = m->body_weldid[m->geom_bodyid[geom]];
  int list[50], n = 0, nadd = 0;
  for (int c = 0; c < d->ncon[0]; c++) {
    const int g1 = d->con_geom[2 * c], g2 = d->con_geom[2 * c + 1];
    if (g1 < 0 || g2 < 0) continue;
    const int w1 = m->body_weldid[m->geom_bodyid[g1]], w2 = m->body_weldid[m->geom_bodyid[g2]];
    for (int side = 0; side < 2; side++) {
      if ((side == 0 ? w1 : w2) != pw) continue;
      const int g = side == 0 ? g2 : g1;
      if (nadd++ >= 50) continue;
      int dup = 0;
      for (int j = 0; j < n; j++) dup |= list[j] == g;
      if (!dup) list[n++] = g;
    }
  }
  if (!n) return;
  const real* gx = d->geom_xpos + 3 * geom;
  const real* gm = d->geom_xmat + 9 * geom;
  for (int v = 0; v < nvt; v++) {
    const real* lp = m->mesh_vert + 3 * (m->mesh_vertadr[mesh] + v);
    real x[3];
    for (int i = 0; i < 3; i++) x[i] = gm[3 * i] * lp[0] + gm[3 * i + 1] * lp[1] + gm[3 * i + 2] * lp[2] + gx[i];
    const real* nrm = m->mesh_normal + 3 * (m->mesh_normaladr[mesh] + v);
    for (int k = 0; k < n; k++) {
      const int g = list[k];
      const real* px = d->geom_xpos + 3 * g;
      const real* pm = d->geom_xmat + 9 * g;
      real dx[3], q[3];
      for (int i = 0; i < 3; i++) dx[i] = x[i] - px[i];
      for (int i = 0; i < 3; i++) q[i] = pm[i] * dx[0] + pm[3 + i] * dx[1] + pm[6 + i] * dx[2];
      real depth = tactile_sdf(m->geom_type[g], q, m->geom_size + 3 * g);
      if (depth > 0) depth = 0;
      if (depth >= 0) continue;
      const real pressure = depth / (0.05 - depth > MINVAL ? 0.05 - depth : MINVAL);
      real f[3];
      for (int i = 0; i < 3; i++) f[i] = nrm[i] * pressure;
      out[v] += dot3(f, nrm);
      /* slip |v_rel . t1|, |v_rel . t2| (sensor.py:2233-2247) enters only with per-vertex tangent
       * frames (mesh_normalnum = 3 vertnum), which this compiler's meshes do not have: 0 */
    }
  }
}

static void contact_sensor(const orc_model* m, orc_data* d, int s) {
  const int spec = m->sensor_intprm[3 * s], reduce = m->sensor_intprm[3 * s + 1];
  static const int fsz[7] = {1, 3, 3, 1, 3, 3, 3};
  int size = 0;
  for (int i = 0; i < 7; i++)
    if (spec & (1 << i)) size += fsz[i];
  if (!size) return;
  const int num = m->sensor_dim[s] / size;
  real* out = d->sensordata + m->sensor_adr[s];
  const int maxm = m->opt_contact_sensor_maxmatch;
  int ids[256];
  real dirs[256], crit[256];
  int nmatch = 0;
  /* every constraint contact of the world, with rows or not (sensor.py:2313-2316; a contact without rows
   * has zero force, contact_force_local) */
  for (int c = 0; c < d->ncon[0]; c++) {
    const real dir = contact_match(m, d, s, c);
    if (dir == 0) continue;
    const int k = nmatch++;
    if (k >= maxm || k >= 256) continue;
    ids[k] = c;
    dirs[k] = dir;
    if (reduce == 1) crit[k] = d->con_dist[c];
    else if (reduce == 2) {
      real f[6];
      contact_force_local(m, d, c, f);
      crit[k] = -(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
    }
  }
  const int nkept = nmatch < maxm ? (nmatch < 256 ? nmatch : 256) : (maxm < 256 ? maxm : 256);
  if (reduce == 3) {
    real np[3] = {0, 0, 0}, nf[3] = {0, 0, 0}, nt[3] = {0, 0, 0}, w = 0, c3[3];
    for (int k = 0; k < nkept; k++) {
      const int c = ids[k];
      real f[6], fg[3], tg[3];
      contact_force_local(m, d, c, f);
      const real wk = sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
      for (int i = 0; i < 3; i++) np[i] += wk * d->con_pos[3 * c + i];
      w += wk;
      const real* F = d->con_frame + 9 * c;
      for (int i = 0; i < 3; i++) {
        fg[i] = dirs[k] * (F[i] * f[0] + F[3 + i] * f[1] + F[6 + i] * f[2]);
        tg[i] = dirs[k] * (F[i] * f[3] + F[3 + i] * f[4] + F[6 + i] * f[5]);
      }
      cross3(c3, d->con_pos + 3 * c, fg);
      for (int i = 0; i < 3; i++) { nf[i] += fg[i]; nt[i] += tg[i] + c3[i]; }
    }
    for (int i = 0; i < 3; i++) np[i] /= (w > MINVAL ? w : MINVAL);
    cross3(c3, np, nf);
    for (int i = 0; i < 3; i++) nt[i] -= c3[i];
    int a = 0;
    if (spec & 1) out[a++] = nmatch;
    if (spec & 2) for (int i = 0; i < 3; i++) out[a++] = nf[i];
    if (spec & 4) for (int i = 0; i < 3; i++) out[a++] = nt[i];
    if (spec & 8) out[a++] = 0;
    if (spec & 16) for (int i = 0; i < 3; i++) out[a++] = np[i];
    if (spec & 32) { out[a++] = 1; out[a++] = 0; out[a++] = 0; }
    if (spec & 64) { out[a++] = 0; out[a++] = 1; out[a++] = 0; }
    return;
  }
  if (reduce == 1 || reduce == 2)
    for (int i = 1; i < nkept; i++) /* stable insertion sort by criteria */
      for (int j = i; j > 0 && crit[j] < crit[j - 1]; j--) {
        real tc = crit[j]; crit[j] = crit[j - 1]; crit[j - 1] = tc;
        real td = dirs[j]; dirs[j] = dirs[j - 1]; dirs[j - 1] = td;
        int ti = ids[j]; ids[j] = ids[j - 1]; ids[j - 1] = ti;
      }
  const int nslots = nkept < num ? nkept : num;
  for (int i = 0; i < nslots; i++) {
    const int c = ids[i];
    const real dir = dirs[i];
    real* o = out + i * size;
    int a = 0;
    real f[6];
    contact_force_local(m, d, c, f);
    const real* F = d->con_frame + 9 * c;
    if (spec & 1) o[a++] = nmatch;
    if (spec & 2) { o[a++] = f[0]; o[a++] = f[1]; o[a++] = dir * f[2]; }
    if (spec & 4) { o[a++] = f[3]; o[a++] = f[4]; o[a++] = dir * f[5]; }
    if (spec & 8) o[a++] = d->con_dist[c];
    if (spec & 16) for (int j = 0; j < 3; j++) o[a++] = d->con_pos[3 * c + j];
    if (spec & 32) for (int j = 0; j < 3; j++) o[a++] = dir * F[j];
    if (spec & 64) for (int j = 0; j < 3; j++) o[a++] = dir * F[3 + j];
  }
  for (int i = nslots; i < num; i++)
    for (int j = 0; j < size; j++) out[i * size + j] = 0;
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
      case SENS_GEOMDIST: case SENS_GEOMNORMAL: case SENS_GEOMFROMTO: collision_sensor(m, d, s); continue;
      case SENS_CONTACT: contact_sensor(m, d, s); continue;
      case SENS_TACTILE: tactile_sensor(m, d, s); continue;
      case SENS_INSIDESITE: {
        const real *p, *R;
        int body;
        obj_frame(m, d, m->sensor_objtype[s], id, &p, &R, &body);
        const int site = m->sensor_refid[s];
        v[0] = inside_geom(d->site_xpos + 3 * site, d->site_xmat + 9 * site, m->site_size + 3 * site, m->site_type[site], p);
        break;
      }
      default: continue;
    }
    sensor_write(m, d, s, v, dim);
  }
}
