/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, fp64 by default, fp32 with -DORC_REAL=float) of the
 * mujoco_warp `step` path for one world at a time.  Each function cites the
 * reference file:line it restates.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product never does.
 *
 * Parity status: the reference (Warp + MuJoCo C) cannot run in this image, so
 * this oracle is pinned by (a) the reference's MuJoCo-free known-answer tests
 * (math_test.py segment/segment and triangular-index KATs) and (b) analytic
 * invariants (see tests/test_oracle.py).  Whole-pipeline outputs are otherwise
 * "parity unpinned" against MuJoCo C.
 *
 * Field lists are X-macros so that the Python ctypes side can build the exact
 * same structs by parsing this header (tests/oracle_ctypes.py).
 */
#ifndef MJW_ORACLE_H
#define MJW_ORACLE_H

#ifndef ORC_REAL
#define ORC_REAL double
#endif
typedef ORC_REAL real;

/* ---- model: int scalars ---- */
#define ORC_MODEL_INT_SCALARS(X)                                                                   \
  X(nq) X(nv) X(nu) X(na) X(nbody) X(njnt) X(ngeom) X(nsite) X(ncam) X(nlight) X(nmocap)          \
  X(nxn) X(nmaxpyramid) X(neq) X(nsensor) X(nsensordata) X(opt_integrator) X(opt_cone) X(opt_solver) X(opt_iterations)             \
  X(opt_ls_iterations) X(opt_disableflags) X(opt_enableflags) X(opt_broadphase_filter) X(opt_ls_parallel) \
  X(opt_ccd_iterations) X(ccd_epa_iterations)                                                      \
  X(is_sparse) X(nflex) X(nflexvert) X(nflexedge) X(nflexelem) X(nflexelemdata) X(nmesh) X(nmeshvert)   \
  X(ntendon) X(nwrap) X(nJten) X(npair) X(ngravcomp) X(has_fluid) X(nhfield) X(nhfielddata) X(opt_contact_sensor_maxmatch)          \
  X(nmeshpoly) X(nmeshpolyvert) X(nmeshpolymap) X(nflexelemedge) X(nflexshelldata) X(nmeshnormal)

/* ---- model: real scalars ---- */
#define ORC_MODEL_REAL_SCALARS(X)                                                                  \
  X(opt_timestep) X(opt_tolerance) X(opt_ls_tolerance) X(opt_impratio_invsqrt) X(stat_meaninertia)         \
  X(opt_ccd_tolerance) X(opt_density) X(opt_viscosity) X(opt_ls_parallel_min_step)

/* ---- model: real arrays (name, element count) ---- */
#define ORC_MODEL_REAL_ARRAYS(X)                                                                   \
  X(opt_gravity, 3) X(opt_magnetic, 3) X(opt_wind, 3) X(sensor_cutoff, nsensor)                    \
  X(qpos0, nq) X(qpos_spring, nq)                                                                  \
  X(body_pos, nbody * 3) X(body_quat, nbody * 4) X(body_ipos, nbody * 3) X(body_iquat, nbody * 4) \
  X(body_mass, nbody) X(body_subtreemass, nbody) X(body_inertia, nbody * 3)                       \
  X(body_invweight0, nbody * 2) X(body_gravcomp, nbody) X(geom_fluid, ngeom * 12)                  \
  X(jnt_solref, njnt * 2) X(jnt_solimp, njnt * 5) X(jnt_pos, njnt * 3) X(jnt_axis, njnt * 3)      \
  X(jnt_stiffness, njnt) X(jnt_range, njnt * 2) X(jnt_actfrcrange, njnt * 2) X(jnt_margin, njnt)  \
  X(dof_solref, nv * 2) X(dof_solimp, nv * 5) X(dof_frictionloss, nv) X(dof_armature, nv)         \
  X(dof_damping, nv) X(dof_invweight0, nv)                                                         \
  X(geom_solmix, ngeom) X(geom_solref, ngeom * 2) X(geom_solimp, ngeom * 5) X(geom_size, ngeom * 3) \
  X(geom_aabb, ngeom * 6) X(geom_rbound, ngeom) X(geom_pos, ngeom * 3) X(geom_quat, ngeom * 4)    \
  X(geom_friction, ngeom * 3) X(geom_margin, ngeom) X(geom_gap, ngeom)                             \
  X(site_pos, nsite * 3) X(site_quat, nsite * 4) X(site_size, nsite * 3)                                                \
  X(cam_pos, ncam * 3) X(cam_quat, ncam * 4) X(cam_poscom0, ncam * 3) X(cam_pos0, ncam * 3)       \
  X(cam_mat0, ncam * 9) X(cam_fovy, ncam) X(cam_sensorsize, ncam * 2) X(cam_intrinsic, ncam * 4)    \
  X(light_pos, nlight * 3) X(light_dir, nlight * 3) X(light_poscom0, nlight * 3)                  \
  X(light_pos0, nlight * 3) X(light_dir0, nlight * 3)                                              \
  X(actuator_dynprm, nu * 10) X(actuator_gainprm, nu * 10) X(actuator_biasprm, nu * 10)           \
  X(actuator_ctrlrange, nu * 2) X(actuator_forcerange, nu * 2) X(actuator_actrange, nu * 2)       \
  X(actuator_gear, nu * 6) X(actuator_cranklength, nu) X(actuator_acc0, nu) X(actuator_lengthrange, nu * 2)                   \
  X(eq_solref, neq * 2) X(eq_solimp, neq * 5) X(eq_data, neq * 11)                               \
  X(flex_radius, nflex) X(flex_margin, nflex) X(flex_damping, nflex) X(flex_friction, nflex * 3)  \
  X(flex_vert, nflexvert * 3) X(flexedge_length0, nflexedge) X(flexedge_invweight0, nflexedge)    \
  X(flex_stiffness, nflexelem * 21) X(flex_bending, nflexedge * 17) X(mesh_vert, nmeshvert * 3) X(mesh_normal, nmeshnormal * 3)      \
  X(mesh_polynormal, nmeshpoly * 3)                                                                \
  X(hfield_size, nhfield * 4) X(hfield_data, nhfielddata)                                          \
  X(tendon_stiffness, ntendon) X(tendon_damping, ntendon) X(tendon_frictionloss, ntendon)          \
  X(tendon_armature, ntendon) X(tendon_margin, ntendon) X(tendon_range, ntendon * 2)               \
  X(tendon_lengthspring, ntendon * 2) X(tendon_solref_lim, ntendon * 2) X(tendon_solimp_lim, ntendon * 5) \
  X(tendon_solref_fri, ntendon * 2) X(tendon_solimp_fri, ntendon * 5) X(tendon_invweight0, ntendon) X(tendon_length0, ntendon) \
  X(tendon_actfrcrange, ntendon * 2) X(wrap_prm, nwrap)                                            \
  X(pair_solref, npair * 2) X(pair_solreffriction, npair * 2) X(pair_solimp, npair * 5)           \
  X(pair_margin, npair) X(pair_gap, npair) X(pair_friction, npair * 5)

/* ---- model: int arrays (name, element count) ---- */
#define ORC_MODEL_INT_ARRAYS(X)                                                                    \
  X(body_parentid, nbody) X(body_rootid, nbody) X(body_weldid, nbody) X(body_mocapid, nbody)      \
  X(body_jntnum, nbody) X(body_jntadr, nbody) X(body_dofnum, nbody) X(body_dofadr, nbody)         \
  X(jnt_type, njnt) X(jnt_qposadr, njnt) X(jnt_dofadr, njnt) X(jnt_bodyid, njnt)                  \
  X(jnt_limited, njnt) X(jnt_actfrclimited, njnt) X(jnt_actgravcomp, njnt)                         \
  X(body_geomadr, nbody) X(body_geomnum, nbody) X(body_fluid_ellipsoid, nbody)                    \
  X(dof_bodyid, nv) X(dof_jntid, nv) X(dof_parentid, nv)                                           \
  X(geom_type, ngeom) X(geom_condim, ngeom) X(geom_bodyid, ngeom) X(geom_priority, ngeom)         \
  X(site_bodyid, nsite) X(site_type, nsite)                                                                      \
  X(cam_mode, ncam) X(cam_bodyid, ncam) X(cam_targetbodyid, ncam) X(cam_resolution, ncam * 2)     \
  X(light_mode, nlight) X(light_bodyid, nlight) X(light_targetbodyid, nlight)                     \
  X(actuator_trntype, nu) X(actuator_dyntype, nu) X(actuator_gaintype, nu)                        \
  X(actuator_biastype, nu) X(actuator_trnid, nu * 2) X(actuator_actadr, nu) X(actuator_actnum, nu) \
  X(actuator_ctrllimited, nu) X(actuator_forcelimited, nu) X(actuator_actlimited, nu)             \
  X(actuator_actearly, nu)                                                                         \
  X(nxn_geom_pair, nxn * 2) X(nxn_pairid, nxn * 2) X(pair_dim, npair)                              \
  X(eq_type, neq) X(eq_obj1id, neq) X(eq_obj2id, neq) X(eq_objtype, neq)                           \
  X(sensor_type, nsensor) X(sensor_datatype, nsensor) X(sensor_objtype, nsensor)                   \
  X(sensor_objid, nsensor) X(sensor_reftype, nsensor) X(sensor_refid, nsensor)                     \
  X(sensor_adr, nsensor) X(sensor_dim, nsensor) X(sensor_needstage, nsensor) X(sensor_intprm, nsensor * 3) \
  X(geom_contype, ngeom) X(geom_conaffinity, ngeom)                                                \
  X(flex_dim, nflex) X(flex_vertadr, nflex) X(flex_vertnum, nflex) X(flex_edgeadr, nflex)          \
  X(flex_edgenum, nflex) X(flex_elemadr, nflex) X(flex_elemnum, nflex) X(flex_elemdataadr, nflex)  \
  X(flex_elemedgeadr, nflex) X(flex_contype, nflex) X(flex_conaffinity, nflex) X(flex_condim, nflex) \
  X(flex_centered, nflex) X(flex_vertbodyid, nflexvert) X(flex_vertflexid, nflexvert)              \
  X(flex_edge, nflexedge * 2) X(flex_edgeflap, nflexedge * 2) X(flex_elem, nflexelemdata)          \
  X(flex_elemedge, nflexelemedge) X(flex_shellnum, nflex) X(flex_shelldataadr, nflex) X(flex_shell, nflexshelldata) X(mesh_normaladr, nmesh) X(mesh_vertadr, nmesh) X(mesh_vertnum, nmesh) X(geom_dataid, ngeom) \
  X(mesh_polyadr, nmesh) X(mesh_polynum, nmesh) X(mesh_polyvertadr, nmeshpoly) X(mesh_polyvertnum, nmeshpoly) \
  X(mesh_polyvert, nmeshpolyvert) X(mesh_polymapadr, nmeshvert) X(mesh_polymapnum, nmeshvert) X(mesh_polymap, nmeshpolymap) \
  X(hfield_nrow, nhfield) X(hfield_ncol, nhfield) X(hfield_adr, nhfield)                          \
  X(tendon_adr, ntendon) X(tendon_num, ntendon) X(tendon_limited, ntendon) X(tendon_actfrclimited, ntendon) \
  X(wrap_objid, nwrap) X(wrap_type, nwrap) X(ten_J_rownnz, ntendon) X(ten_J_rowadr, ntendon) X(ten_J_colind, nJten)

/* ---- per-world data: real arrays (name, element count per world) ---- */
#define ORC_DATA_REAL_ARRAYS(X)                                                                    \
  X(time, 1) X(qpos, nq) X(qvel, nv) X(act, na) X(ctrl, nu) X(qacc_warmstart, nv)                 \
  X(qfrc_applied, nv) X(xfrc_applied, nbody * 6) X(mocap_pos, nmocap * 3) X(mocap_quat, nmocap * 4) \
  X(qacc, nv) X(act_dot, na)                                                                       \
  X(xpos, nbody * 3) X(xquat, nbody * 4) X(xmat, nbody * 9) X(xipos, nbody * 3) X(ximat, nbody * 9) \
  X(xanchor, njnt * 3) X(xaxis, njnt * 3) X(geom_xpos, ngeom * 3) X(geom_xmat, ngeom * 9)         \
  X(site_xpos, nsite * 3) X(site_xmat, nsite * 9) X(cam_xpos, ncam * 3) X(cam_xmat, ncam * 9)     \
  X(light_xpos, nlight * 3) X(light_xdir, nlight * 3)                                              \
  X(subtree_com, nbody * 3) X(subtree_linvel, nbody * 3) X(subtree_angmom, nbody * 3) X(cdof, nv * 6) X(cinert, nbody * 10) X(crb, nbody * 10)              \
  X(qM, nv * nv) X(qLD, nv * nv)                                                                   \
  X(actuator_length, nu) X(actuator_moment, nu * nv) X(actuator_velocity, nu) X(actuator_force, nu) \
  X(cvel, nbody * 6) X(cdof_dot, nv * 6) X(qfrc_bias, nv) X(qfrc_spring, nv) X(qfrc_damper, nv)   \
  X(qfrc_gravcomp, nv) X(qfrc_fluid, nv)                                                           \
  X(qfrc_passive, nv) X(qfrc_actuator, nv) X(qfrc_smooth, nv) X(qacc_smooth, nv)                  \
  X(qfrc_constraint, nv) X(cacc, nbody * 6) X(cfrc_int, nbody * 6) X(cfrc_ext, nbody * 6)         \
  X(sensordata, nsensordata)                                                                       \
  X(efc_J, njmax * nv) X(efc_pos, njmax) X(efc_margin, njmax) X(efc_D, njmax) X(efc_vel, njmax)   \
  X(efc_aref, njmax) X(efc_frictionloss, njmax) X(efc_force, njmax) X(efc_Ma, nv)                 \
  X(efc_prm, njmax * 9) /* per row, the inputs of efc_row besides pos_aref / vel (tests only) */     \
  X(con_dist, nconmax) X(con_pos, nconmax * 3) X(con_frame, nconmax * 9)                          \
  X(con_includemargin, nconmax) X(con_friction, nconmax * 5) X(con_solref, nconmax * 2)           \
  X(con_solreffriction, nconmax * 2) X(con_solimp, nconmax * 5) X(solver_cost, 1)                 \
  X(flexvert_xpos, nflexvert * 3) X(flexedge_length, nflexedge) X(flexedge_velocity, nflexedge)   \
  X(flexedge_J, nflexedge * 6) X(ten_length, ntendon) X(ten_velocity, ntendon) X(ten_J, nJten)

/* ---- per-world data: int arrays ---- */
#define ORC_DATA_INT_ARRAYS(X)                                                                     \
  X(ne, 1) X(nf, 1) X(nl, 1) X(nefc, 1) X(ncon, 1) X(ncollision, 1) X(solver_niter, 1)            \
  X(efc_type, njmax) X(efc_id, njmax) X(efc_state, njmax)                                          \
  X(con_dim, nconmax) X(con_geom, nconmax * 2) X(con_efc_address, nconmax * 10) X(eq_active, neq) \
  X(con_flex, nconmax * 2) X(con_vert, nconmax * 2)

typedef struct orc_model {
#define ORC_DECL_I(name) int name;
#define ORC_DECL_R(name) real name;
#define ORC_DECL_RA(name, n) const real* name;
#define ORC_DECL_IA(name, n) const int* name;
  ORC_MODEL_INT_SCALARS(ORC_DECL_I)
  ORC_MODEL_REAL_SCALARS(ORC_DECL_R)
  ORC_MODEL_REAL_ARRAYS(ORC_DECL_RA)
  ORC_MODEL_INT_ARRAYS(ORC_DECL_IA)
} orc_model;

typedef struct orc_data {
  int njmax;
  int nconmax;
#define ORC_DECL_DRA(name, n) real* name;
#define ORC_DECL_DIA(name, n) int* name;
  ORC_DATA_REAL_ARRAYS(ORC_DECL_DRA)
  ORC_DATA_INT_ARRAYS(ORC_DECL_DIA)
} orc_data;

#ifdef __cplusplus
extern "C" {
#endif

/* batched entry points: `d` points at world 0 of (nworld, ...) arrays */
int orc_real_size(void);
void orc_step(const orc_model* m, const orc_data* d, int nworld, int nthread);
void orc_forward(const orc_model* m, const orc_data* d, int nworld, int nthread);
/* stage entry points (one stage for all worlds) */
void orc_fwd_position(const orc_model* m, const orc_data* d, int nworld);
void orc_fwd_velocity(const orc_model* m, const orc_data* d, int nworld);
void orc_fwd_actuation(const orc_model* m, const orc_data* d, int nworld);
void orc_fwd_acceleration(const orc_model* m, const orc_data* d, int nworld);
void orc_solve(const orc_model* m, const orc_data* d, int nworld);
void orc_euler(const orc_model* m, const orc_data* d, int nworld);
/* math KATs (math_test.py) */
void orc_closest_segment_to_segment_points(const real* a0, const real* a1, const real* b0, const real* b1,
                                           real* best_a, real* best_b);
int orc_upper_tri_index(int n, int i, int j);
int orc_upper_trid_index(int n, int i, int j);
real orc_halton(int index, int base);
/* collision KATs (collision_gjk_test.py, collision_primitive_core_test.py) */
int orc_kat_hfield_support(const real* prism, const real* dir, real margin, real* out);
int orc_kat_ccd(const int* type, const real* pos, const real* mat, const real* size, const real* mesh_vert, const int* vertadr,
                const int* vertnum, real margin, real tolerance, int iterations, int multiccd, real* out);
void orc_kat_efc_row(int disableflags, real timestep, real pos_aref, real pos_imp, real invweight, const real* solref,
                     const real* solimp, real vel, real* out);
int orc_kat_ccd_model(const int* type, const real* pos, const real* mat, const real* size, const real* mesh_vert, const int* vertadr,
                      const int* vertnum, real margin, real tolerance, int iterations, int multiccd, const orc_model* pm,
                      const int* meshid, real* out);
int orc_kat_wrap(int fn, const real* a, int ind, real radius, real* out);
int orc_kat_geom_triangle(int gt, const real* gp, const real* gr, const real* gs, const real* tri, real tr, real* out);
void orc_ctrl_noise(const orc_model* m, real* ctrl, const real* center, int ncenter, int step, real std,
                    real rate, int nworld, int world_offset);

#ifdef __cplusplus
}
#endif
#endif
