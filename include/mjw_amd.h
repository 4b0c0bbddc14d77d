/*
 * mjw_amd.h -- C ABI of the MI355X batched MuJoCo stepper (libmjw_amd.so).
 *
 * Drop-in boundary for the `mjw.step(m, d)` path of mujoco_warp.  Each entry
 * point replaces one reference function (file:line in mujoco_warp/_src):
 *
 *   mjw_step              <- forward.step                 forward.py:1003-1018
 *   mjw_forward           <- forward.forward              forward.py:972-1000
 *   mjw_fwd_position      <- forward.fwd_position         forward.py:513-537
 *   mjw_contact_rows      <- constraint.make_constraint   constraint.py:2718-2779 (contact rows again from
 *                            d.contact after a contactfilter callback, collision_driver.py:788-789)
 *   mjw_fwd_velocity      <- forward.fwd_velocity         forward.py:592-613
 *   mjw_fwd_actuation     <- forward.fwd_actuation        forward.py:836-927
 *   mjw_fwd_acceleration  <- forward.fwd_acceleration     forward.py:949-969
 *   mjw_solve             <- solver.solve                 solver.py:3296-3343
 *   mjw_euler             <- forward.euler                forward.py:326-354
 *   mjw_stage             <- smooth.kinematics / com_pos / camlight / tendon / crb / transmission /
 *                            com_vel / rne, passive.passive, constraint.make_constraint (one stage, below)
 *   mjw_sensor            <- sensor.sensor_pos/_vel/_acc  sensor.py:761,1377,2447
 *   mjw_ctrl_noise        <- benchmark.ctrl_noise         _src/benchmark.py:41-83
 *
 * Ownership: the caller owns every buffer (device pointers below); the library
 * never allocates or frees device memory and keeps no global mutable state.
 * All launches are asynchronous on the caller's HIP stream (graph capturable).
 * Return value: 0 on success, nonzero HIP error code otherwise
 * (mjw_last_error() gives the message).
 *
 * Field lists are X-macros: the Python host (mujoco_warp_amd/_lib.py) parses
 * them to build byte-identical ctypes structs.
 */
#ifndef MJW_AMD_H
#define MJW_AMD_H

#include <stdint.h>

#define MJW_ABI_VERSION 34

/* ---- model: int scalars ---- */
#define MJW_MODEL_INT_SCALARS(X)                                                                   \
  X(nq) X(nv) X(nu) X(na) X(nbody) X(njnt) X(ngeom) X(nsite) X(ncam) X(nlight) X(nmocap)          \
  X(nxn) X(nlevel) X(nlimited) X(nlimited_ball) X(nmaxcondim) X(nmaxpyramid) X(nv_pad) X(nJmom)    \
  X(neq) X(neq_cw)                                                                                 \
  X(nsensor) X(nsensordata) X(sensor_rne_postconstraint) X(nsensor_acc)                           \
  X(nxn_ccd) X(nxn_box) X(opt_ccd_iterations) X(ccd_epa_iterations)                                           \
  X(opt_integrator) X(opt_cone) X(opt_solver) X(opt_iterations) X(opt_ls_iterations)             \
  X(opt_disableflags) X(opt_enableflags) X(opt_broadphase_filter) X(opt_ls_parallel)               \
  X(is_sparse) X(nM) X(ntree) X(njrow)                                                             \
  X(nflex) X(nflexvert) X(nflexedge) X(nflexelem) X(nflexelemdata) X(nflexinc) X(nflexcg) X(nplane) \
  X(nflexelemedge) X(nflexshelldata)                                                               \
  X(nmesh) X(nmeshvert) X(ntendon) X(nwrap) X(nJten) X(ten_maxnnz) X(nmuscle) X(sp_nH)   \
  X(npair) X(ngravcomp) X(has_fluid) X(nten_spatial) X(act_maxnnz) X(nbodytrn) X(nsitetrn)             \
  X(nsensorcollision) X(nsensorccd) X(nhfield) X(nhfielddata) X(opt_contact_sensor_maxmatch)           \
  X(nmeshpoly) X(nmeshpolyvert) X(nmeshpolymap) X(nmaxpolygon) X(nmaxmeshdeg) X(nsensortaxel) X(nmeshnormal) X(nsensorcontact)

/* ---- model: float arrays, batchable (leading dim nb = 1 or nworld, indexed worldid % nb) ---- */
#define MJW_MODEL_REAL_ARRAYS(X)                                                                   \
  X(opt_timestep, 1) X(opt_tolerance, 1) X(opt_ls_tolerance, 1) X(opt_impratio_invsqrt, 1)        \
  X(opt_ccd_tolerance, 1)                                                                          \
  X(opt_gravity, 3) X(opt_magnetic, 3) X(stat_meaninertia, 1)                                      \
  X(opt_wind, 3) X(opt_density, 1) X(opt_viscosity, 1) X(opt_ls_parallel_min_step, 1)             \
  X(qpos0, nq) X(qpos_spring, nq)                                                                  \
  X(body_pos, nbody * 3) X(body_quat, nbody * 4) X(body_ipos, nbody * 3) X(body_iquat, nbody * 4) \
  X(body_mass, nbody) X(body_subtreemass, nbody) X(body_inertia, nbody * 3)                       \
  X(body_invweight0, nbody * 2) X(body_gravcomp, nbody)                                            \
  X(jnt_solref, njnt * 2) X(jnt_solimp, njnt * 5) X(jnt_pos, njnt * 3) X(jnt_axis, njnt * 3)      \
  X(jnt_stiffness, njnt) X(jnt_range, njnt * 2) X(jnt_actfrcrange, njnt * 2) X(jnt_margin, njnt)  \
  X(dof_solref, nv * 2) X(dof_solimp, nv * 5) X(dof_frictionloss, nv) X(dof_armature, nv)         \
  X(dof_damping, nv) X(dof_invweight0, nv)                                                         \
  X(geom_solmix, ngeom) X(geom_solref, ngeom * 2) X(geom_solimp, ngeom * 5) X(geom_size, ngeom * 3) \
  X(geom_aabb, ngeom * 6) X(geom_rbound, ngeom) X(geom_pos, ngeom * 3) X(geom_quat, ngeom * 4)    \
  X(geom_friction, ngeom * 3) X(geom_margin, ngeom) X(geom_gap, ngeom) X(geom_fluid, ngeom * 12)  \
  X(site_pos, nsite * 3) X(site_quat, nsite * 4) X(site_size, nsite * 3)                                                \
  X(cam_pos, ncam * 3) X(cam_quat, ncam * 4) X(cam_poscom0, ncam * 3) X(cam_pos0, ncam * 3)       \
  X(cam_mat0, ncam * 9) X(cam_fovy, ncam) X(cam_sensorsize, ncam * 2) X(cam_intrinsic, ncam * 4)    \
  X(light_pos, nlight * 3) X(light_dir, nlight * 3) X(light_poscom0, nlight * 3)                  \
  X(light_pos0, nlight * 3) X(light_dir0, nlight * 3)                                              \
  X(actuator_dynprm, nu * 10) X(actuator_gainprm, nu * 10) X(actuator_biasprm, nu * 10)           \
  X(actuator_ctrlrange, nu * 2) X(actuator_forcerange, nu * 2) X(actuator_actrange, nu * 2)       \
  X(actuator_gear, nu * 6) X(actuator_acc0, nu) X(actuator_lengthrange, nu * 2) X(actuator_cranklength, nu)                   \
  X(eq_solref, neq * 2) X(eq_solimp, neq * 5) X(eq_data, neq * 11)                               \
  X(sensor_cutoff, nsensor)                                                                        \
  X(flex_radius, nflex) X(flex_margin, nflex) X(flex_damping, nflex) X(flex_friction, nflex * 3)  \
  X(flexedge_length0, nflexedge) X(flexedge_invweight0, nflexedge)                                \
  X(flex_stiffness, nflexelem * 21) X(flex_bending, nflexedge * 17) X(mesh_normal, nmeshnormal * 3) \
  X(mesh_vert, nmeshvert * 3) X(hfield_size, nhfield * 4) X(hfield_data, nhfielddata)             \
  X(mesh_polynormal, nmeshpoly * 3)                                                                \
  X(tendon_stiffness, ntendon) X(tendon_damping, ntendon) X(tendon_frictionloss, ntendon)          \
  X(tendon_armature, ntendon) X(tendon_margin, ntendon) X(tendon_range, ntendon * 2)               \
  X(tendon_lengthspring, ntendon * 2) X(tendon_solref_lim, ntendon * 2) X(tendon_solimp_lim, ntendon * 5) \
  X(tendon_solref_fri, ntendon * 2) X(tendon_solimp_fri, ntendon * 5) X(tendon_invweight0, ntendon)  \
  X(tendon_actfrcrange, ntendon * 2) X(tendon_length0, ntendon) X(wrap_prm, nwrap) X(wrap_pulley_scale, nwrap)                                          \
  X(pair_solref, npair * 2) X(pair_solreffriction, npair * 2) X(pair_solimp, npair * 5)           \
  X(pair_margin, npair) X(pair_gap, npair) X(pair_friction, npair * 5)

/* ---- model: int arrays (never batched) ---- */
#define MJW_MODEL_INT_ARRAYS(X)                                                                    \
  X(body_parentid, nbody) X(body_rootid, nbody) X(body_weldid, nbody) X(body_mocapid, nbody)      \
  X(body_jntnum, nbody) X(body_jntadr, nbody) X(body_dofnum, nbody) X(body_dofadr, nbody)         \
  X(body_subtree_end, nbody) X(body_level, nbody) X(level_body, nbody) X(level_adr, nlevel + 1)    \
  X(jnt_type, njnt) X(jnt_qposadr, njnt) X(jnt_dofadr, njnt) X(jnt_bodyid, njnt)                  \
  X(jnt_limited, njnt) X(jnt_actfrclimited, njnt) X(jnt_limited_slide_hinge_adr, nlimited)        \
  X(jnt_limited_ball_adr, nlimited_ball) X(jnt_actgravcomp, njnt)                                 \
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
  X(nxn_geom_pair, nxn * 2) X(nxn_pairid, nxn * 2) X(nxn_ccdid, nxn) X(pair_dim, npair)            \
  X(eq_type, neq) X(eq_obj1id, neq) X(eq_obj2id, neq) X(eq_objtype, neq)                                             \
  X(sensor_type, nsensor) X(sensor_datatype, nsensor) X(sensor_objtype, nsensor)                   \
  X(sensor_objid, nsensor) X(sensor_reftype, nsensor) X(sensor_refid, nsensor)                     \
  X(sensor_adr, nsensor) X(sensor_dim, nsensor) X(sensor_needstage, nsensor) X(sensor_intprm, nsensor * 3) \
  X(sensor_collision_adr, nsensor) X(sensor_collision_num, nsensor) X(sensor_collision_pair, nsensorcollision * 4) \
  X(M_rownnz, nv) X(M_rowadr, nv) X(M_colind, nM) X(tree_dofadr, ntree + 1)                        \
  X(flex_dim, nflex) X(flex_vertadr, nflex) X(flex_edgeadr, nflex) X(flex_edgenum, nflex)          \
  X(flex_elemadr, nflex) X(flex_elemnum, nflex) X(flex_elemdataadr, nflex) X(flex_elemedgeadr, nflex) \
  X(flex_condim, nflex) X(flex_cgeomadr, nflex + 1) X(flex_cgeom, nflexcg) X(plane_geom, nplane)   \
  X(flex_vertbodyid, nflexvert) X(flex_vertflexid, nflexvert) X(flex_edge, nflexedge * 2)          \
  X(flex_edgeflap, nflexedge * 2) X(flex_elem, nflexelemdata) X(flex_elemedge, nflexelemedge)      \
  X(flex_shellnum, nflex) X(flex_shelldataadr, nflex) X(flex_shell, nflexshelldata)               \
  X(taxel_vertadr, nsensortaxel) X(taxel_sensorid, nsensortaxel) X(mesh_normaladr, nmesh) X(mesh_normalnum, nmesh) \
  X(flexvert_incadr, nflexvert + 1) X(flexvert_inc, nflexinc)                                     \
  X(mesh_vertadr, nmesh) X(mesh_vertnum, nmesh) X(geom_dataid, ngeom)                            \
  X(mesh_polyadr, nmesh) X(mesh_polynum, nmesh) X(mesh_polyvertadr, nmeshpoly) X(mesh_polyvertnum, nmeshpoly) \
  X(mesh_polyvert, nmeshpolyvert) X(mesh_polymapadr, nmeshvert) X(mesh_polymapnum, nmeshvert) X(mesh_polymap, nmeshpolymap) \
  X(hfield_nrow, nhfield) X(hfield_ncol, nhfield) X(hfield_adr, nhfield)                          \
  X(tendon_adr, ntendon) X(tendon_num, ntendon) X(tendon_limited, ntendon) X(tendon_actfrclimited, ntendon) \
  X(wrap_objid, nwrap) X(wrap_type, nwrap) X(ten_J_rownnz, ntendon) X(ten_J_rowadr, ntendon) X(ten_J_colind, nJten)

/* ---- data: float arrays, (nworld, count) world-major like mujoco_warp types.Data ----
 * Sparse models (is_sparse, the reference's io.py:67-74 switch) store qM / qLD as (nworld, nM) rows of
 * ancestors ascending then the diagonal (M_rowadr / M_colind), and efc_J as (nworld, njmax_pad, njrow)
 * stored slot-major (slot k of row r at [k * njmax_pad + r]) with efc_J_colind / efc_J_rownnz; dense models keep qM (nv_pad, nv_pad), qLD (nv, nv), efc_J
 * (njmax_pad, nv_pad).  sp_* / efc_JT_* / sp_cnt are sparse-path workspace (size 0 when dense); ncon_world holds a
 * world's contact-pool range (first slot, count / span): the sparse path's, and the dense contact-rows pass's;
 * sp_idx16 holds the CG's 16-bit copies of efc_J_colind and of the transposed index's rows (two uint16 per int).
 * world_order / world_key: the dense path's longest-first world order (a permutation of the worlds, rebuilt
 * every step from the previous step's solver iterations) and each world's iteration bucket. */
#define MJW_DATA_REAL_ARRAYS(X)                                                                    \
  X(time, 1) X(qpos, nq) X(qvel, nv) X(act, na) X(ctrl, nu) X(qacc_warmstart, nv)                 \
  X(qfrc_applied, nv) X(xfrc_applied, nbody * 6) X(mocap_pos, nmocap * 3) X(mocap_quat, nmocap * 4) \
  X(qacc, nv) X(act_dot, na) X(energy, 2)                                                          \
  X(xpos, nbody * 3) X(xquat, nbody * 4) X(xmat, nbody * 9) X(xipos, nbody * 3) X(ximat, nbody * 9) \
  X(xanchor, njnt * 3) X(xaxis, njnt * 3) X(geom_xpos, ngeom * 3) X(geom_xmat, ngeom * 9)         \
  X(site_xpos, nsite * 3) X(site_xmat, nsite * 9) X(cam_xpos, ncam * 3) X(cam_xmat, ncam * 9)     \
  X(light_xpos, nlight * 3) X(light_xdir, nlight * 3)                                              \
  X(subtree_com, nbody * 3) X(subtree_linvel, nbody * 3) X(subtree_angmom, nbody * 3) X(cdof, nv * 6) X(cinert, nbody * 10) X(crb, nbody * 10)              \
  X(qM, nv_pad * nv_pad) X(qLD, nv * nv)                                                           \
  X(actuator_length, nu) X(actuator_moment, nJmom) X(actuator_velocity, nu) X(actuator_force, nu) \
  X(cvel, nbody * 6) X(cdof_dot, nv * 6) X(qfrc_bias, nv) X(qfrc_spring, nv) X(qfrc_damper, nv)   \
  X(qfrc_gravcomp, nv) X(qfrc_fluid, nv) X(qfrc_passive, nv) X(qfrc_actuator, nv) X(qfrc_smooth, nv) \
  X(qacc_smooth, nv) X(qfrc_constraint, nv) X(cacc, nbody * 6) X(cfrc_int, nbody * 6)             \
  X(cfrc_ext, nbody * 6)                                                                           \
  X(efc_J, njmax_pad * nv_pad) X(efc_pos, njmax) X(efc_margin, njmax) X(efc_D, njmax_pad)         \
  X(efc_vel, njmax) X(efc_aref, njmax) X(efc_frictionloss, njmax) X(efc_force, njmax)             \
  X(efc_Ma, nv) X(sensordata, nsensordata) X(ccd_out, nxn_ccd * 32)                                 \
  X(qpos_t0, nq) X(qvel_t0, nv) X(act_t0, na) X(qvel_rk, nv) X(qacc_rk, nv) X(act_dot_rk, na)     \
  X(flexvert_xpos, nflexvert * 3) X(flexedge_length, nflexedge) X(flexedge_velocity, nflexedge)   \
  X(flexedge_J, nflexedge * 6) X(flex_frc, nflexelem * 12 + nflexedge * 12)                       \
  X(sp_body, nbody * 6) X(sp_vec, nv * 10) X(sp_row, njmax * 3) X(sp_LD, nM) X(sp_H, sp_nH * sp_nH) \
  X(efc_JT_val, njmax_pad * njrow)                                                                 \
  X(ten_length, ntendon) X(ten_velocity, ntendon) X(ten_J, nJten)

/* ---- data: int arrays, (nworld, count) ---- */
#define MJW_DATA_INT_ARRAYS(X)                                                                     \
  X(ne, 1) X(nf, 1) X(nl, 1) X(nefc, 1) X(solver_niter, 1)                                         \
  X(moment_rownnz, nu) X(moment_rowadr, nu) X(moment_colind, nJmom)                                \
  X(efc_type, njmax) X(efc_id, njmax) X(efc_state, njmax_pad) X(eq_active, neq)                   \
  X(efc_J_colind, njmax_pad * njrow) X(efc_J_rownnz, njmax) X(efc_JT_rowind, njmax_pad * njrow)   \
  X(efc_JT_adr, nv + 1) X(sp_cnt, nv + 1) X(ncon_world, 2)                                        \
  X(sp_idx16, njmax_pad * njrow)                                                                   \
  X(world_order, 1) X(world_key, 1)

/* ---- contact pool: float arrays, (naconmax, count) ---- */
#define MJW_CONTACT_REAL_ARRAYS(X)                                                                 \
  X(contact_dist, 1) X(contact_pos, 3) X(contact_frame, 9) X(contact_includemargin, 1)            \
  X(contact_friction, 5) X(contact_solref, 2) X(contact_solreffriction, 2) X(contact_solimp, 5)

/* ---- contact pool: int arrays, (naconmax, count) ---- */
#define MJW_CONTACT_INT_ARRAYS(X)                                                                  \
  X(contact_dim, 1) X(contact_geom, 2) X(contact_efc_address, nmaxpyramid) X(contact_worldid, 1)  \
  X(contact_type, 1) X(contact_geomcollisionid, 1) X(contact_flex, 2) X(contact_vert, 2)

typedef struct mjw_model_t {
#define MJW_DECL_I(name) int32_t name;
#define MJW_DECL_RA(name, n) const float* name; int32_t name##_nb; int32_t name##_cnt;
#define MJW_DECL_IA(name, n) const int32_t* name;
  MJW_MODEL_INT_SCALARS(MJW_DECL_I)
  MJW_MODEL_REAL_ARRAYS(MJW_DECL_RA)
  MJW_MODEL_INT_ARRAYS(MJW_DECL_IA)
} mjw_model_t;

/* world-order workspace (mjw_data_t.sched): non-null enables the longest-first order (its words are spare since
   round 6: the counter-reset kernel histograms world_key itself) */
#define MJW_SCHED_BUCKETS 32
#define MJW_SCHED_WORDS (2 * MJW_SCHED_BUCKETS + 2)

typedef struct mjw_data_t {
  int32_t nworld;     /* worlds held by these buffers */
  int32_t njmax;      /* max constraint rows per world */
  int32_t njmax_pad;  /* padded row count of efc_J / efc_D / efc_state */
  int32_t naconmax;   /* contact pool capacity (all worlds) */
  int32_t world_offset; /* global id of world 0 (multi-GPU sharding); affects ctrl noise only */
  int32_t pad_;
  int32_t* nacon;      /* (1,) contacts written this step (may exceed naconmax) */
  int32_t* ncollision; /* (1,) broadphase pairs this step; when ncollision == nacon + 1 (one 8-B aligned pair,
                          as put_data allocates them) the step adds both with one 64-bit atomic per world */
  int32_t* sched;      /* (MJW_SCHED_WORDS,) world-order workspace of the dense path: histogram of
                        * the previous step's solver-iteration buckets, bucket cursors, valid flag */
#define MJW_DECL_DRA(name, n) float* name;
#define MJW_DECL_DIA(name, n) int32_t* name;
  MJW_DATA_REAL_ARRAYS(MJW_DECL_DRA)
  MJW_DATA_INT_ARRAYS(MJW_DECL_DIA)
  MJW_CONTACT_REAL_ARRAYS(MJW_DECL_DRA)
  MJW_CONTACT_INT_ARRAYS(MJW_DECL_DIA)
} mjw_data_t;

#ifdef __cplusplus
extern "C" {
#endif

int mjw_abi_version(void);
const char* mjw_last_error(void);
/* sizeof checks for the Python binding */
int mjw_sizeof_model(void);
int mjw_sizeof_data(void);
/* per-world LDS bytes the fused step needs for this model and njmax */
int mjw_lds_bytes(const mjw_model_t* m, int njmax);

/* stream: a hipStream_t (NULL = default stream) */
int mjw_step(const mjw_model_t* m, const mjw_data_t* d, void* stream);
/* mjw_step with timing: hipEvent_t handles recorded on `stream` before the forward kernel,
 * between the forward and the dense factor/solve/euler kernel, and after it (bench.py uses
 * this to time the dominant kernel live; on the generic path only ev_begin/ev_end bracket it).
 * No reference counterpart (the reference times with wp.ScopedTimer/event_trace, benchmark.py). */
int mjw_step_events(const mjw_model_t* m, const mjw_data_t* d, void* stream, void* ev_begin, void* ev_mid, void* ev_end);

/* mjw_step with a launch trace: events[0] is recorded on `stream` before the step and events[i + 1]
 * right after the step's i-th kernel launch (i < nevents - 1), kernel_ids[i] names that kernel
 * (mjw_kernel_name); *nlaunch = launches traced.  The events must exist (hipEventCreate).  bench.py
 * times every kernel of the step with it on the stream they run on.  No reference counterpart (the
 * reference's event_trace, benchmark.py, times its Warp kernels the same way). */
int mjw_step_trace(const mjw_model_t* m, const mjw_data_t* d, void* stream, void** events, int nevents, int* kernel_ids,
                   int* nlaunch);
const char* mjw_kernel_name(int kernel_id);

int mjw_forward(const mjw_model_t* m, const mjw_data_t* d, void* stream);
int mjw_fwd_position(const mjw_model_t* m, const mjw_data_t* d, void* stream);
int mjw_contact_rows(const mjw_model_t* m, const mjw_data_t* d, void* stream);
int mjw_fwd_velocity(const mjw_model_t* m, const mjw_data_t* d, void* stream);
int mjw_fwd_actuation(const mjw_model_t* m, const mjw_data_t* d, void* stream);
int mjw_fwd_acceleration(const mjw_model_t* m, const mjw_data_t* d, void* stream);
int mjw_solve(const mjw_model_t* m, const mjw_data_t* d, void* stream);
int mjw_euler(const mjw_model_t* m, const mjw_data_t* d, void* stream);
/* One stage of every world, its inputs the Data fields the earlier stages wrote and its outputs written
 * back (dense-path models; round 6).  `stage` (MJW_STAGE_*) names the reference function it replaces:
 *   1 kinematics          smooth.py:357-415   (qpos, mocap -> body / joint / geom / site frames)
 *   2 com_pos             smooth.py:601-632   (frames -> subtree_com, cinert, cdof)
 *   3 camlight            smooth.py:635-803   (frames, subtree_com -> camera / light frames)
 *   4 tendon              smooth.py:3627-3700 (qpos, frames -> ten_length, ten_J)
 *   5 crb                 smooth.py:888-912   (cinert, cdof -> crb, qM incl. armature)
 *   6 make_constraint     constraint.py:2718-2779 (contacts in d.contact + frames -> efc rows)
 *   7 transmission        smooth.py:2605-2700 (actuator_length / moment; not for BODY transmissions)
 *   8 com_vel             smooth.py:1935-2038 (+ actuator_velocity, forward.py:540-562)
 *   9 passive             passive.py:535-563
 *  10 rne                 smooth.py:1276-1300 (flg_acc = False; + tendon_bias, :1878-1932) */
enum { MJW_STAGE_KINEMATICS = 1, MJW_STAGE_COM_POS = 2, MJW_STAGE_CAMLIGHT = 3, MJW_STAGE_TENDON = 4, MJW_STAGE_CRB = 5,
       MJW_STAGE_MAKE_CONSTRAINT = 6, MJW_STAGE_TRANSMISSION = 7, MJW_STAGE_COM_VEL = 8, MJW_STAGE_PASSIVE = 9, MJW_STAGE_RNE = 10 };
int mjw_stage(const mjw_model_t* m, const mjw_data_t* d, int stage, void* stream);
/* sensors of the stages in `stages` (bit 0: sensor_pos, sensor.py:761; bit 1: sensor_vel, :1377;
 * bit 2: sensor_acc with rne_postconstraint, :2447) from the Data of the current step; mjw_step /
 * mjw_forward run all three themselves, the stage entry points above run none */
int mjw_sensor(const mjw_model_t* m, const mjw_data_t* d, int stages, void* stream);
/* Runge-Kutta 4 (forward.py:457-491 rungekutta4): expects `forward` to have run on the current state
 * (mjw_step does this itself for RK4 models); runs three more forward passes and advances the state.
 * The t0 copies and the weighted sums live in the Data workspace fields qpos_t0 ... act_dot_rk. */
int mjw_rungekutta4(const mjw_model_t* m, const mjw_data_t* d, void* stream);
/* one RK4 bookkeeping op, for hosts that run `forward` themselves between them (Python callbacks):
 * op 0 = save t0 and accumulate B[0] (scale), 1 = _rk_perturb_state (forward.py:357-399),
 * 2 = _rk_accumulate (:402-454), 3 = restore t0 and _advance (:484-491, :213-274) */
int mjw_rk4_op(const mjw_model_t* m, const mjw_data_t* d, int op, float scale, void* stream);
/* per-step control noise (Ornstein-Uhlenbeck + Halton) of the reference benchmark;
 * center: device float[nu] or NULL; world ids are d->world_offset + local id */
/* Device self-checks of the wave primitives of the dense path (no reference counterpart):
 * which = 0: in = n x 64 floats, out[w] = sum of chunk w, out[n + 64w + l] = in[64w + l] + in[64w + (l^32)];
 * which = 1: in = n row-major 32x32 SPD matrices, out = their inverses (Cholesky + MFMA X^T X). */
int mjw_selftest(int which, const float* in, float* out, int n, void* stream);
/* Device replay of the reference's collision known-answer tests (csrc/mjw_kat.hip, tests/test_gpu_golden.py):
 * which = 0: ccd() as collision_gjk_test.py:34-265 `_geom_dist` calls it (+ box multi-contact), one record of
 *            48 floats per case in `in`, aux = {max ccd_iterations, mesh vertices...}, 8 floats out per case;
 * which = 1: sphere / capsule / box / cylinder vs triangle (collision_primitive_core_test.py), 32 floats in,
 *            16 out per case, aux unused. */
int mjw_kat(int which, const float* in, const float* aux, float* out, int n, void* stream);

/* qfrc_actuator from the Data's actuator_force and moment rows (forward.py:899-927), for hosts that run
 * the act_dyn / act_gain / act_bias callbacks (forward.py:876-881) between mjw_fwd_actuation and the
 * moment map; dense path only */
int mjw_actuator_map(const mjw_model_t* m, const mjw_data_t* d, void* stream);

int mjw_ctrl_noise(const mjw_model_t* m, const mjw_data_t* d, const float* center, int step, float std, float rate,
                   void* stream);

/* The collision sub-stages (mujoco_warp/__init__.py:33-35) over the reference's CollisionContext arrays
 * (collision_core.py:345-365), each `naconmax` long: collision_pair (2 ints, type-ordered geoms),
 * collision_pairid (2 ints: explicit <pair> id or -1 / -2 excluded, collision-sensor id or -1),
 * collision_worldid.  Both read the geom frames d.geom_xpos / d.geom_xmat of the position stage.
 * mjw_nxn_broadphase replaces nxn_broadphase (collision_driver.py:697-731): survivors of
 * opt_broadphase_filter over the filtered NXN list, counted in d.ncollision (which the caller zeroes), slots
 * past naconmax dropped.  mjw_sap_broadphase replaces sap_broadphase (:554-643): bounding spheres projected on
 * the reference's fixed direction and sorted per world (ngeom <= 4096), the sweep's candidates (_sap_range
 * :421-441) that are NXN pairs through the same filter, appended the same way (round 6; ABI 34).
 * mjw_primitive_narrowphase replaces primitive_narrowphase (collision_primitive.py:1461-1549): contacts of
 * the candidates [0, min(ncollision, naconmax)) whose type pair (t1 <= t2) has bit 8 t1 + t2 set in
 * typemask, appended to the contact pool at d.nacon as write_contact does (collision_core.py:160-232). */
int mjw_nxn_broadphase(const mjw_model_t* m, const mjw_data_t* d, int* collision_pair, int* collision_pairid, int* collision_worldid,
                       void* stream);
int mjw_sap_broadphase(const mjw_model_t* m, const mjw_data_t* d, int* collision_pair, int* collision_pairid, int* collision_worldid,
                       void* stream);
int mjw_primitive_narrowphase(const mjw_model_t* m, const mjw_data_t* d, const int* collision_pair, const int* collision_pairid,
                              const int* collision_worldid, unsigned long long typemask, void* stream);

#ifdef __cplusplus
}
#endif
#endif
