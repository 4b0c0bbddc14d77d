"""Per-field error report of the HIP path against the fp64 oracle on the C3 / C4 / C5 models (GPU box).

For franka (scene.xml), apollo (scene_flat.xml, keyframe "stand"), cloth and aloha_cloth: every smooth
stage's outputs, qM, qacc_smooth (normwise + fp64 backward error), the constraint rows (same count /
order / type; J, pos, vel, D, aref), the solve from the oracle's own rows (fp64 cost ratio, qacc
normwise) and one full step (qpos, qvel).  `norm` = max |got - want| / max |want| per world (worst
world), `elem` = the smallest elementwise rtol passing with an absolute floor of 1e-6 * scale (the
north-star rung of tests/test_gpu_parity_strict.py).  The strict model tests take their tolerances
from this report (profiles/r03_parity_models.json).
Shared by tests/test_gpu_parity_models.py (the assertions) and tools/parity_models.py (the JSON
report, usage: python tools/parity_models.py [out.json] [model ...]).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
  sys.path.insert(0, ROOT)

from tests.common import franka_model, franka_states, gpu_from_state, np_, oracle_from_state  # noqa: E402

SMOOTH = {
  "fwd_position": ("xpos", "xquat", "xmat", "xipos", "ximat", "xanchor", "xaxis", "geom_xpos", "geom_xmat", "site_xpos", "site_xmat",
                   "subtree_com", "cinert", "cdof", "crb", "cam_xpos", "cam_xmat", "light_xpos", "light_xdir", "actuator_length",
                   "flexvert_xpos", "flexedge_length"),
  "fwd_velocity": ("actuator_velocity", "cvel", "cdof_dot", "qfrc_spring", "qfrc_damper", "qfrc_gravcomp", "qfrc_fluid", "qfrc_passive",
                   "qfrc_bias", "flexedge_velocity"),
  "fwd_actuation": ("actuator_force", "qfrc_actuator"),
  "fwd_acceleration": ("qfrc_smooth",),
}


def err(got, want):
  got = np.asarray(got, np.float64).reshape(len(want), -1)
  want = np.asarray(want, np.float64).reshape(len(want), -1)
  if want.size == 0:
    return None
  scale = np.abs(want).max(axis=1, keepdims=True) + 1e-30
  e = np.abs(got - want)
  return dict(norm=float((e / scale).max()), elem=float((np.maximum(e - 1e-6 * scale, 0) / np.maximum(np.abs(want), 1e-30)).max()),
              abs=float(e.max()))


def merge(a, b):
  if a is None:
    return b
  if b is None:
    return a
  return {k: max(a[k], b[k]) for k in a}


# passive_test.py:160-205 test_gravcomp's model (gravity 1 2 3, contacts off, one joint routes its
# gravcomp to the actuators)
GRAVCOMP_XML = """<mujoco><option gravity="1 2 3"><flag contact="disable"/></option><worldbody>
<body gravcomp="1"><geom type="sphere" size=".1" pos="1 0 0"/><joint name="joint0" type="hinge" axis="0 1 0" actuatorgravcomp="true"/></body>
<body gravcomp="1"><geom type="sphere" size=".1"/><joint name="joint1" type="hinge" axis="1 0 0"/><joint type="hinge" axis="0 1 0"/><joint type="hinge" axis="0 0 1"/></body>
<body gravcomp="1"><geom type="sphere" size=".1"/><joint type="hinge" axis="0 1 0"/></body>
<body gravcomp="0"><geom type="sphere" size=".1"/><joint type="hinge" axis="0 1 0"/></body>
</worldbody><actuator><motor joint="joint0"/><motor joint="joint1"/></actuator></mujoco>"""

# fluid: the inertia-box model on a chain of boxes / capsules (passive_test.py:62-96 uses one free box), and
# the ellipsoid model on every geom type it handles (passive_test.py:98-127 uses one sphere), wind on
FLUID_BOX_XML = """<mujoco><option density="1.2" viscosity="0.3" wind="0.4 -0.2 0.1"/><worldbody><geom type="plane" size="5 5 .1"/>
<body pos="0 0 1"><freejoint/><geom type="box" size=".1 .2 .15"/>
  <body pos=".2 0 0"><joint type="hinge" axis="0 1 0"/><geom type="capsule" size=".05" fromto="0 0 0 .3 0 0"/>
    <body pos=".3 0 0"><joint type="ball"/><geom type="box" size=".08 .05 .02"/></body></body></body>
<body pos="1 0 1"><joint type="slide" axis="1 0 0"/><joint type="hinge" axis="0 0 1"/><geom type="sphere" size=".1"/></body>
</worldbody></mujoco>"""

FLUID_ELLIPSOID_XML = """<mujoco><option density="1.3" viscosity="0.07" wind="0.1 0.2 -0.05"/><worldbody><geom type="plane" size="5 5 .1"/>
<body pos="0 0 1"><freejoint/><geom type="sphere" size=".1" fluidshape="ellipsoid"/>
  <body pos=".3 0 0"><joint type="hinge" axis="0 1 0"/><geom type="capsule" size=".04 .1" fluidshape="ellipsoid" fluidcoef=".4 .3 1.2 .8 .6"/>
    <geom type="box" size=".05 .08 .02" pos="0 .1 0" fluidshape="ellipsoid"/></body></body>
<body pos="1 0 1"><freejoint/><geom type="cylinder" size=".06 .12" fluidshape="ellipsoid"/><geom type="ellipsoid" size=".1 .05 .03" pos=".1 0 0"/></body>
</worldbody></mujoco>"""


def _random_pose(mjm, nworld, seed, qvel_sd=0.5, key=None):
  rng = np.random.default_rng(seed)
  q0 = mjm.key_qpos[key] if key is not None else mjm.qpos0
  qpos = np.tile(q0, (nworld, 1)) + rng.normal(0, 0.05, (nworld, mjm.nq))
  qvel = rng.normal(0, qvel_sd, (nworld, mjm.nv))
  ctrl = rng.normal(0, 0.5, (nworld, mjm.nu))
  return qpos, qvel, ctrl


def setup(name):
  """(mjm, qpos, qvel, ctrl, njmax, nconmax, nworld) of a C3-C5 parity workload, or of a model of the
  reference's passive tests (pendula.xml, gravcomp, fluid)."""
  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  if name in ("pendula", "pendula_nograv"):
    # the reference's test_data/pendula.xml (free / ball / slide / hinge chains, limits, armature, fixed
    # tendons, jointinparent motors, gravcomp bodies with an actuatorgravcomp joint), nv = 36: the dense
    # Jacobian override (io.py:142-144 allows nv <= 60) runs it on the generic world-per-wave kernel
    mjm = mjw.load_model(os.path.join(ROOT, "models", "test_data", "pendula.xml"))
    mjm.opt.jacobian = 0
    if name == "pendula_nograv":
      mjm.opt.disableflags |= 128  # DisableBit.GRAVITY: gravcomp off, qfrc_gravcomp = 0
    return (mjm,) + _random_pose(mjm, 8, 3, key=0) + (64, 8, 8)
  if name in ("gravcomp", "gravcomp_sparse"):
    mjm = mjcf.load_model_from_string(GRAVCOMP_XML)
    mjm.opt.jacobian = 1 if name == "gravcomp_sparse" else 0
    return (mjm,) + _random_pose(mjm, 8, 4) + (16, 4, 8)
  if name in ("fluid_box", "fluid_ellipsoid"):
    mjm = mjcf.load_model_from_string(FLUID_BOX_XML if name == "fluid_box" else FLUID_ELLIPSOID_XML)
    qpos, qvel, ctrl = _random_pose(mjm, 8, 5, qvel_sd=1.0)
    return mjm, qpos, qvel, ctrl, 64, 16, 8

  if name == "franka":
    mjm = franka_model()
    # pools sized so that neither side drops rows or contacts (the device pool is global, the
    # oracle's per world): the random poses drive the hand up to 0.2 m into the floor, 18 contacts
    # (73 rows > 64: the generic LDS-solver kernel, mjw_step.hip, runs this workload)
    return (mjm,) + franka_states(mjm, 16, seed=22) + (96, 24, 16)
  if name == "franka_dense":
    # the same states without the two buried-hand worlds: every world within the register-resident
    # dense kernel's njmax <= 64 (mjw_dense.h), the path the C3 benchmark runs
    mjm = franka_model()
    q, v, c = franka_states(mjm, 16, seed=22)
    keep = np.array([w for w in range(16) if w not in (2, 6)])
    return mjm, q[keep], v[keep], c[keep], 64, 16, len(keep)
  if name == "apollo":
    mjm = mjw.load_model(os.path.join(ROOT, "models", "apptronik_apollo", "scene_flat.xml"))
    nworld = 32
    rng = np.random.default_rng(7)
    qpos = np.tile(mjm.key_qpos[0], (nworld, 1))
    qpos[:, 7:] += rng.normal(0, 0.05, (nworld, mjm.nq - 7))
    qvel = rng.normal(0, 0.2, (nworld, mjm.nv))
    ctrl = np.tile(mjm.key_ctrl[0], (nworld, 1))
    return mjm, qpos, qvel, ctrl, 64, 16, nworld
  from tests.cloth_common import aloha_model, aloha_states, cloth_model, cloth_states

  if name == "cloth":
    mjm = cloth_model()
    return (mjm,) + cloth_states(mjm, 2, seed=1) + (3000, 200, 2)
  mjm = aloha_model()
  return (mjm,) + aloha_states(mjm, 2, seed=1) + (16384, 4096, 2)


def dense_M(mjm, d, od, w):
  nv = mjm.nv
  if int(np.asarray(mjm.opt.jacobian)) == 1 or d.qM.dim() == 2:
    from tests.cloth_common import dense_qM

    return dense_qM(mjm, np_(d.qM[w])), od.qM[w].reshape(nv, nv)
  return np_(d.qM[w])[:nv, :nv], od.qM[w].reshape(nv, nv)


def rows_of(mjm, d, od, w, sparse, njmax):
  """(gpu row ids, oracle row ids, dense gpu J rows): identical order on the dense path; through the
  matched contacts on the sparse path (tests/test_cloth.py)."""
  nv = mjm.nv
  n = min(int(od.nefc[w, 0]), njmax)
  if not sparse:
    return np.arange(n), np.arange(n), np_(d.efc.J[w, :n, :nv])
  from tests.cloth_common import dense_J, gpu_contacts, oracle_contacts
  from tests.test_cloth import _match_rows

  pairs = _match_rows(d, od, w, gpu_contacts(d, w), oracle_contacts(od, w))
  g = np.array([p[0] for p in pairs], dtype=int)
  o = np.array([p[1] for p in pairs], dtype=int)
  return g, o, dense_J(d, w, n, nv)[g]


def rows_at_gpu_pos(mjm, d, od, w, g, o, njmax):
  """Errors of the GPU's efc D / aref against the reference's row formula evaluated in fp64 at the GPU's own
  pos_aref (= efc_pos - efc_margin), pos_imp and efc_vel: the row's remaining inputs (invweight, solref,
  solimp) are model / contact parameters, taken from the oracle (efc_prm).  pos_imp is pos_aref for most
  rows; for connect / weld rows it is the norm of the group's pos_aref, for elliptic friction rows the
  normal row's (the group: rows with the same type and id).  Returns ({D, aref: err}, rows covered)."""
  from oracle import orc

  g, o = np.asarray(g, int), np.asarray(o, int)
  if len(o) == 0:
    return {"D": None, "aref": None}, 0
  prm = np.asarray(od.efc_prm[w], np.float64).reshape(njmax, 9)[o]
  pa_o = (od.efc_pos[w] - od.efc_margin[w])[o]
  pa_g = (np_(d.efc.pos[w]).astype(np.float64) - np_(d.efc.margin[w]).astype(np.float64))[g]
  typ, ids = od.efc_type[w][o], od.efc_id[w][o]
  pi_g = pa_g.copy()
  keep = np.ones(len(o), bool)
  for i in np.nonzero(prm[:, 0] != pa_o)[0]:
    grp = np.nonzero((typ == typ[i]) & (ids == ids[i]))[0]
    nrm_o = float(np.linalg.norm(pa_o[grp]))
    if abs(prm[i, 0] - nrm_o) <= 1e-12 * max(1.0, abs(nrm_o)):
      pi_g[i] = float(np.linalg.norm(pa_g[grp]))
    elif abs(prm[i, 0] - pa_o[grp[0]]) <= 1e-12 * max(1.0, abs(pa_o[grp[0]])):
      pi_g[i] = pa_g[grp[0]]
    else:
      keep[i] = False
  vel_g = np_(d.efc.vel[w]).astype(np.float64)[g]
  D_ref, aref_ref = orc.efc_row_params(int(mjm.opt.disableflags), float(mjm.opt.timestep), pa_g[keep], pi_g[keep], prm[keep, 1],
                                       prm[keep, 2:4], prm[keep, 4:9], vel_g[keep])
  out = {"D": err(np_(d.efc.D[w])[g][keep][None], D_ref[None]), "aref": err(np_(d.efc.aref[w])[g][keep][None], aref_ref[None])}
  return out, int(keep.sum())


def efc_cost(J, D, aref, types_, M, qacc_smooth, qacc, fl=None, nf=0):
  """fp64 primal cost (solver.py): Gauss term + rows; equality always quadratic, friction loss
  Huber, limits / contacts quadratic while J qacc - aref < 0."""
  dq = qacc - qacc_smooth
  jar = J @ qacc - aref
  c = 0.5 * dq @ M @ dq
  for i in range(len(jar)):
    t = types_[i]
    if t == 0:
      c += 0.5 * D[i] * jar[i] ** 2
    elif t == 1:
      f = fl[i]
      rf = f / D[i] if D[i] > 0 else 0.0
      if jar[i] <= -rf:
        c += -f * (0.5 * rf + jar[i])
      elif jar[i] >= rf:
        c += -f * (0.5 * rf - jar[i])
      else:
        c += 0.5 * D[i] * jar[i] ** 2
    elif jar[i] < 0:
      c += 0.5 * D[i] * jar[i] ** 2
  return c


def report(name):
  import torch

  import mujoco_warp_amd as mjw

  mjm, qpos, qvel, ctrl, njmax, nconmax, nworld = setup(name)
  sparse = bool(mjw.put_model(mjm, device="cpu").is_sparse)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=nconmax)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=nconmax)
  out = {"nworld": nworld, "sparse": sparse, "fields": {}}
  for st, fields in SMOOTH.items():
    getattr(mjw, st)(m, d)
    getattr(od, st)()
    torch.cuda.synchronize()
    for f in fields:
      g = getattr(d, f, None)
      if g is None or g.numel() == 0:
        continue
      try:
        want = getattr(od, f)
      except AttributeError:
        continue
      e = err(np_(g).reshape(nworld, -1), want)
      if e is not None:
        out["fields"][f] = e
  nv = mjm.nv
  eM = None
  bw = 0.0
  for w in range(nworld):
    Mg, Mo = dense_M(mjm, d, od, w)
    eM = merge(eM, err(Mg[None], Mo[None]))
    r = Mo @ np_(d.qacc_smooth[w]) - od.qfrc_smooth[w]
    bw = max(bw, float(np.abs(r).max() / (np.abs(od.qfrc_smooth[w]).max() + 1e-300)))
  out["fields"]["qM"] = eM
  out["fields"]["qacc_smooth"] = err(np_(d.qacc_smooth), od.qacc_smooth)
  out["qacc_smooth_backward"] = bw
  out["force_scale"] = float(np.abs(od.qfrc_smooth).max())
  # qfrc_smooth = passive - bias + actuator: when the summands cancel (gravity compensation against the gravity
  # bias) fp32 rounding of the summands, not of the result, bounds its error
  summ = np.maximum(np.maximum(np.abs(od.qfrc_bias).max(axis=1), np.abs(od.qfrc_passive).max(axis=1)), np.abs(od.qfrc_actuator).max(axis=1))
  out["cancel_scale"] = max(1.0, float((summ / (np.abs(od.qfrc_smooth).max(axis=1) + 1e-300)).max()))
  # the same quantities from the fp32 build of the oracle (the reference's arithmetic type, sequential
  # order): what fp32 evaluation of the formulas achieves on this state, against the same fp64 oracle
  _, o32 = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=nconmax, real_bits=32)
  o32.forward()
  bw32 = 0.0
  for w in range(nworld):
    Mo = dense_M(mjm, d, od, w)[1]
    r32 = Mo @ np.asarray(o32.qacc_smooth[w], np.float64) - od.qfrc_smooth[w]
    bw32 = max(bw32, float(np.abs(r32).max() / (np.abs(od.qfrc_smooth[w]).max() + 1e-300)))
  out["fp32_oracle"] = {"qfrc_smooth": err(np.asarray(o32.qfrc_smooth, np.float64), od.qfrc_smooth), "qacc_smooth_backward": bw32,
                        "qacc_smooth": err(np.asarray(o32.qacc_smooth, np.float64), od.qacc_smooth)}
  # qacc_smooth = M^-1 qfrc_smooth: its forward error carries cond(M) times the (checked) residual
  out["cond_M"] = max(float(np.linalg.cond(od.qM[w].reshape(nv, nv))) for w in range(nworld))
  # rows
  counts_equal = all(int(d.nefc[w]) == int(od.nefc[w, 0]) for w in range(nworld))
  out["rows_counts_equal"] = bool(counts_equal)
  out["rows_count_mismatch"] = [
    dict(world=w, gpu=[int(d.nefc[w]), int(d.ne[w]), int(d.nf[w]), int(d.nl[w])], oracle=[int(od.nefc[w, 0]), int(od.ne[w, 0]), int(od.nf[w, 0]), int(od.nl[w, 0])],
         ncon_oracle=int(od.ncon[w, 0]), dist_oracle=[float(x) for x in od.con_dist[w, : int(od.ncon[w, 0])]])
    for w in range(nworld) if int(d.nefc[w]) != int(od.nefc[w, 0])
  ]
  rowerr = {}
  types_equal = True
  nrows = 0
  for w in range(nworld):
    g, o, Jg = rows_of(mjm, d, od, w, sparse, njmax)
    nrows += len(o)
    Jo = od.efc_J[w].reshape(njmax, nv)[o]
    types_equal &= bool(np.array_equal(d.efc.type[w].cpu().numpy()[g], od.efc_type[w][o]))
    if len(o) == 0:
      continue
    rowerr["J"] = merge(rowerr.get("J"), err(Jg.reshape(1, -1), Jo.reshape(1, -1)))
    for f in ("pos", "vel", "D", "aref"):
      rowerr[f] = merge(rowerr.get(f), err(np_(getattr(d.efc, f)[w])[g][None], getattr(od, "efc_" + f)[w][o][None]))
    rowerr["pos_abs"] = max(rowerr.get("pos_abs", 0.0), float(np.abs(np_(d.efc.pos[w])[g] - od.efc_pos[w][o]).max()))
    # D / aref as functions of the GPU's own row positions (constraint.py:52-121 in fp64, the oracle's
    # orc_kat_efc_row), with the row's other inputs (invweight, solref, solimp) from the oracle
    e_at, n_at = rows_at_gpu_pos(mjm, d, od, w, g, o, njmax)
    for f in ("D", "aref"):
      rowerr[f + "_at_gpu_pos"] = merge(rowerr.get(f + "_at_gpu_pos"), e_at[f])
    rowerr["rows_at_gpu_pos"] = rowerr.get("rows_at_gpu_pos", 0) + n_at
  out["rows"] = rowerr
  out["rows_types_equal"] = types_equal
  out["rows_total"] = nrows
  # solve from the same smooth state: the oracle's rows define the fp64 cost
  mjw.solve(m, d)
  od.solve()
  torch.cuda.synchronize()
  ratio, qn = 0.0, 0.0
  for w in range(nworld):
    n = min(int(od.nefc[w, 0]), njmax)
    Mg, Mo = dense_M(mjm, d, od, w)
    J = od.efc_J[w].reshape(njmax, nv)[:n]
    args = (J, od.efc_D[w, :n], od.efc_aref[w, :n], od.efc_type[w, :n], Mo, od.qacc_smooth[w])
    c_or = efc_cost(*args, od.qacc[w], fl=od.efc_frictionloss[w, :n])
    c_gpu = efc_cost(*args, np_(d.qacc[w]), fl=od.efc_frictionloss[w, :n])
    c_0 = efc_cost(*args, od.qacc_smooth[w], fl=od.efc_frictionloss[w, :n])
    # relative excess over the oracle optimum (no rows: qacc = qacc_smooth, nothing to compare)
    if n:
      ratio = max(ratio, (c_gpu - c_or) / max(abs(c_or), 1e-300))
    qn = max(qn, float(np.abs(np_(d.qacc[w]) - od.qacc[w]).max() / (np.abs(od.qacc[w]).max() + 1e-300)))
    _ = c_0
  out["solve_cost_excess"] = ratio
  out["solve_qacc_norm"] = qn
  out["solver_niter_gpu"] = np_(d.solver_niter).ravel().tolist()
  out["solver_niter_oracle"] = np.asarray(od.solver_niter).ravel().tolist()
  # one full step from the initial state
  m2, d2 = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=nconmax)
  om2, od2 = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=nconmax)
  mjw.step(m2, d2)
  od2.step()
  torch.cuda.synchronize()
  for f in ("qpos", "qvel", "qacc"):
    out["step_" + f] = err(np_(getattr(d2, f)), getattr(od2, f))
  if mjm.nsensordata:
    out["step_sensordata"] = err(np_(d2.sensordata), od2.sensordata)
  return out
