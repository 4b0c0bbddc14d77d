"""The reference's stage and support functions (mujoco_warp/__init__.py:26-112) on this build
(mujoco_warp_amd/stages.py).

CPU: every name the reference exports exists here, except the subsystems DESIGN.md §7 leaves out.
GPU: the stage functions, chained, reproduce the fused step's fields and each reads the earlier stages'
Data fields (an edit there is what it sees); the support functions agree with what the HIP
kernels computed from the same state -- jac' qvel with the body's cvel, xfrc_accumulate with the xfrc part
of qfrc_smooth, solve_m with qacc_smooth (dense humanoid and sparse cloth), subtree_vel's root entries with
the directly summed momenta, and energy_pos + energy_vel conserved along a frictionless pendulum rollout.
"""

import re

import numpy as np
import pytest

from tests.common import HUMANOID, np_, random_states

# out of scope: rendering / rays, inverse dynamics, islands, BVH and SDF collision; the
# broad- / narrowphase sub-stages (tests/test_collision_stages.py), the set_const family,
# set_length_range and deriv_smooth_vel are implemented (stages.py)
OUT_OF_SCOPE = {
  "RenderContext", "create_render_context", "get_depth", "get_rgb", "get_segmentation", "render", "ray", "rays", "refit_bvh",
  "inverse", "island", "sdf_narrowphase",
}


def test_reference_api_names_exist():
  import mujoco_warp_amd as mjw

  src = open("/root/reference/mujoco_warp/__init__.py").read() if __import__("os").path.exists("/root/reference") else None
  if src is None:
    pytest.skip("reference tree not present (GPU box)")
  names = {b for _, b in re.findall(r"import (\w+) as (\w+)", src)}
  missing = sorted(n for n in names - OUT_OF_SCOPE if not hasattr(mjw, n))
  assert not missing, missing


def _humanoid(nworld, seed=3):
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model(HUMANOID)
  qpos, qvel, ctrl = random_states(mjm, nworld, seed=seed, qpos_noise=0.1, qvel_noise=0.5)
  m = mjw.put_model(mjm, device="cuda")
  d = mjw.make_data(mjm, nworld=nworld, nconmax=24, njmax=64, device="cuda", m=m)
  d.qpos[:] = torch.as_tensor(qpos, dtype=torch.float32, device="cuda")
  d.qvel[:] = torch.as_tensor(qvel, dtype=torch.float32, device="cuda")
  d.ctrl[:] = torch.as_tensor(ctrl, dtype=torch.float32, device="cuda")
  return mjm, m, d


@pytest.mark.gpu
def test_gpu_stage_aliases_match_forward():
  import torch

  import mujoco_warp_amd as mjw

  _, m, d = _humanoid(16)
  _, m2, d2 = _humanoid(16)
  mjw.forward(m, d)
  for f in (mjw.kinematics, mjw.com_pos, mjw.camlight, mjw.crb, mjw.tendon, mjw.collision, mjw.make_constraint, mjw.transmission,
            mjw.com_vel, mjw.passive, mjw.rne, mjw.fwd_actuation, mjw.factor_m, mjw.solve, mjw.rne_postconstraint):
    f(m2, d2)
  torch.cuda.synchronize()
  for name in ("xpos", "xquat", "subtree_com", "cinert", "cdof", "qM", "qLD", "actuator_length", "cvel", "cdof_dot", "qfrc_bias",
               "qfrc_passive", "qacc_smooth", "qacc", "cacc", "cfrc_int"):
    np.testing.assert_allclose(np_(getattr(d2, name)), np_(getattr(d, name)), rtol=1e-5, atol=1e-5, err_msg=name)


@pytest.mark.gpu
def test_gpu_stages_read_the_data_fields():
  """Each stage function reads the Data fields the earlier stages wrote and writes only its own outputs
  (smooth.py:357-415 kinematics, 601-632 com_pos, 888-912 crb, 1276-1300 rne; constraint.py:2718-2779):
  kinematics leaves qM alone; com_pos takes an edited xipos; crb takes an edited cinert; rne with cvel and
  cdof_dot zeroed gives the bias of the same state at rest; make_constraint rebuilds forward's rows."""
  import torch

  import mujoco_warp_amd as mjw

  mjm, m, d = _humanoid(8)
  mjw.forward(m, d)
  torch.cuda.synchronize()
  base = {k: getattr(d, k).clone() for k in ("xpos", "xipos", "subtree_com", "cinert", "qM", "qfrc_bias", "cvel", "cdof_dot")}
  efc = (d.nefc.clone(), d.efc.J.clone(), d.efc.D.clone(), d.efc.aref.clone(), d.efc.type.clone())
  # kinematics: frames from qpos, nothing downstream touched
  d.qM.fill_(7.0)
  mjw.kinematics(m, d)
  torch.cuda.synchronize()
  assert torch.all(d.qM == 7.0)
  np.testing.assert_allclose(np_(d.xpos), np_(base["xpos"]), rtol=0, atol=1e-6)
  d.qM.copy_(base["qM"])
  # com_pos: an edited xipos moves subtree_com as the mass-weighted subtree mean says
  nb = mjm.nbody
  delta = torch.zeros_like(d.xipos)
  delta[:, 1:, 0] = 0.05  # every body shifted by 5 cm in x
  d.xipos.add_(delta)
  mjw.com_pos(m, d)
  torch.cuda.synchronize()
  xipos = np_(d.xipos)
  mass = np.asarray(mjm.body_mass, np.float64)
  for b in range(1, nb):
    sub = [j for j in range(b, nb) if _ancestor(mjm, j, b)]
    want = (mass[sub, None] * xipos[:, sub, :]).sum(axis=1) / mass[sub].sum()
    np.testing.assert_allclose(np_(d.subtree_com)[:, b], want, rtol=0, atol=2e-6)
  assert np.abs(np_(d.subtree_com)[:, 1, 0] - np_(base["subtree_com"])[:, 1, 0] - 0.05).max() < 1e-5
  # crb: twice the inertias give twice the mass matrix outside the armature diagonal
  d.xipos.copy_(base["xipos"])
  mjw.com_pos(m, d)
  d.cinert.mul_(2.0)
  mjw.crb(m, d)
  torch.cuda.synchronize()
  arm = np.diag(np.asarray(mjm.dof_armature, np.float64))
  nv = mjm.nv
  q0 = np_(base["qM"])[:, :nv, :nv]
  np.testing.assert_allclose(np_(d.qM)[:, :nv, :nv], 2.0 * (q0 - arm) + arm, rtol=1e-5, atol=1e-5)
  d.cinert.copy_(base["cinert"])
  mjw.crb(m, d)
  # rne at rest: cvel = cdof_dot = 0 leaves gravity only, as forward on the same state with qvel = 0
  d.cvel.zero_()
  d.cdof_dot.zero_()
  mjw.rne(m, d)
  torch.cuda.synchronize()
  _, m2, d2 = _humanoid(8)
  d2.qvel.zero_()
  mjw.forward(m2, d2)
  torch.cuda.synchronize()
  np.testing.assert_allclose(np_(d.qfrc_bias), np_(d2.qfrc_bias), rtol=1e-5, atol=1e-4)
  # com_vel restores cvel / cdof_dot from qvel; make_constraint rebuilds forward's rows from d.contact
  mjw.com_vel(m, d)
  mjw.make_constraint(m, d)
  torch.cuda.synchronize()
  np.testing.assert_allclose(np_(d.cvel), np_(base["cvel"]), rtol=1e-5, atol=1e-5)
  np.testing.assert_allclose(np_(d.cdof_dot), np_(base["cdof_dot"]), rtol=1e-5, atol=1e-5)
  assert torch.equal(d.nefc, efc[0])
  for w in range(8):
    n = int(d.nefc[w])
    assert torch.equal(d.efc.type[w, :n], efc[4][w, :n])
    np.testing.assert_allclose(np_(d.efc.J[w, :n]), np_(efc[1][w, :n]), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(np_(d.efc.D[w, :n]), np_(efc[2][w, :n]), rtol=1e-5)
    np.testing.assert_allclose(np_(d.efc.aref[w, :n]), np_(efc[3][w, :n]), rtol=1e-5, atol=1e-5)


def _ancestor(mjm, j, b):
  while j > b:
    j = int(mjm.body_parentid[j])
  return j == b


@pytest.mark.gpu
def test_gpu_jac_times_qvel_is_body_velocity():
  import torch

  import mujoco_warp_amd as mjw

  mjm, m, d = _humanoid(8)
  mjw.forward(m, d)
  nw, nv, nb = 8, mjm.nv, mjm.nbody
  rng = np.random.default_rng(0)
  body = torch.as_tensor(rng.integers(1, nb, nw), device="cuda")
  point = d.xipos.reshape(nw, nb, 3)[torch.arange(nw, device="cuda"), body] + 0.1
  jacp = torch.zeros(nw, 3, nv, device="cuda")
  jacr = torch.zeros(nw, 3, nv, device="cuda")
  mjw.jac(m, d, jacp, jacr, point, body)
  v = torch.einsum("wkn,wn->wk", jacp, d.qvel)
  w = torch.einsum("wkn,wn->wk", jacr, d.qvel)
  cvel = d.cvel.reshape(nw, nb, 6)[torch.arange(nw, device="cuda"), body]
  root = m.body_rootid.to(torch.long)[body]
  off = point - d.subtree_com.reshape(nw, nb, 3)[torch.arange(nw, device="cuda"), root]
  np.testing.assert_allclose(np_(w), np_(cvel[:, :3]), rtol=1e-4, atol=1e-5)
  np.testing.assert_allclose(np_(v), np_(cvel[:, 3:] + torch.cross(cvel[:, :3], off, dim=-1)), rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_gpu_xfrc_accumulate_matches_qfrc_smooth():
  import torch

  import mujoco_warp_amd as mjw

  mjm, m, d = _humanoid(8, seed=4)
  rng = np.random.default_rng(1)
  d.xfrc_applied[:] = torch.as_tensor(rng.normal(0, 5.0, (8, mjm.nbody, 6)), dtype=torch.float32, device="cuda")
  d.qfrc_applied[:] = 0
  mjw.fwd_position(m, d)
  mjw.fwd_velocity(m, d)
  mjw.fwd_actuation(m, d)
  mjw.fwd_acceleration(m, d)
  q = torch.zeros_like(d.qvel)
  mjw.xfrc_accumulate(m, d, q)
  want = d.qfrc_smooth - (d.qfrc_passive - d.qfrc_bias + d.qfrc_actuator)
  assert float(want.abs().max()) > 1.0
  np.testing.assert_allclose(np_(q), np_(want), rtol=1e-3, atol=2e-3)


@pytest.mark.gpu
def test_gpu_solve_m_matches_qacc_smooth_dense_and_sparse():
  import torch

  import mujoco_warp_amd as mjw
  from tests.cloth_common import cloth_model, cloth_states

  _, m, d = _humanoid(8, seed=5)
  mjw.fwd_position(m, d)
  mjw.fwd_velocity(m, d)
  mjw.fwd_actuation(m, d)
  mjw.factor_m(m, d)
  x = torch.zeros_like(d.qvel)
  mjw.solve_m(m, d, x, d.qfrc_smooth)
  np.testing.assert_allclose(np_(x), np_(d.qacc_smooth), rtol=1e-3, atol=1e-3)

  mjm = cloth_model()
  qpos, qvel, _ = cloth_states(mjm, 2, seed=1)
  m = mjw.put_model(mjm, device="cuda")
  d = mjw.make_data(mjm, nworld=2, nconmax=400, njmax=4000, device="cuda", m=m)
  d.qpos[:] = torch.as_tensor(qpos, dtype=torch.float32, device="cuda")
  d.qvel[:] = torch.as_tensor(qvel, dtype=torch.float32, device="cuda")
  mjw.forward(m, d)
  torch.cuda.synchronize()
  x = torch.zeros_like(d.qvel)
  mjw.solve_m(m, d, x, d.qfrc_smooth)
  scale = float(d.qacc_smooth.abs().max())
  np.testing.assert_allclose(np_(x), np_(d.qacc_smooth), rtol=1e-3, atol=1e-4 * scale)


@pytest.mark.gpu
def test_gpu_subtree_vel_root_momenta():
  import torch

  import mujoco_warp_amd as mjw

  mjm, m, d = _humanoid(4, seed=6)
  mjw.forward(m, d)
  linvel, angmom = mjw.subtree_vel(m, d)
  nb = mjm.nbody
  mass = np.asarray(mjm.body_mass)
  xipos, ximat = np_(d.xipos).reshape(4, nb, 3), np_(d.ximat).reshape(4, nb, 3, 3)
  cvel, sc = np_(d.cvel).reshape(4, nb, 6), np_(d.subtree_com).reshape(4, nb, 3)
  root = np.asarray(mjm.body_rootid)
  for w in range(4):
    v = cvel[w, :, 3:] - np.cross(xipos[w] - sc[w, root], cvel[w, :, :3])  # body COM velocities
    p = (mass[:, None] * v).sum(0)
    np.testing.assert_allclose(np_(linvel)[w, 0] * mjm.body_subtreemass[0], p, rtol=1e-4, atol=1e-4)
    spin = np.einsum("bij,bj->bi", ximat[w], np.asarray(mjm.body_inertia) * np.einsum("bji,bj->bi", ximat[w], cvel[w, :, :3]))
    L = spin.sum(0) + np.cross(xipos[w] - sc[w, 0], mass[:, None] * v).sum(0)
    np.testing.assert_allclose(np_(angmom)[w, 0], L, rtol=1e-3, atol=1e-3)


@pytest.mark.gpu
def test_gpu_energy_conserved_on_pendulum():
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model_from_string("""<mujoco><option timestep="0.0005"/><worldbody>
    <body pos="0 0 1"><joint name="h" type="hinge" axis="0 1 0" stiffness="3"/>
      <geom type="capsule" fromto="0 0 0 .4 0 0" size=".03" contype="0" conaffinity="0"/>
      <body pos=".4 0 0"><joint type="ball" stiffness="1"/><geom type="sphere" size=".05" pos=".1 0 0" contype="0" conaffinity="0"/></body>
    </body></worldbody></mujoco>""")
  m = mjw.put_model(mjm, device="cuda")
  d = mjw.make_data(mjm, nworld=2, device="cuda", m=m)
  d.qvel[:] = torch.as_tensor(np.random.default_rng(2).normal(0, 1.0, (2, mjm.nv)), dtype=torch.float32, device="cuda")

  def energy():
    mjw.forward(m, d)
    mjw.energy_pos(m, d)
    mjw.energy_vel(m, d)
    torch.cuda.synchronize()
    return np_(d.energy).reshape(2, 2).sum(1)

  e0 = energy()
  for _ in range(200):
    mjw.step(m, d)
  e1 = energy()
  assert np.all(np.abs(e1 - e0) <= 1e-2 * np.abs(e0) + 1e-3), (e0, e1)


@pytest.mark.gpu
def test_gpu_energy_flag_fills_d_energy():
  """opt.enableflags ENERGY: step fills d.energy like energy_pos / energy_vel on the pre-step state
  (forward.py:975-991); without the flag the step leaves it zero."""
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import types

  mjm, m, d = _humanoid(4, seed=8)
  _, m2, d2 = _humanoid(4, seed=8)
  m.opt.enableflags |= types.EnableBit.ENERGY
  mjw.step(m, d)
  mjw.forward(m2, d2)
  mjw.energy_pos(m2, d2)
  mjw.energy_vel(m2, d2)
  torch.cuda.synchronize()
  assert float(np.abs(np_(d.energy)).max()) > 0
  np.testing.assert_allclose(np_(d.energy), np_(d2.energy), rtol=1e-5, atol=1e-5)
  _, m3, d3 = _humanoid(4, seed=8)
  mjw.step(m3, d3)
  torch.cuda.synchronize()
  assert float(np.abs(np_(d3.energy)).max()) == 0.0


def test_set_const_fixed_subtreemass():
  """set_const_fixed (io.py:2197-2219) on the CPU tensors: the compiler's body_subtreemass, and a per-world
  batched body_mass giving per-world subtree masses."""
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model(HUMANOID)
  m = mjw.put_model(mjm, device="cpu")
  d = mjw.make_data(mjm, nworld=3, device="cpu", m=m)
  mjw.set_const_fixed(m, d)
  np.testing.assert_allclose(m.body_subtreemass.numpy()[0], mjm.body_subtreemass, rtol=1e-6)
  m.body_mass = m.body_mass.repeat(3, 1) * torch.tensor([[1.0], [2.0], [0.5]])
  mjw.set_const_fixed(m, d)
  assert m.body_subtreemass.shape == (3, mjm.nbody)
  np.testing.assert_allclose(m.body_subtreemass.numpy()[1], 2.0 * mjm.body_subtreemass, rtol=1e-6)


def test_energy_pos_reads_batched_springs_per_world():
  """energy_pos (sensor.py:2854-2890) on CPU tensors with per-world (batched *) joint stiffness, qpos_spring
  and tendon spring fields: each world's potential is its own 0.5 k dif^2, including a world whose only
  non-zero stiffness is on a joint that world 0 leaves at zero."""
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model_from_string("""<mujoco><option gravity="0 0 0"/><worldbody>
  <body><joint name="a" type="hinge"/><geom size=".1"/><body pos="1 0 0"><joint name="b" type="slide"/><geom size=".1"/></body></body>
  <body pos="0 2 0"><joint type="ball"/><geom size=".1"/></body></worldbody>
  <tendon><fixed stiffness="1" springlength="0 .1"><joint joint="a" coef="1"/><joint joint="b" coef="2"/></fixed></tendon></mujoco>""")
  m = mjw.put_model(mjm, device="cpu")
  d = mjw.make_data(mjm, nworld=3, device="cpu", m=m)
  rng = np.random.default_rng(0)
  d.qpos[:, :2] = torch.as_tensor(rng.normal(0, 0.5, (3, 2)), dtype=torch.float32)
  d.qpos[:, 2:] = torch.nn.functional.normalize(torch.as_tensor(rng.normal(size=(3, 4)), dtype=torch.float32), dim=-1)
  m.jnt_stiffness = torch.tensor([[2.0, 0.0, 0.0], [0.0, 3.0, 0.0], [1.0, 1.0, 4.0]])
  m.qpos_spring = m.qpos_spring.repeat(3, 1)
  m.qpos_spring[1, 1] = 0.25
  m.tendon_stiffness = torch.tensor([[1.0], [0.0], [5.0]])
  m.tendon_lengthspring = torch.tensor([[[0.0, 0.1]], [[0.0, 0.1]], [[-1.0, -0.5]]])
  L = (d.qpos[:, 0] + 2 * d.qpos[:, 1]).double()
  d.ten_length[:] = L.float().reshape(3, 1)
  mjw.energy_pos(m, d)
  q = d.qpos.double()
  from mujoco_warp_amd.stages import _quat_sub

  ball = _quat_sub(q[:, 2:6], torch.tensor([[1.0, 0, 0, 0]], dtype=torch.float64).expand(3, 4))
  k, qs = m.jnt_stiffness.double(), m.qpos_spring.double()
  want = 0.5 * (k[:, 0] * (q[:, 0] - qs[:, 0]) ** 2 + k[:, 1] * (q[:, 1] - qs[:, 1]) ** 2 + k[:, 2] * (ball * ball).sum(-1))
  lo, hi = m.tendon_lengthspring[:, 0, 0].double(), m.tendon_lengthspring[:, 0, 1].double()
  disp = torch.where(L > hi, hi - L, torch.where(L < lo, lo - L, torch.zeros_like(L)))
  want += 0.5 * m.tendon_stiffness[:, 0].double() * disp * disp
  np.testing.assert_allclose(d.energy[:, 0].numpy(), want.numpy(), rtol=1e-5)
  assert float(d.energy[1, 0]) > 0  # world 1: stiffness only on the slide, with its own spring reference


@pytest.mark.gpu
def test_gpu_set_const_fixed_per_world_mass():
  """Scaling every body mass of world 1 by 2 (batched body_mass + set_const_fixed) leaves its subtree COMs
  equal to world 0's and doubles its composite inertia."""
  import torch

  import mujoco_warp_amd as mjw

  mjm, m, d = _humanoid(2, seed=9)
  d.qpos[1] = d.qpos[0]
  d.qvel[1] = d.qvel[0]
  m.body_mass = m.body_mass.repeat(2, 1) * torch.tensor([[1.0], [2.0]], device="cuda")
  m.body_inertia = m.body_inertia.repeat(2, 1, 1) * torch.tensor([1.0, 2.0], device="cuda").reshape(2, 1, 1)
  mjw.set_const_fixed(m, d)
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()
  sc = np_(d.subtree_com)
  np.testing.assert_allclose(sc[1], sc[0], rtol=1e-5, atol=1e-6)
  crb = np_(d.crb)
  np.testing.assert_allclose(crb[1], 2.0 * crb[0], rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["humanoid", "franka", "tendon", "humanoid_sparse", "tendon_sparse"])
def test_gpu_set_const_0_reproduces_put_model(model):
  """set_const_0 on the device (qpos0 position stage, M^-1 in fp64 from the fp32 qM) reproduces the
  constants put_model took from the compiler (mjcf.py, the same definitions in fp64 on the host);
  `_sparse`: the same models on the sparse path (ancestor-row qM expanded first)."""
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf
  from tests.common import franka_model

  if model.startswith("humanoid"):
    mjm = mjcf.load_model(HUMANOID)
  elif model == "franka":
    mjm = franka_model()
  else:
    mjm = mjcf.load_model_from_string("""<mujoco><worldbody><body><joint name="a" axis="0 1 0"/><geom size=".1" pos=".2 0 0"/>
      <body pos=".4 0 0"><joint name="b" axis="0 1 0"/><geom size=".1" pos=".2 0 0"/></body></body></worldbody>
      <tendon><fixed name="t"><joint joint="a" coef="1"/><joint joint="b" coef="-.5"/></fixed></tendon>
      <actuator><motor tendon="t" gear="2"/><motor joint="b"/></actuator></mujoco>""")
  if model.endswith("_sparse"):
    mjw.override_model(mjm, ["opt.jacobian=sparse"])
  m = mjw.put_model(mjm, device="cuda")
  assert m.is_sparse == model.endswith("_sparse")
  d = mjw.make_data(mjm, nworld=2, device="cuda", m=m)
  fields = ["dof_invweight0", "body_invweight0", "actuator_acc0"]
  fields += ["cam_pos0", "cam_poscom0", "cam_mat0"] if mjm.ncam else []
  fields += ["light_pos0", "light_poscom0", "light_dir0"] if mjm.nlight else []
  want = {f: np_(getattr(m, f))[0] for f in fields}
  want_mi = float(np_(m.stat.meaninertia).reshape(-1)[0])
  q = d.qpos.clone()
  mjw.forward(m, d)
  before = {k: getattr(d, k).clone() for k in ("nacon", "nefc")}
  J0 = d.efc.J.clone()
  len0 = np.asarray(getattr(mjm, "tendon_length0", np.zeros(0)), dtype=np.float64)
  mjw.set_const_0(m, d)
  torch.cuda.synchronize()
  assert torch.equal(d.qpos, q)
  # the contact pool and the constraint rows are the forward's, not the qpos0 position stage's
  for k, v in before.items():
    assert torch.equal(getattr(d, k), v), k
  assert torch.equal(d.efc.J, J0)
  if len0.size:  # io.py:2263: tendon_length0 = ten_length at qpos0, per world
    np.testing.assert_allclose(np_(m.tendon_length0).reshape(2, -1), np.tile(len0, (2, 1)), rtol=1e-5, atol=1e-6)
  np.testing.assert_allclose(np_(m.stat.meaninertia), want_mi, rtol=1e-5)
  for f, w in want.items():
    got = np_(getattr(m, f))
    assert got.shape[0] == 2
    np.testing.assert_allclose(got[1].reshape(w.shape), w, rtol=2e-4, atol=2e-6, err_msg=f)
