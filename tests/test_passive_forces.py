"""Gravity compensation (passive.py:246-272, forward.py:806-833) and the fluid model (passive.py:276-533).

The reference's passive tests (passive_test.py) compare with MuJoCo C at run time, so the oracle
restatement is pinned here by physics with closed forms:
  * gravcomp = 1 on every body cancels gravity exactly: a chain at rest stays at rest; gravcomp = g
    scales the gravity torque by (1 - g); an actuatorgravcomp joint moves its share from qfrc_passive
    to qfrc_actuator (and under the joint's actuator force range);
  * the ellipsoid fluid model of a sphere gives Stokes' drags (6 pi mu r v, 8 pi mu r^3 w) for
    viscosity alone and the blunt-body drag 1/2 rho (0.5 pi r^2) ... for density alone; the inertia-box
    model of a box recovers the box's edges, so its drags are 3 pi mu (mean edge) v and
    1/2 rho (face area) |v| v; wind w on a body at rest equals the body moving at -w;
  * massless bodies feel no fluid force (passive_test.py:129-155), and the compiler's added-mass
    coefficients of a sphere are V / 2 (kappa = 2/3 on every axis).
`-m gpu` tests compare the HIP path with the oracle on the same models (tests/test_gpu_parity_models.py
runs the strict per-field report on pendula.xml, the gravcomp test model on the dense and sparse paths,
and two fluid models).
"""

import math

import numpy as np
import pytest

from tests.common import gpu_from_state, np_, oracle_from_state


def _load(xml):
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(xml)


def _forward(mjm, qpos=None, qvel=None, ctrl=None, nworld=1):
  qpos = np.tile(mjm.qpos0, (nworld, 1)) if qpos is None else np.atleast_2d(qpos)
  qvel = np.zeros((nworld, mjm.nv)) if qvel is None else np.atleast_2d(qvel)
  ctrl = np.zeros((nworld, mjm.nu)) if ctrl is None else np.atleast_2d(ctrl)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=16, nconmax=8)
  od.forward()
  return od


CHAIN = """<mujoco><option gravity="{g}"><flag contact="disable"/></option><worldbody>
<body pos="0 0 1" gravcomp="{gc}"><joint type="hinge" axis="0 1 0"/><geom type="capsule" fromto="0 0 0 .4 0 .1" size=".05"/>
  <body pos=".4 0 .1" gravcomp="{gc}"><joint type="ball"/><geom type="box" size=".1 .05 .03" pos=".1 0 0"/>
    <body pos=".2 0 0" gravcomp="{gc}"><joint type="slide" axis="1 0 1"/><geom type="sphere" size=".07"/></body></body></body>
<body pos="1 1 1" gravcomp="{gc}"><freejoint/><geom type="box" size=".1 .2 .3"/></body>
</worldbody></mujoco>"""


def test_ngravcomp_counts_bodies():
  """io_test.py:1491-1518: bodies with gravcomp > 0."""
  import mujoco_warp_amd as mjw

  mjm = _load("""<mujoco><worldbody><body name="body1" gravcomp="1"><freejoint/><geom size=".1"/></body>
  <body name="body2" pos="1 0 0" gravcomp="0"><freejoint/><geom size=".1"/></body>
  <body name="body3" pos="2 0 0" gravcomp="1"><freejoint/><geom size=".1"/></body></worldbody></mujoco>""")
  assert mjm.ngravcomp == 2
  m = mjw.put_model(mjm, device="cpu")
  assert m.ngravcomp == 2 and not m.has_fluid


def test_oracle_full_gravcomp_holds_still():
  mjm = _load(CHAIN.format(g="0.3 -0.2 -9.81", gc=1))
  od = _forward(mjm)
  np.testing.assert_allclose(od.qfrc_gravcomp, od.qfrc_bias, rtol=1e-12, atol=1e-12)
  np.testing.assert_allclose(od.qacc, 0.0, atol=1e-12)
  for _ in range(50):
    od.step()
  np.testing.assert_allclose(od.qpos, np.tile(mjm.qpos0, (1, 1)), atol=1e-12)


def test_oracle_partial_gravcomp_scales_gravity():
  """A resting chain: the gravity torque (qfrc_bias at qvel = 0) is scaled by (1 - gravcomp)."""
  g = "0.3 -0.2 -9.81"
  rng = np.random.default_rng(0)
  m0 = _load(CHAIN.format(g=g, gc=0))
  qpos = m0.qpos0 + rng.normal(0, 0.2, m0.nq)
  base = _forward(_load(CHAIN.format(g=g, gc=0)), qpos)
  half = _forward(_load(CHAIN.format(g=g, gc=0.25)), qpos)
  np.testing.assert_allclose(half.qfrc_gravcomp, 0.25 * base.qfrc_bias, rtol=1e-10, atol=1e-12)
  np.testing.assert_allclose(half.qfrc_passive - half.qfrc_bias, -0.75 * base.qfrc_bias, rtol=1e-10, atol=1e-12)


GC_XML = """<mujoco><option gravity="1 2 3"><flag contact="disable"/></option><worldbody>
<body gravcomp="1"><geom type="sphere" size=".1" pos="1 0 0"/><joint name="joint0" type="hinge" axis="0 1 0" actuatorgravcomp="true" {rng}/></body>
<body gravcomp="1"><geom type="sphere" size=".1" pos="0 1 0"/><joint name="joint1" type="hinge" axis="1 0 0"/></body>
</worldbody><actuator><motor joint="joint0"/><motor joint="joint1"/></actuator></mujoco>"""


def test_oracle_actuatorgravcomp_routes_to_actuators():
  mjm = _load(GC_XML.format(rng=""))
  od = _forward(mjm)
  gc = od.qfrc_gravcomp[0]
  # joint0: sphere of mass 4/3 pi 1e-3 * 1000 at x = 1, gravity (1, 2, 3): -(r x m g)_y = 3 m
  m = 4.0 / 3.0 * math.pi * 1e-3 * 1000
  np.testing.assert_allclose(gc[0], 3 * m, rtol=1e-12)
  # joint1: at y = 1 about x: -(r x m g)_x = -(1 * 3 m - 0) ... = -3 m
  np.testing.assert_allclose(gc[1], -3 * m, rtol=1e-12)
  np.testing.assert_allclose(od.qfrc_passive[0], [0.0, gc[1]], atol=1e-12)   # joint0's share is not passive
  np.testing.assert_allclose(od.qfrc_actuator[0], [gc[0], 0.0], atol=1e-12)  # ... but actuator force
  np.testing.assert_allclose(od.qacc, 0.0, atol=1e-10)
  # the joint's actuator force range clamps the routed gravcomp (forward.py:829-831)
  lim = _forward(_load(GC_XML.format(rng='actuatorfrcrange="-1 1"')))
  np.testing.assert_allclose(lim.qfrc_actuator[0, 0], 1.0, rtol=1e-12)
  # actuation disabled: no actuator force at all (forward.py:839-842), the share is lost
  off = _load(GC_XML.format(rng=""))
  off.opt.disableflags |= 2048
  od = _forward(off)
  np.testing.assert_allclose(od.qfrc_actuator, 0.0)
  np.testing.assert_allclose(od.qfrc_gravcomp[0, 0], 3 * m, rtol=1e-12)


@pytest.mark.parametrize("flags", [128, 32 | 64])
def test_oracle_gravcomp_off(flags):
  """Gravity disabled (passive.py:829) or springs and dampers both disabled (the early return at
  passive.py:734-740): no gravity compensation."""
  mjm = _load(GC_XML.format(rng=""))
  mjm.opt.disableflags |= flags
  od = _forward(mjm)
  np.testing.assert_allclose(od.qfrc_gravcomp, 0.0)
  np.testing.assert_allclose(od.qfrc_passive, 0.0)


SPHERE = """<mujoco><option density="{rho}" viscosity="{mu}" wind="{w}" gravity="0 0 0"/><worldbody>
<body><freejoint/><geom type="sphere" size="{r}" {shape}/></body></worldbody></mujoco>"""


def test_compiler_sphere_added_mass():
  from mujoco_warp_amd import mjcf

  mjm = _load(SPHERE.format(rho=1, mu=0, w="0 0 0", r=0.1, shape='fluidshape="ellipsoid"'))
  V = 4.0 / 3.0 * math.pi * 0.1**3
  np.testing.assert_allclose(mjm.geom_fluid[0, :6], [1, 0.5, 0.25, 1.5, 1.0, 1.0])
  np.testing.assert_allclose(mjm.geom_fluid[0, 6:9], V / 2, rtol=1e-12)
  np.testing.assert_allclose(mjm.geom_fluid[0, 9:], 0.0, atol=1e-18)
  k = [mjcf.added_mass_kappa(*np.roll([0.1, 0.3, 0.05], -i)) for i in range(3)]
  assert abs(sum(k) - 2.0) < 1e-12 and all(0 < x < 2 for x in k)
  assert np.all(_load(SPHERE.format(rho=1, mu=0, w="0 0 0", r=0.1, shape="")).geom_fluid == 0)


@pytest.mark.parametrize("shape", ['fluidshape="ellipsoid"', ""])
def test_oracle_sphere_stokes_drag(shape):
  """Viscosity alone: Stokes' drag force 6 pi mu r v and torque 8 pi mu r^3 w (ellipsoid model: the
  equivalent sphere diameter is 2/3 of the semi-axes' sum).  The inertia-box model of a sphere uses the
  box of equal inertia: edge sqrt(12/5) r."""
  mu, r = 0.07, 0.1
  mjm = _load(SPHERE.format(rho=0, mu=mu, w="0 0 0", r=r, shape=shape))
  v, w = np.array([0.3, -0.2, 0.5]), np.array([-1.0, 0.4, 2.0])
  od = _forward(mjm, qvel=np.concatenate([v, w]))
  f = od.qfrc_fluid[0]
  if shape:
    np.testing.assert_allclose(f[:3], -6 * math.pi * mu * r * v, rtol=1e-10)
    np.testing.assert_allclose(f[3:], -8 * math.pi * mu * r**3 * w, rtol=1e-10)
  else:
    diam = math.sqrt(12.0 / 5.0) * r
    np.testing.assert_allclose(f[:3], -3 * math.pi * mu * diam * v, rtol=1e-10)
    np.testing.assert_allclose(f[3:], -math.pi * mu * diam**3 * w, rtol=1e-10)
  np.testing.assert_allclose(od.qfrc_passive, od.qfrc_fluid, rtol=1e-12)


def test_oracle_sphere_blunt_drag_and_wind():
  """Density alone, translation only: drag 1/2 rho |v| v (0.5 pi r^2) (blunt drag coefficient 0.5,
  projected area = max area); wind w on a body at rest = body moving at -w."""
  rho, r = 1.3, 0.1
  v = np.array([0.4, -1.2, 0.7])
  mjm = _load(SPHERE.format(rho=rho, mu=0, w="0 0 0", r=r, shape='fluidshape="ellipsoid"'))
  f = _forward(mjm, qvel=np.concatenate([v, np.zeros(3)])).qfrc_fluid[0]
  np.testing.assert_allclose(f[:3], -rho * np.linalg.norm(v) * 0.5 * math.pi * r * r * v, rtol=1e-10)
  np.testing.assert_allclose(f[3:], 0.0, atol=1e-14)
  windy = _load(SPHERE.format(rho=rho, mu=0.05, w=" ".join(map(str, -v)), r=r, shape='fluidshape="ellipsoid"'))
  moving = _load(SPHERE.format(rho=rho, mu=0.05, w="0 0 0", r=r, shape='fluidshape="ellipsoid"'))
  np.testing.assert_allclose(_forward(windy).qfrc_fluid, _forward(moving, qvel=np.concatenate([v, np.zeros(3)])).qfrc_fluid, rtol=1e-12)


def test_oracle_inertia_box_drags():
  """The inertia-box model of a box recovers its edges (2a, 2b, 2c): viscous drag 3 pi mu (mean edge) v,
  quadratic drag 1/2 rho (face area) |v_i| v_i per axis (the box at the identity orientation)."""
  a, b, c = 0.1, 0.2, 0.3
  rho, mu = 1.1, 0.2
  xml = f"""<mujoco><option density="{rho}" viscosity="{mu}" gravity="0 0 0"/><worldbody>
  <body><freejoint/><geom type="box" size="{a} {b} {c}"/></body></worldbody></mujoco>"""
  v = np.array([0.5, -0.3, 0.8])
  f = _forward(_load(xml), qvel=np.concatenate([v, np.zeros(3)])).qfrc_fluid[0]
  e = 2 * np.array([a, b, c])
  want = -3 * math.pi * mu * e.mean() * v - 0.5 * rho * np.array([e[1] * e[2], e[0] * e[2], e[0] * e[1]]) * np.abs(v) * v
  np.testing.assert_allclose(f[:3], want, rtol=1e-10)
  np.testing.assert_allclose(f[3:], 0.0, atol=1e-14)


def test_oracle_fluid_skips_massless_body():
  """passive_test.py:129-155: an empty free body (mass 0) with a massive child: the child's force only,
  applied at the child's xipos."""
  mjm = _load("""<mujoco><option density="1.2" viscosity="0.1"/><worldbody><geom name="floor" type="plane" size="10 10 0.1"/>
  <body name="empty_root" pos="0 0 0.5"><freejoint/><body name="child" pos="0.1 0 0"><geom type="sphere" size="0.1" mass="1"/></body></body>
  </worldbody></mujoco>""")
  assert mjm.body_mass[1] == 0
  od = _forward(mjm, qvel=np.array([[0.2, -0.1, 0.3, 0.5, -0.4, 0.1]]))
  assert np.all(np.isfinite(od.qfrc_fluid)) and np.abs(od.qfrc_fluid).max() > 0


def test_put_model_refuses_fluid_with_implicit():
  """io.py:126-130."""
  import mujoco_warp_amd as mjw

  mjm = _load(SPHERE.format(rho=1, mu=0.1, w="0 0 0", r=0.1, shape=""))
  mjm.opt.integrator = 3
  with pytest.raises(NotImplementedError, match="fluid"):
    mjw.put_model(mjm, device="cpu")
  m = _load(SPHERE.format(rho=0, mu=0, w="1 0 0", r=0.1, shape=""))
  m.opt.integrator = 3  # wind alone is no fluid force source without density or viscosity
  mjw.put_model(m, device="cpu")


@pytest.mark.gpu
def test_gpu_full_gravcomp_holds_still():
  """The HIP path: a gravity-compensated chain at rest stays at rest for 200 steps (Euler, CG)."""
  import torch

  import mujoco_warp_amd as mjw

  mjm = _load(CHAIN.format(g="0.3 -0.2 -9.81", gc=1))
  nworld = 4
  m, d = gpu_from_state(mjm, np.tile(mjm.qpos0, (nworld, 1)), np.zeros((nworld, mjm.nv)), np.zeros((nworld, 0)), njmax=16, nconmax=4)
  for _ in range(200):
    mjw.step(m, d)
  torch.cuda.synchronize()
  assert np.abs(np_(d.qpos) - mjm.qpos0).max() < 1e-5
  assert np.abs(np_(d.qfrc_gravcomp) - np_(d.qfrc_bias)).max() < 1e-5 * np.abs(np_(d.qfrc_bias)).max()


@pytest.mark.gpu
@pytest.mark.parametrize("staged", [False, True])
@pytest.mark.parametrize("sparse", [False, True])
def test_gpu_actuatorgravcomp_routing(staged, sparse):
  """qfrc_gravcomp / qfrc_passive / qfrc_actuator of the routed joint against the oracle, through the
  fused forward and through the staged path with an act_bias callback (mjw_actuator_map), on the dense
  and the sparse (workgroup-per-world) pipelines."""
  import torch

  import mujoco_warp_amd as mjw

  mjm = _load(GC_XML.format(rng='actuatorfrcrange="-1 1"'))
  if sparse:
    mjm.opt.jacobian = 1
  rng = np.random.default_rng(2)
  qpos, qvel, ctrl = rng.normal(0, 0.5, (4, mjm.nq)), rng.normal(0, 1, (4, mjm.nv)), rng.normal(0, 0.3, (4, mjm.nu))
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=16, nconmax=4)
  assert m.is_sparse == sparse
  if staged:
    m.callback.act_bias = lambda m_, d_: None
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=16, nconmax=4)
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  for f in ("qfrc_gravcomp", "qfrc_passive", "qfrc_actuator", "qacc"):
    want = getattr(od, f)
    np.testing.assert_allclose(np_(getattr(d, f)), want, rtol=1e-5, atol=1e-6 * (np.abs(want).max() + 1e-3), err_msg=f)
