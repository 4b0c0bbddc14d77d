"""Flexes of every dimension: dim-1 (cables), dim-2 membranes and dim-3 (volumetric) flexcomps, pins.

The reference runs them through the same kernels as the dim-2 cloth: flex kinematics / edges
(smooth.py:228-355), `_flex_elasticity` over the element's local edges (passive.py:566-662, dims 1-3),
flex edge equality rows, vertex-plane contacts (collision_flex.py:261-378) and the dim-3 shell
triangles against primitives (:531-683).  Its own test (forward_test.py:652 `test_multiflex`) runs
`forward` on `flex/multiflex.xml` (a pinned rope, a pinned towel and a soft block; copied with rope.xml
/ floppy.xml into models/test_data/flex).

Compiler constants: MuJoCo's compiler is absent here, so the element metric is restated from the Saint
Venant-Kirchhoff energy (mjcf._svk_metric) and pinned by that definition: 1/4 s' M s equals the
energy evaluated directly from the deformation gradient for random elements, and the oracle's elastic
force is minus the gradient of that energy (finite differences).  The tetrahedralisation and the shell
order are parity unpinned.  Under `-m gpu` the sparse device pipeline follows the oracle on the same
scenes.
"""

import os

import numpy as np
import pytest

from tests.common import ROOT, gpu_from_state, np_, oracle_from_state

FLEX = os.path.join(ROOT, "models", "test_data", "flex")

SMALL = """<mujoco><option solver="CG" tolerance="1e-8" timestep=".001"/>
<worldbody>
  <geom name="floor" type="plane" size="0 0 1"/>
  <geom name="ball" type="sphere" size=".12" pos=".35 -.45 .22"/>
  <body name="flexes" pos="0 0 .5">
    <flexcomp type="grid" count="6 1 1" spacing=".1 .1 .1" pos="-.3 .3 0" radius=".02" name="rope" dim="1" mass=".5">
      <edge equality="true"/>
      <contact condim="3" contype="0" conaffinity="0"/>
      <pin id="0"/>
    </flexcomp>
    <flexcomp type="grid" count="4 3 1" spacing=".1 .1 .1" pos=".3 .3 0" radius=".01" name="sheet" dim="2" mass=".2">
      <contact condim="3" contype="0" conaffinity="0"/>
      <elasticity young="3e3" poisson=".3" thickness=".01" elastic2d="both" damping=".001"/>
      <pin id="0"/>
    </flexcomp>
    <flexcomp type="grid" count="3 2 2" spacing=".1 .1 .1" pos=".3 -.4 -.2" radius="0" name="block" dim="3" mass="2">
      <contact condim="3" solref=".01 1"/>
      <elasticity young="2e4" damping=".002" poisson=".2"/>
    </flexcomp>
  </body>
</worldbody></mujoco>"""


def _small():
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(SMALL)


def _direct_energy(X, x, young, poisson, dim, thickness, radius):
  """SVK energy of one element from its deformation gradient (rest X, deformed x)."""
  lam = young * poisson / ((1 + poisson) * (1 - 2 * poisson))
  mu = young / (2 * (1 + poisson))
  Dm, Ds = (X[1:] - X[0]).T, (x[1:] - x[0]).T
  if dim == 1:
    L0, L = np.linalg.norm(Dm[:, 0]), np.linalg.norm(Ds[:, 0])
    eps = (L * L - L0 * L0) / (2 * L0 * L0)
    return 0.5 * young * (L0 * np.pi * radius**2) * eps**2
  if dim == 2:
    # rest triangle in its own plane: orthonormal basis (u, v), F maps 2D rest coordinates to 3D
    u = Dm[:, 0] / np.linalg.norm(Dm[:, 0])
    nrm = np.cross(Dm[:, 0], Dm[:, 1])
    v = np.cross(nrm / np.linalg.norm(nrm), u)
    P = np.array([[Dm[:, k] @ u, Dm[:, k] @ v] for k in range(2)]).T  # 2 x 2
    F = Ds @ np.linalg.inv(P)  # 3 x 2
    E = 0.5 * (F.T @ F - np.eye(2))
    lam2 = 2 * lam * mu / (lam + 2 * mu)
    vol = 0.5 * np.linalg.norm(nrm) * thickness
    return vol * (mu * np.trace(E @ E) + 0.5 * lam2 * np.trace(E) ** 2)
  F = Ds @ np.linalg.inv(Dm)
  E = 0.5 * (F.T @ F - np.eye(3))
  vol = abs(np.linalg.det(Dm)) / 6
  return vol * (mu * np.trace(E @ E) + 0.5 * lam * np.trace(E) ** 2)


@pytest.mark.parametrize("dim", [1, 2, 3])
def test_svk_metric_is_the_direct_energy(dim):
  from mujoco_warp_amd import mjcf

  rng = np.random.default_rng(dim)
  for _ in range(5):
    X = rng.normal(size=(dim + 1, 3))
    x = X + 0.1 * rng.normal(size=X.shape)
    young, poisson, th, rad = 1e4, 0.3, 0.01, 0.02
    M = mjcf._svk_metric(X, young, poisson, dim, th, rad)
    ed = mjcf._FLEX_LOCAL_EDGES[dim]
    s = np.array([np.sum((x[j] - x[i]) ** 2) - np.sum((X[j] - X[i]) ** 2) for i, j in ed])
    np.testing.assert_allclose(0.25 * s @ M @ s, _direct_energy(X, x, young, poisson, dim, th, rad), rtol=1e-9)


def test_compiler_grids_pins_and_shells():
  mjm = _small()
  assert mjm.flex_dim.tolist() == [1, 2, 3]
  assert mjm.flex_elemnum.tolist() == [5, 2 * 3 * 2, 2 * 1 * 1 * 6]
  assert mjm.flex_edgenum[0] == 5
  # a 3 x 2 x 2 block: every cube face is split into two boundary triangles
  assert mjm.flex_shellnum.tolist() == [0, 0, 2 * (2 * 1 + 2 * 1 + 1 * 1) * 2]
  assert mjm.nflexelemedge == 5 * 1 + 12 * 3 + 12 * 6
  # pinned vertices: no dofs; the rope keeps 5 of its 6 vertices, the sheet 11 of 12, the block all 12
  assert mjm.nv == 3 * (5 + 11 + 12)
  # shell triangles point away from the block
  sh = mjm.flex_shell.reshape(-1, 3) + mjm.flex_vertadr[2]
  from mujoco_warp_amd import mjcf

  x = np.array([mjcf._body_world_pos(b) for b in mjcf_bodies(mjm, 2)])
  cen = x.mean(axis=0)
  for a, b, c in sh - mjm.flex_vertadr[2]:
    n = np.cross(x[b] - x[a], x[c] - x[a])
    assert n @ (x[a] - cen) > 0


def mjcf_bodies(mjm, f):
  """The compiler's vertex bodies of flex f (rest frames from body_pos up the tree)."""

  class B:
    def __init__(self, i):
      self.i = i
      self.pos = mjm.body_pos[i]
      self.quat = mjm.body_quat[i]
      self.parent = B(int(mjm.body_parentid[i])) if i > 0 else None

  vb = mjm.flex_vertbodyid[mjm.flex_vertadr[f]:mjm.flex_vertadr[f] + mjm.flex_vertnum[f]]
  return [B(int(b)) for b in vb]


def test_oracle_elastic_force_is_minus_the_energy_gradient():
  """A lone block (no damping, gravity off): qfrc_passive = -dE/dq, E = sum over elements of 1/4 s'Ms."""
  from mujoco_warp_amd import mjcf

  xml = """<mujoco><option gravity="0 0 0" timestep=".001"/><worldbody>
    <flexcomp type="grid" count="2 2 2" spacing=".1 .1 .1" radius="0" name="b" dim="3" mass="1">
      <contact contype="0" conaffinity="0"/><elasticity young="1e4" poisson=".25"/>
    </flexcomp></worldbody></mujoco>"""
  mjm = mjcf.load_model_from_string(xml)
  rng = np.random.default_rng(0)
  q = mjm.qpos0 + 0.01 * rng.normal(size=mjm.nq)
  _, od = oracle_from_state(mjm, q[None], np.zeros((1, mjm.nv)), np.zeros((1, mjm.nu)), njmax=64, nconmax=8)
  od.fwd_position()
  od.fwd_velocity()
  frc = od.qfrc_passive[0].copy()

  def energy(qq):
    X = np.array([mjcf._body_world_pos(b) for b in mjcf_bodies(mjm, 0)])
    x = X + (qq - mjm.qpos0).reshape(-1, 3)  # three slide dofs per vertex body, parent = world
    E = 0.0
    ed = mjcf._FLEX_LOCAL_EDGES[3]
    for el in range(mjm.flex_elemnum[0]):
      t = mjm.flex_elem[4 * el:4 * el + 4]
      M = np.zeros((6, 6))
      M[np.triu_indices(6)] = mjm.flex_stiffness[el][:21]
      M = M + np.triu(M, 1).T
      s = np.array([np.sum((x[t[j]] - x[t[i]]) ** 2) - np.sum((X[t[j]] - X[t[i]]) ** 2) for i, j in ed])
      E += 0.25 * s @ M @ s
    return E

  h = 1e-6
  grad = np.array([(energy(q + h * np.eye(mjm.nq)[k]) - energy(q - h * np.eye(mjm.nq)[k])) / (2 * h) for k in range(mjm.nq)])
  np.testing.assert_allclose(frc, -grad, rtol=1e-5, atol=1e-6 * np.abs(grad).max())


@pytest.mark.parametrize("name", ["multiflex", "rope", "floppy"])
def test_oracle_reference_flex_scenes_step(name):
  """forward_test.py:652 runs forward on multiflex.xml; here the oracle also steps each scene."""
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model(os.path.join(FLEX, f"{name}.xml"))
  assert mjm.nflex > 0
  _, od = oracle_from_state(mjm, mjm.qpos0[None], np.zeros((1, mjm.nv)), np.zeros((1, mjm.nu)), njmax=12000, nconmax=3000)
  od.forward()
  assert np.isfinite(od.qacc).all()
  for _ in range(20):
    od.step()
  assert np.isfinite(od.qpos).all()
  # pinned vertices stay where they are; edge equality keeps rope segments near their rest length
  if name == "rope":
    od.fwd_position()
    np.testing.assert_allclose(od.flexedge_length[0], mjm.flexedge_length0, rtol=2e-2)


def test_oracle_soft_block_rests_on_floor():
  mjm = _small()
  _, od = oracle_from_state(mjm, mjm.qpos0[None], np.zeros((1, mjm.nv)), np.zeros((1, mjm.nu)), njmax=1024, nconmax=256)
  pin0 = None
  ncon, zmin = [], []
  for i in range(700):
    od.step()
    if i % 25 == 0:
      od.fwd_position()
      x = od.flexvert_xpos[0].reshape(-1, 3)
      pin0 = x[mjm.flex_vertadr[0]].copy() if pin0 is None else pin0
      np.testing.assert_allclose(x[mjm.flex_vertadr[0]], pin0, atol=1e-12)  # the pinned rope end
      ncon.append(int(od.ncon[0, 0]))
      zmin.append(float(x[mjm.flex_vertadr[2]:, 2].min()))
  assert np.isfinite(od.qpos).all()
  # the block starts on the ball (shell-sphere contacts), falls off it onto the floor (vertex-plane
  # contacts; the soft block bounces and tumbles there) and does not sink through it
  assert ncon[0] > 0 and max(ncon[len(ncon) // 2:]) > 0
  assert min(zmin) > -0.05  # soft contacts (solref 0.02) at impact speed


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["small", "multiflex"])
def test_gpu_flex_dims_match_oracle(scene):
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = _small() if scene == "small" else mjcf.load_model(os.path.join(FLEX, "multiflex.xml"))
  nworld = 2
  rng = np.random.default_rng(3)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  qpos[1] += 0.002 * rng.normal(size=mjm.nq)
  qvel = 0.01 * rng.normal(size=(nworld, mjm.nv))
  ctrl = np.zeros((nworld, mjm.nu))
  njmax, nconmax = (1024, 256) if scene == "small" else (12000, 3000)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=nconmax)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=nconmax)
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  for f in ("flexedge_length", "qfrc_passive"):
    want = getattr(od, f)
    got = np_(getattr(d, f)).reshape(want.shape)
    np.testing.assert_allclose(got, want, rtol=2e-4, atol=2e-4 * max(1.0, np.abs(want).max()), err_msg=f)
  for w in range(nworld):
    assert int(np_(d.nefc)[w]) == int(od.nefc[w, 0])
  err = np.abs(np_(d.qacc) - od.qacc).max() / max(1.0, np.abs(od.qacc).max())
  assert err < 5e-3, err
  for _ in range(10):
    mjw.step(m, d)
  torch.cuda.synchronize()
  assert torch.isfinite(d.qpos).all()


def test_explicit_flex_matches_the_flexcomp():
  """<deformable><flex body=... element=...> over hand-made vertex bodies compiles to the flexcomp's
  tables and dynamics (a 3 x 3 sheet with bending and membrane elasticity)."""
  from mujoco_warp_amd import mjcf

  opts = '<edge equality="true"/><contact contype="0" conaffinity="0"/><elasticity young="1e3" poisson=".2" thickness=".01" elastic2d="both"/>'
  comp = mjcf.load_model_from_string(f"""<mujoco><worldbody><geom type="plane" size="0 0 1"/>
    <flexcomp type="grid" count="3 3 1" spacing=".1 .1 .1" pos="0 0 .3" radius=".01" name="s" dim="2" mass=".9">{opts}</flexcomp>
    </worldbody></mujoco>""")
  bodies, names = [], []
  for i in range(9):
    ix, iy = divmod(i, 3)
    x, y = 0.1 * (ix - 1), 0.1 * (iy - 1)
    names.append(f"v{i}")
    bodies.append(f'<body name="v{i}" pos="{x} {y} .3"><inertial pos="0 0 0" mass=".1" diaginertia="0 0 0"/>'
                  + "".join(f'<joint type="slide" axis="{ax}"/>' for ax in ("1 0 0", "0 1 0", "0 0 1")) + "</body>")
  elems = " ".join(" ".join(map(str, t)) for t in comp.flex_elem.reshape(-1, 3))
  expl = mjcf.load_model_from_string(f"""<mujoco><worldbody><geom type="plane" size="0 0 1"/>{''.join(bodies)}</worldbody>
    <deformable><flex name="s" dim="2" radius=".01" body="{' '.join(names)}" element="{elems}">{opts}</flex></deformable></mujoco>""")
  for f in ("flex_edge", "flex_edgeflap", "flex_elemedge", "flexedge_length0", "flex_bending", "flex_stiffness", "flex_vertbodyid"):
    np.testing.assert_allclose(np.asarray(getattr(expl, f), float), np.asarray(getattr(comp, f), float), rtol=1e-12, atol=1e-12, err_msg=f)
  rng = np.random.default_rng(1)
  q = comp.qpos0 + 0.01 * rng.normal(size=comp.nq)
  v = 0.1 * rng.normal(size=comp.nv)
  outs = []
  for mjm in (comp, expl):
    _, od = oracle_from_state(mjm, q[None], v[None], np.zeros((1, mjm.nu)), njmax=128, nconmax=32)
    od.forward()
    outs.append(od.qacc[0].copy())
  np.testing.assert_allclose(outs[1], outs[0], rtol=1e-10, atol=1e-10)
