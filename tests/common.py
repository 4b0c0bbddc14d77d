"""Shared parity-test helpers: build matching GPU and oracle states, compare outputs.

The oracle (oracle/orc.py) is the checker only; it is never on the product path.
"""

from __future__ import annotations

import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HUMANOID = os.path.join(ROOT, "models", "humanoid.xml")
FRANKA = os.path.join(ROOT, "models", "franka_emika_panda", "scene.xml")

# free boxes over a plane (plane-box narrowphase); boxes do not collide with each other
# (contype 2 / conaffinity 1) because box-box is not built yet
BOXES_XML = """<mujoco><option timestep="0.002"/><worldbody><geom type="plane" size="5 5 .1"/>
<body pos="-.5 0 .2"><freejoint/><geom type="box" size=".1 .08 .06" contype="2" conaffinity="1"/></body>
<body pos=".0 0 .2"><freejoint/><geom type="box" size=".05 .12 .04" contype="2" conaffinity="1"/></body>
<body pos=".5 0 .2"><freejoint/><geom type="box" size=".07 .07 .07" contype="2" conaffinity="1" condim="1"/></body>
</worldbody></mujoco>"""


def humanoid_model(solver="CG", iterations=None, ls_iterations=None):
  from mujoco_warp_amd import mjcf

  m = mjcf.load_model(HUMANOID)
  m.opt.solver = {"CG": 1, "NEWTON": 2}[solver]
  if iterations is not None:
    m.opt.iterations = iterations
  if ls_iterations is not None:
    m.opt.ls_iterations = ls_iterations
  return m


def franka_model(solver=None):
  from mujoco_warp_amd import mjcf

  m = mjcf.load_model(FRANKA)
  if solver is not None:
    m.opt.solver = {"CG": 1, "NEWTON": 2}[solver]
  return m


def franka_states(mjm, nworld, seed=0, qvel_noise=0.3):
  """Joint positions uniform inside the joint ranges, controls inside ctrlrange (seeded)."""
  rng = np.random.default_rng(seed)
  lo, hi = mjm.jnt_range[:, 0], mjm.jnt_range[:, 1]
  qpos = lo + (hi - lo) * rng.uniform(0.05, 0.95, (nworld, mjm.nq))
  qvel = rng.normal(0, qvel_noise, (nworld, mjm.nv))
  cr = mjm.actuator_ctrlrange
  ctrl = cr[:, 0] + (cr[:, 1] - cr[:, 0]) * rng.uniform(0, 1, (nworld, mjm.nu))
  return qpos, qvel, ctrl


def boxes_states(mjm, nworld, seed=0):
  """Three free boxes at random orientations, lowered so that corners touch or penetrate the plane."""
  from mujoco_warp_amd.mjcf import quat_to_mat

  rng = np.random.default_rng(seed)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  for w in range(nworld):
    for b in range(3):
      q = rng.normal(size=4)
      q /= np.linalg.norm(q)
      R = quat_to_mat(q)
      half = mjm.geom_size[1 + b]
      lowest = np.abs(R @ np.diag(half)).sum(axis=1)[2]  # half extent along z
      qpos[w, 7 * b + 2] = lowest - rng.uniform(-0.004, 0.01)
      qpos[w, 7 * b + 3 : 7 * b + 7] = q
  qvel = rng.normal(0, 0.2, (nworld, mjm.nv))
  return qpos, qvel, np.zeros((nworld, mjm.nu))


def random_states(mjm, nworld, seed=0, key=0, qpos_noise=0.05, qvel_noise=0.5, ctrl_noise=1.0):
  """Per-world randomized states around a keyframe (test_data.fixture style, seeded)."""
  rng = np.random.default_rng(seed)
  qpos = np.tile(mjm.key_qpos[key], (nworld, 1))
  qpos[:, 7:] += rng.normal(0, qpos_noise, (nworld, mjm.nq - 7))
  qpos[:, :3] += rng.normal(0, qpos_noise * 0.2, (nworld, 3))
  q = qpos[:, 3:7] + rng.normal(0, qpos_noise * 0.2, (nworld, 4))
  qpos[:, 3:7] = q / np.linalg.norm(q, axis=1, keepdims=True)
  qvel = rng.normal(0, qvel_noise, (nworld, mjm.nv))
  ctrl = np.clip(rng.normal(0, ctrl_noise, (nworld, mjm.nu)), -1, 1)
  return qpos, qvel, ctrl


def oracle_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=64, real_bits=64, qacc_warmstart=None):
  from oracle import orc

  om = orc.OracleModel(mjm, real_bits=real_bits)
  od = orc.OracleData(om, qpos.shape[0], njmax, nconmax)
  od.qpos[:] = qpos
  od.qvel[:] = qvel
  od.ctrl[:] = ctrl
  if qacc_warmstart is not None:
    od.qacc_warmstart[:] = qacc_warmstart
  return om, od


def gpu_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=24, qacc_warmstart=None):
  import torch

  import mujoco_warp_amd as mjw

  nworld = qpos.shape[0]
  m = mjw.put_model(mjm, device="cuda")
  d = mjw.make_data(mjm, nworld=nworld, nconmax=nconmax, njmax=njmax, device="cuda", m=m)
  d.qpos[:] = torch.as_tensor(qpos, dtype=torch.float32, device="cuda")
  d.qvel[:] = torch.as_tensor(qvel, dtype=torch.float32, device="cuda")
  d.ctrl[:] = torch.as_tensor(ctrl, dtype=torch.float32, device="cuda")
  if qacc_warmstart is not None:
    d.qacc_warmstart[:] = torch.as_tensor(qacc_warmstart, dtype=torch.float32, device="cuda")
  return m, d


def np_(t):
  return t.detach().cpu().numpy().astype(np.float64)


def assert_close(name, got, want, rtol, atol):
  got = np.asarray(got, dtype=np.float64)
  want = np.asarray(want, dtype=np.float64)
  assert got.shape == want.shape, f"{name}: shape {got.shape} != {want.shape}"
  err = np.abs(got - want)
  tol = atol + rtol * np.abs(want)
  bad = err > tol
  if bad.any():
    i = np.unravel_index(np.argmax(err - tol), err.shape)
    raise AssertionError(f"{name}: {bad.sum()} / {bad.size} out of tolerance; worst at {i}: got {got[i]} want {want[i]} (rtol={rtol}, atol={atol})")


def gpu_rows(d, w, nv):
  """GPU efc rows of world w as numpy dict (first nefc rows)."""
  n = min(int(d.nefc[w]), d.njmax)
  return dict(
    n=int(d.nefc[w]),
    J=np_(d.efc.J[w, :n, :nv]),
    D=np_(d.efc.D[w, :n]),
    aref=np_(d.efc.aref[w, :n]),
    pos=np_(d.efc.pos[w, :n]),
    vel=np_(d.efc.vel[w, :n]),
    margin=np_(d.efc.margin[w, :n]),
    type=d.efc.type[w, :n].cpu().numpy(),
  )


def oracle_rows(od, w, nv):
  n = min(int(od.nefc[w, 0]), od.njmax)
  return dict(
    n=int(od.nefc[w, 0]),
    J=od.efc_J[w].reshape(od.njmax, nv)[:n],
    D=od.efc_D[w, :n],
    aref=od.efc_aref[w, :n],
    pos=od.efc_pos[w, :n],
    vel=od.efc_vel[w, :n],
    margin=od.efc_margin[w, :n],
    type=od.efc_type[w, :n],
  )


def dense_efc_J(m, d, w):
  """The first nefc constraint Jacobian rows of world w as a dense (n, nv) array, from either layout."""
  n = min(int(d.nefc[w]), d.njmax)
  if not m.is_sparse:
    return np_(d.efc.J[w, :n, :m.nv])
  from tests.cloth_common import dense_J

  return dense_J(d, w, n, m.nv)
