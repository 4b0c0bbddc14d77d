"""The contactfilter callback (collision_driver.py:788-789): called after the narrowphase filled d.contact,
before make_constraint reads it (constraint.py:2718-2779).  This build runs the callback after the position
stage and then rebuilds the constraint rows from the contact pool as the callback left it
(mjw_contact_rows: the position stage with the contacts read back from the pool; a contact whose `type` lost
the CONSTRAINT bit gets no rows, constraint.py:1731).

Checks (-m gpu, humanoid in floor contact, and the sparse cloth path): a no-op filter gives the fused step
bitwise; a filter that takes every contact out equals the model with contacts disabled; a filter that halves
the sliding friction equals the model whose geoms have half the friction.  Parity with the reference is
pinned through these equivalences (the reference has no contactfilter test of its own).
"""

import numpy as np
import pytest

from tests.common import HUMANOID, np_, random_states


def test_contactfilter_is_a_staged_callback():
  import importlib

  fwd = importlib.import_module("mujoco_warp_amd.forward")
  assert "contactfilter" in fwd._STAGED_CALLBACKS and not fwd._UNSUPPORTED_CALLBACKS


def _humanoid(nworld, seed=5, **geom_scale):
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf, types

  mjm = mjcf.load_model(HUMANOID)
  mjm.opt.solver = types.SolverType.CG  # the benchmark's solver
  if geom_scale.get("friction"):
    mjm.geom_friction = mjm.geom_friction.copy()
    mjm.geom_friction[:, 0] *= geom_scale["friction"]
  if geom_scale.get("nocontact"):
    mjm.opt.disableflags |= types.DisableBit.CONTACT
  qpos, qvel, ctrl = random_states(mjm, nworld, seed=seed, qpos_noise=0.1, qvel_noise=0.5)
  qpos[:, 2] -= 0.35  # into the floor: several contacts per world
  m = mjw.put_model(mjm, device="cuda")
  d = mjw.make_data(mjm, nworld=nworld, nconmax=32, njmax=64, device="cuda", m=m)
  d.qpos[:] = torch.as_tensor(qpos, dtype=torch.float32, device="cuda")
  d.qvel[:] = torch.as_tensor(qvel, dtype=torch.float32, device="cuda")
  d.ctrl[:] = torch.as_tensor(ctrl, dtype=torch.float32, device="cuda")
  return m, d


STATE = ("qpos", "qvel", "qacc", "qacc_warmstart", "qfrc_constraint")


def _per_world(d, field):
  """A contact field grouped by world, each world's contacts in pool-slot order: the pool interleaves the
  worlds in the order their atomics landed, which differs from run to run; within a world the slots
  ascend in pair order."""
  n = int(d.nacon[0])
  w = np_(d.contact.worldid)[:n]
  v = np_(getattr(d.contact, field))[:n]
  return [v[w == i] for i in range(int(w.max()) + 1)]


def _assert_contacts_equal(d, d2, field):
  a, b = _per_world(d, field), _per_world(d2, field)
  assert len(a) == len(b)
  for i, (x, y) in enumerate(zip(a, b)):
    np.testing.assert_array_equal(x, y, err_msg=f"{field} world {i}")


@pytest.mark.gpu
def test_gpu_contactfilter_noop_equals_fused_step():
  import torch

  import mujoco_warp_amd as mjw

  m, d = _humanoid(64)
  m2, d2 = _humanoid(64)
  calls = []
  m2.callback.contactfilter = lambda mm, dd: calls.append(int(dd.nacon[0]))
  for _ in range(3):
    mjw.step(m, d)
    mjw.step(m2, d2)
  torch.cuda.synchronize()
  assert len(calls) == 3 and min(calls) >= 64
  assert int(d.nacon[0]) == int(d2.nacon[0])
  for name in STATE + ("nefc",):
    np.testing.assert_array_equal(np_(getattr(d, name)), np_(getattr(d2, name)), err_msg=name)
  for f in ("efc_address", "dist", "frame", "friction", "geom"):
    _assert_contacts_equal(d, d2, f)
  np.testing.assert_array_equal(np_(d.efc.J), np_(d2.efc.J))


@pytest.mark.gpu
def test_gpu_contactfilter_drop_all_equals_contacts_disabled():
  import torch

  import mujoco_warp_amd as mjw

  m, d = _humanoid(32)
  mr, dr = _humanoid(32, nocontact=True)

  def drop(mm, dd):
    dd.contact.type.zero_()

  m.callback.contactfilter = drop
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()
  n = int(d.nacon[0])
  assert n >= 32
  assert (np_(d.contact.efc_address)[:n] == -1).all()
  mjw.step(m, d)
  mjw.step(mr, dr)
  torch.cuda.synchronize()
  np.testing.assert_array_equal(np_(d.nefc), np_(dr.nefc))
  for name in STATE:
    np.testing.assert_allclose(np_(getattr(d, name)), np_(getattr(dr, name)), rtol=1e-6, atol=1e-6, err_msg=name)


@pytest.mark.gpu
def test_gpu_contactfilter_friction_edit_equals_model_friction():
  import torch

  import mujoco_warp_amd as mjw

  m, d = _humanoid(32, seed=9)
  mr, dr = _humanoid(32, seed=9, friction=0.5)

  def half(mm, dd):
    n = int(dd.nacon[0])
    dd.contact.friction[:n, :2] *= 0.5

  m.callback.contactfilter = half
  for _ in range(2):
    mjw.step(m, d)
    mjw.step(mr, dr)
  torch.cuda.synchronize()
  assert int(d.nacon[0]) == int(dr.nacon[0]) >= 32
  _assert_contacts_equal(d, dr, "friction")
  for name in STATE:
    np.testing.assert_allclose(np_(getattr(d, name)), np_(getattr(dr, name)), rtol=1e-6, atol=1e-6, err_msg=name)


@pytest.mark.gpu
def test_gpu_contactfilter_sparse_path():
  """Cloth (sparse / flex path): a no-op filter equals the fused step; dropping every contact leaves only
  the equality / friction / limit rows."""
  import torch

  import mujoco_warp_amd as mjw
  from tests.cloth_common import cloth_model, cloth_states

  mjm = cloth_model()
  qpos, qvel, _ = cloth_states(mjm, 4, seed=2)

  def make():
    m = mjw.put_model(mjm, device="cuda")
    d = mjw.make_data(mjm, nworld=4, nconmax=400, njmax=4000, device="cuda", m=m)
    d.qpos[:] = torch.as_tensor(qpos, dtype=torch.float32, device="cuda")
    d.qvel[:] = torch.as_tensor(qvel, dtype=torch.float32, device="cuda")
    return m, d

  m, d = make()
  m2, d2 = make()
  m2.callback.contactfilter = lambda mm, dd: None
  for _ in range(2):
    mjw.step(m, d)
    mjw.step(m2, d2)
  torch.cuda.synchronize()
  assert int(d.nacon[0]) > 0
  for name in ("qpos", "qvel", "nefc"):
    np.testing.assert_array_equal(np_(getattr(d, name)), np_(getattr(d2, name)), err_msg=name)
  m3, d3 = make()

  def drop(mm, dd):
    dd.contact.type.zero_()

  m3.callback.contactfilter = drop
  mjw.fwd_position(m3, d3)
  torch.cuda.synchronize()
  ne, nf, nl, nefc = (np_(getattr(d3, k)) for k in ("ne", "nf", "nl", "nefc"))
  np.testing.assert_array_equal(nefc, ne + nf + nl)
  assert int(d3.nacon[0]) > 0
