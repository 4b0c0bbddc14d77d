"""Reference API surface around the step path: get_state / set_state,
contact_force, mul_m, step1 / step2, the sensor stage functions.

CPU tests run the torch-side helpers on CPU tensors; `-m gpu` tests check that the split / staged
entry points reproduce the fused step.
"""

import os

import numpy as np
import pytest
import torch

from tests.common import HUMANOID, ROOT, np_

APOLLO = os.path.join(ROOT, "models", "apptronik_apollo", "scene_flat.xml")


def _cpu_data(path, nworld=3):
  import mujoco_warp_amd as mjw

  mjm = mjw.load_model(path)
  m = mjw.put_model(mjm, device="cpu")
  d = mjw.make_data(mjm, nworld=nworld, nconmax=8, njmax=32, device="cpu", m=m)
  return mjm, m, d


def test_state_roundtrip_and_size():
  import mujoco_warp_amd as mjw
  from mujoco_warp_amd.types import State

  mjm, m, d = _cpu_data(HUMANOID)
  g = torch.Generator().manual_seed(0)
  for name in ("qpos", "qvel", "ctrl", "qacc_warmstart", "qfrc_applied", "xfrc_applied", "time"):
    getattr(d, name).copy_(torch.rand(getattr(d, name).shape, generator=g))
  sig = int(State.INTEGRATION)
  n = mjw.state_size(m, sig)
  assert n == 1 + mjm.nq + mjm.nv + mjm.na + mjm.nv + mjm.nu + mjm.nv + 6 * mjm.nbody  # mj_stateSize
  st = torch.zeros((d.nworld, n))
  mjw.get_state(m, d, st, sig)
  assert torch.equal(st[:, 1 : 1 + mjm.nq], d.qpos)
  _, _, d2 = _cpu_data(HUMANOID)
  mjw.set_state(m, d2, st, sig)
  for name in ("qpos", "qvel", "ctrl", "qacc_warmstart", "qfrc_applied", "xfrc_applied", "time"):
    assert torch.equal(getattr(d2, name), getattr(d, name)), name
  # per-world mask: only world 1 is written
  _, _, d3 = _cpu_data(HUMANOID)
  mjw.set_state(m, d3, st, int(State.QPOS), active=torch.tensor([False, True, False]))
  assert torch.equal(d3.qpos[1], st[1, : mjm.nq]) and torch.equal(d3.qpos[0], torch.as_tensor(mjm.qpos0, dtype=torch.float32))
  with pytest.raises(ValueError):
    mjw.get_state(m, d, st, 1 << 13)


def test_contact_force_decodes_pyramid():
  """Pyramidal rows (f1+, f1-, f2+, f2-) -> normal = sum, tangent_i = (f_i+ - f_i-) mu_i (support.py:241-263)."""
  import mujoco_warp_amd as mjw

  mjm, m, d = _cpu_data(HUMANOID)
  d.nacon[0] = 2
  d.contact.dim[:2] = torch.tensor([3, 1])
  d.contact.worldid[:2] = torch.tensor([1, 2])
  d.contact.efc_address[0, :4] = torch.tensor([5, 6, 7, 8])
  d.contact.efc_address[1, :1] = torch.tensor([3])
  d.contact.friction[0] = torch.tensor([0.5, 0.25, 0.1, 0.1, 0.1])
  d.efc.force[1, 5:9] = torch.tensor([1.0, 2.0, 4.0, 3.0])
  d.efc.force[2, 3] = 7.0
  R = torch.tensor([[0.0, 0.0, 1.0], [1.0, 0.0, 0.0], [0.0, 1.0, 0.0]])
  d.contact.frame[0] = R
  force = torch.zeros((3, 6))
  mjw.contact_force(m, d, torch.tensor([0, 1, 5]), False, force)
  np.testing.assert_allclose(force[0].numpy(), [10.0, -0.5, 0.25, 0, 0, 0], atol=1e-6)
  np.testing.assert_allclose(force[1].numpy(), [7.0, 0, 0, 0, 0, 0])
  assert torch.all(force[2] == 0)  # id >= nacon
  mjw.contact_force(m, d, torch.tensor([0]), True, force[:1])
  np.testing.assert_allclose(force[0, :3].numpy(), (torch.tensor([10.0, -0.5, 0.25]) @ R).numpy(), atol=1e-6)


def test_mul_m_dense():
  import mujoco_warp_amd as mjw

  mjm, m, d = _cpu_data(HUMANOID)
  nv = mjm.nv
  A = torch.rand((d.nworld, nv, nv))
  d.qM[:, :nv, :nv] = A + A.transpose(1, 2)
  v = torch.rand((d.nworld, nv))
  res = torch.zeros_like(v)
  mjw.mul_m(m, d, res, v, skip=torch.tensor([False, True, False]))
  want = torch.einsum("wij,wj->wi", d.qM[:, :nv, :nv], v)
  assert torch.allclose(res[0], want[0]) and torch.all(res[1] == 0) and torch.allclose(res[2], want[2])


# ---- GPU ---------------------------------------------------------------------------------------
def _apollo_gpu(nworld=16, seed=0):
  import mujoco_warp_amd as mjw
  from tests.common import gpu_from_state

  mjm = mjw.load_model(APOLLO)
  rng = np.random.default_rng(seed)
  qpos = np.tile(mjm.key_qpos[0], (nworld, 1))
  qpos[:, 7:] += rng.normal(0, 0.05, (nworld, mjm.nq - 7))
  qvel = rng.normal(0, 0.2, (nworld, mjm.nv))
  ctrl = np.tile(mjm.key_ctrl[0], (nworld, 1))
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=16)
  m2, d2 = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=64, nconmax=16)
  return mjm, m, d, m2, d2


@pytest.mark.gpu
def test_gpu_step1_step2_equals_step():
  import mujoco_warp_amd as mjw

  mjm, m, d, m2, d2 = _apollo_gpu()
  for _ in range(3):
    mjw.step(m, d)
    mjw.step1(m2, d2)
    mjw.step2(m2, d2)
  torch.cuda.synchronize()
  np.testing.assert_array_equal(np_(d.qpos), np_(d2.qpos))
  np.testing.assert_array_equal(np_(d.sensordata), np_(d2.sensordata))


@pytest.mark.gpu
def test_gpu_callbacks_take_the_staged_path_with_sensors():
  import mujoco_warp_amd as mjw

  mjm, m, d, m2, d2 = _apollo_gpu(seed=1)
  calls = []
  m2.callback.control = lambda mm, dd: calls.append(1)
  mjw.forward(m, d)
  mjw.forward(m2, d2)
  torch.cuda.synchronize()
  assert calls == [1]
  np.testing.assert_array_equal(np_(d.sensordata), np_(d2.sensordata))
  np.testing.assert_array_equal(np_(d.qacc), np_(d2.qacc))


@pytest.mark.gpu
def test_gpu_get_set_state_roundtrip():
  import mujoco_warp_amd as mjw
  from mujoco_warp_amd.types import State

  mjm, m, d, m2, d2 = _apollo_gpu(seed=2)
  mjw.step(m, d)
  sig = int(State.FULLPHYSICS | State.CTRL | State.WARMSTART)
  st = torch.zeros((d.nworld, mjw.state_size(m, sig)), device=d.qpos.device)
  mjw.get_state(m, d, st, sig)
  mjw.set_state(m2, d2, st, sig)
  mjw.step(m, d)
  mjw.step(m2, d2)
  torch.cuda.synchronize()
  np.testing.assert_array_equal(np_(d.qpos), np_(d2.qpos))


def _humanoid_gpu(seed, gain_scale=1.0):
  import mujoco_warp_amd as mjw
  from tests.common import gpu_from_state, humanoid_model, random_states

  mjm = humanoid_model("CG")
  mjm.actuator_gainprm = np.array(mjm.actuator_gainprm, dtype=np.float64) * gain_scale
  qpos, qvel, ctrl = random_states(mjm, 8, seed=seed)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  return mjm, m, d


@pytest.mark.gpu
def test_gpu_act_callbacks_run_between_force_and_moment_map():
  """act_dyn / act_gain / act_bias (forward.py:876-881) run in that order after the actuator forces and
  before the moment map: a gain callback that doubles every humanoid motor force (FIXED gain, no bias,
  no force limit) steps bitwise like a model whose gains are doubled (x2 is exact in fp32), and the
  callbacks see the forces _actuator_force computed."""
  import mujoco_warp_amd as mjw

  mjm, m, d = _humanoid_gpu(seed=90)
  assert not np.asarray(mjm.actuator_forcelimited).any() and (np.asarray(mjm.actuator_biastype) == 0).all()
  _, m2, d2 = _humanoid_gpu(seed=90, gain_scale=2.0)
  order, seen = [], []

  def gain(mm, dd):
    order.append("gain")
    seen.append(dd.actuator_force.clone())
    dd.actuator_force.mul_(2.0)

  m.callback.act_dyn = lambda mm, dd: order.append("dyn")
  m.callback.act_gain = gain
  m.callback.act_bias = lambda mm, dd: order.append("bias")
  for _ in range(3):
    mjw.step(m, d)
    mjw.step(m2, d2)
  torch.cuda.synchronize()
  assert order == ["dyn", "gain", "bias"] * 3
  assert float(seen[0].abs().max()) > 0
  np.testing.assert_array_equal(np_(d.actuator_force), np_(d2.actuator_force))
  np.testing.assert_array_equal(np_(d.qfrc_actuator), np_(d2.qfrc_actuator))
  np.testing.assert_array_equal(np_(d.qpos), np_(d2.qpos))
  np.testing.assert_array_equal(np_(d.qvel), np_(d2.qvel))


@pytest.mark.gpu
def test_gpu_world_order_does_not_change_results():
  """The dense path's longest-first world order (d.sched, mjw_step.hip reset_counters_kernel): after a
  step, world_order is a permutation of the worlds ordered by the recorded iteration buckets, and 5
  steps give bitwise the same state as with d.sched = None (identity order)."""
  import torch

  import mujoco_warp_amd as mjw
  from tests.common import gpu_from_state, humanoid_model, np_, random_states

  mjm = humanoid_model("CG")
  nworld = 257
  qpos, qvel, ctrl = random_states(mjm, nworld, seed=90)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  m2, d2 = gpu_from_state(mjm, qpos, qvel, ctrl)
  d2.sched = None
  for i in range(5):
    if i == 4:
      torch.cuda.synchronize()
      key4 = d.world_key.cpu().numpy().copy()  # the buckets step 4 recorded
    mjw.step(m, d)
    mjw.step(m2, d2)
  torch.cuda.synchronize()
  for f in ("qpos", "qvel", "qacc", "act", "solver_niter"):
    assert np.array_equal(np_(getattr(d, f)), np_(getattr(d2, f))), f
  # step 5 walked the permutation its counter-reset kernel built from step 4's buckets: most
  # iterations (smallest key) first
  order = d.world_order.cpu().numpy()
  assert sorted(order.tolist()) == list(range(nworld))
  assert np.all(np.diff(key4[order]) >= 0)
  assert len(np.unique(key4)) > 1


@pytest.mark.gpu
def test_gpu_world_order_from_any_keys():
  """The counter-reset kernel builds world_order from world_key alone (no histogram the dense kernels
  count): any key values -- out of range, stale -- give a permutation sorted by the clamped key, and one
  bucket holding 7/8 of the worlds or more gives the identity (franka: every world 1-2 Newton iterations)."""
  import torch

  import mujoco_warp_amd as mjw
  from tests.common import gpu_from_state, humanoid_model, random_states

  mjm = humanoid_model("CG")
  nworld = 1000
  qpos, qvel, ctrl = random_states(mjm, nworld, seed=91)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  rng = np.random.default_rng(91)
  keys = rng.integers(-5, 40, size=nworld).astype(np.int32)
  d.world_key.copy_(torch.as_tensor(keys, device=d.world_key.device))
  mjw.step(m, d)
  torch.cuda.synchronize()
  order = d.world_order.cpu().numpy()
  assert sorted(order.tolist()) == list(range(nworld))
  assert np.all(np.diff(np.clip(keys, 0, 31)[order]) >= 0)
  keys = np.full(nworld, 3, np.int32)
  keys[: nworld // 8 - 1] = 7
  d.world_key.copy_(torch.as_tensor(keys, device=d.world_key.device))
  mjw.step(m, d)
  torch.cuda.synchronize()
  np.testing.assert_array_equal(d.world_order.cpu().numpy(), np.arange(nworld))


@pytest.mark.gpu
def test_gpu_pool_counters_adjacent_or_not():
  """io.py allocates nacon and ncollision adjacent, and the dense step adds a world's broadphase count and
  its contact-slot reservation with one 64-bit atomic (mjw_step.hip collision_and_constraints); a caller
  that swaps in its own ncollision tensor gets the two 32-bit atomics instead: same counts, same state."""
  import torch

  import mujoco_warp_amd as mjw
  from tests.common import gpu_from_state, humanoid_model, np_, random_states

  mjm = humanoid_model("CG")
  nworld = 300
  qpos, qvel, ctrl = random_states(mjm, nworld, seed=92)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl)
  m2, d2 = gpu_from_state(mjm, qpos, qvel, ctrl)
  assert d.ncollision.data_ptr() == d.nacon.data_ptr() + 4
  d2.ncollision = torch.zeros(1, dtype=torch.int32, device=d2.nacon.device)
  assert d2.ncollision.data_ptr() != d2.nacon.data_ptr() + 4
  for _ in range(3):
    mjw.step(m, d)
    mjw.step(m2, d2)
  torch.cuda.synchronize()
  assert int(d.nacon[0]) == int(d2.nacon[0]) > 0
  assert int(d.ncollision[0]) == int(d2.ncollision[0]) > 0
  for f in ("qpos", "qvel", "qacc"):
    assert np.array_equal(np_(getattr(d, f)), np_(getattr(d2, f))), f
