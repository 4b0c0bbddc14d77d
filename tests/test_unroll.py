"""End-to-end pin: the reference's long-horizon unroll test, aloha lifts the pot (unroll_test.py:38-56).

The reference's only mujoco-free end-to-end expectation for the whole step (kinematics -> mesh collisions
-> constraint rows -> Newton solve -> Euler, ~1000 steps): `models/aloha_pot/scene.xml` (copied as input
data from the reference's `test_data/aloha_pot/`), reset to key `lift_pot0`, forward once and
qacc_warmstart = qacc (the fixture, test_data/__init__.py:99-100), the step captured once as a graph, then
for every row of `make_trajectory(mjm, find_keys(mjm, "lift_pot"))` (io.py:2591-2626): ctrl <- row,
replay.  Afterwards the reference asserts

  xpos[0, pot, 2] > 0.069 and xpos[0, lid, 2] > 0.16

with pot = mj_name2id(BODY, "partnet_100015") and lid = mj_name2id(BODY, "partnet_100015/link_0").  The
scene names the pot's root body "partnet_100015/" (trailing slash), so the reference's lookup returns -1
and numpy's xpos[0, -1] is the last body, which is the lid: the reference effectively asserts the lid
above 0.069 and 0.16.  These tests assert exactly that, and in addition the pot's own root body
("partnet_100015/") above 0.069, for both friction cones (the reference's parameters).

The CPU tests run the checker (the fp64 / fp32 C oracle) through the same trajectory; the `gpu` tests run
the HIP path through the C-ABI, once with the register-resident dense kernel (njmax 64) and once with the
generic solver kernel (njmax 256).
"""

import os

import numpy as np
import pytest

from common import ROOT

POT_XML = os.path.join(ROOT, "models", "aloha_pot", "scene.xml")
CONES = ["PYRAMIDAL", "ELLIPTIC"]


def _model(cone):
  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model(POT_XML)
  mjw.override_model(mjm, {"opt.cone": cone})
  return mjm


def _bodies(mjm):
  names = mjm.body_names
  # mj_name2id semantics: -1 when absent (then numpy index -1 = the last body, as in the reference)
  pot_ref = names.index("partnet_100015") if "partnet_100015" in names else -1
  lid = names.index("partnet_100015/link_0")
  pot_root = names.index("partnet_100015/")
  return pot_ref, lid, pot_root


def _check(xpos, mjm):
  pot_ref, lid, pot_root = _bodies(mjm)
  z = {"pot (reference lookup)": xpos[pot_ref, 2], "lid": xpos[lid, 2], "pot root body": xpos[pot_root, 2]}
  assert np.isfinite(xpos).all(), z
  assert xpos[pot_ref, 2] > 0.069, z
  assert xpos[lid, 2] > 0.16, z
  assert xpos[pot_root, 2] > 0.069, z
  return z


def test_trajectory_helpers():
  """find_keys / make_trajectory against the reference's definitions on the pot keys."""
  import mujoco_warp_amd as mjw

  mjm = _model("PYRAMIDAL")
  keys = mjw.find_keys(mjm, "lift_pot")
  assert [mjm.key_names[k] for k in keys] == [f"lift_pot{i}" for i in range(8)]
  traj = mjw.make_trajectory(mjm, keys)
  # keys at t = 0, .25, .5, .75, 1.25, 1.5, 1.75, 2.0 with dt = 0.002: 1001 rows, each key's ctrl
  # appears exactly at its own time step
  assert traj.shape == (1001, mjm.nu)
  np.testing.assert_array_equal(traj[0], mjm.key_ctrl[keys[0]])
  np.testing.assert_array_equal(traj[-1], mjm.key_ctrl[keys[-1]])
  # row 50 (t = 0.1) between key 0 and key 1 (t = 0.25): the reference restarts the blend one step after a
  # key (prev_time = the time after the key's own row, io.py:2622-2624), so frac = (0.1 - 0.002) / 0.248
  f = (0.1 - 0.002) / (0.25 - 0.002)
  np.testing.assert_allclose(traj[50], (1 - f) * mjm.key_ctrl[keys[0]] + f * mjm.key_ctrl[keys[1]], rtol=0, atol=1e-9)
  with pytest.raises(ValueError):
    mjw.make_trajectory(mjm, [keys[1], keys[0]])


def test_zero_key_quaternion_is_identity():
  """The pot's free-joint quaternion is stored as 0 0 0 0 in the keys; MuJoCo normalises it to identity."""
  mjm = _model("PYRAMIDAL")
  k = mjm.key_names.index("lift_pot0")
  j = [i for i in range(mjm.njnt) if int(mjm.jnt_type[i]) == 0][0]
  a = int(mjm.jnt_qposadr[j])
  np.testing.assert_array_equal(mjm.key_qpos[k][a + 3:a + 7], [1.0, 0.0, 0.0, 0.0])


@pytest.mark.parametrize("bits", [64, 32])
@pytest.mark.parametrize("cone", CONES)
def test_oracle_lifts_pot(cone, bits):
  """The checker itself passes the reference's end-to-end expectation (fp64 and fp32 builds)."""
  import mujoco_warp_amd as mjw
  from oracle import orc

  mjm = _model(cone)
  key = mjw.find_keys(mjm, "lift_pot0")[0]
  traj = mjw.make_trajectory(mjm, mjw.find_keys(mjm, "lift_pot"))
  od = orc.OracleData(orc.OracleModel(mjm, real_bits=bits), 1, 1024, 256)
  od.qpos[:] = mjm.key_qpos[key]
  od.qvel[:] = mjm.key_qvel[key]
  od.ctrl[:] = mjm.key_ctrl[key]
  od.forward()
  od.qacc_warmstart[:] = od.qacc
  for c in traj:
    od.ctrl[:] = c
    od.step()
  _check(np.asarray(od.xpos, dtype=np.float64).reshape(mjm.nbody, 3), mjm)


@pytest.mark.gpu
@pytest.mark.parametrize("njmax", [64, 256])
@pytest.mark.parametrize("cone", CONES)
def test_gpu_lifts_pot(cone, njmax):
  """The HIP path (graph replay, ctrl written per step on the device) passes unroll_test.py:38-56."""
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = _model(cone)
  key = mjw.find_keys(mjm, "lift_pot0")[0]
  traj = mjw.make_trajectory(mjm, mjw.find_keys(mjm, "lift_pot"))
  mjd = mjcf.MjData(mjm)
  mjcf.reset_data_keyframe(mjm, mjd, key)
  dev = torch.device("cuda:0")
  m = mjw.put_model(mjm, device=dev)
  nworld = 2  # two replicas: they must stay bitwise equal
  d = mjw.put_data(mjm, mjd, nworld=nworld, nconmax=64, njmax=njmax, device=dev, m=m)
  mjw.forward(m, d)
  d.qacc_warmstart.copy_(d.qacc)
  ctrl_dev = torch.as_tensor(traj.astype(np.float32), device=dev)
  torch.cuda.synchronize()
  cs = torch.cuda.Stream(device=dev)
  cs.wait_stream(torch.cuda.current_stream(dev))
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g, stream=cs):
    mjw.step(m, d)
  nefc_max = 0
  for i in range(len(traj)):
    d.ctrl.copy_(ctrl_dev[i].expand(nworld, -1))
    g.replay()
    if i % 50 == 0:
      nefc_max = max(nefc_max, int(d.nefc.max()))
  torch.cuda.synchronize()
  assert int(d.nacon[0]) <= d.naconmax and nefc_max <= njmax
  xpos = d.xpos.double().cpu().numpy()
  z = _check(xpos[0], mjm)
  assert torch.equal(d.qpos[0], d.qpos[1])
  print(f"{cone} njmax={njmax}: {z}, nefc max {nefc_max}")
