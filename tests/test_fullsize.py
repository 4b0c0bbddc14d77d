"""Size-independent properties at BASELINE.json's full sizes:
the headline config (humanoid, nworld=8192, Euler+CG, nconmax 24, njmax 64) and C4 (apollo,
nworld=4096, Newton) stepped with the benchmark's control noise.

* every world stays finite and within its row / contact capacity over the rollout;
* sharding invariance: the 8192 worlds stepped as two shards of 4096 with world_offset 0 / 4096
  (what each rank does in bench.py --gpus 2) are bitwise identical to the single 8192-world run;
* determinism: two runs of the same rollout are bitwise identical.
"""

import os

import numpy as np
import pytest

from tests.common import HUMANOID, ROOT, np_


def _setup(path, nworld, nconmax, njmax, solver=None, world_offset=0):
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model(path)
  if solver:
    mjw.override_model(mjm, [f"opt.solver={solver}"])
  mjd = mjcf.MjData(mjm)
  mjcf.reset_data_keyframe(mjm, mjd, 0)
  m = mjw.put_model(mjm, device="cuda")
  d = mjw.put_data(mjm, mjd, nworld=nworld, nconmax=nconmax, njmax=njmax, device="cuda", m=m)
  d.world_offset = world_offset
  center = torch.as_tensor(np.asarray(mjm.key_ctrl[0], dtype=np.float32), device="cuda")
  return mjm, m, d, center


def _roll(m, d, center, nstep, start=0):
  import mujoco_warp_amd as mjw

  for i in range(start, start + nstep):
    mjw.ctrl_noise(m, d, i, center=center)
    mjw.step(m, d)


@pytest.mark.gpu
def test_gpu_humanoid_fullsize_rollout_and_sharding():
  import torch

  mjm, m, d, c = _setup(HUMANOID, 8192, 24, 64, solver="CG")
  _roll(m, d, c, 100)
  torch.cuda.synchronize()
  q = np_(d.qpos)
  assert np.isfinite(q).all()
  assert int(d.nacon[0]) <= d.naconmax and int(d.nefc.max()) <= d.njmax
  assert float(d.qpos[:, 2].min()) > 0.0  # no world fell through the floor
  halves = []
  for off in (0, 4096):
    _, mh, dh, ch = _setup(HUMANOID, 4096, 24, 64, solver="CG", world_offset=off)
    _roll(mh, dh, ch, 100)
    halves.append(np_(dh.qpos))
  torch.cuda.synchronize()
  np.testing.assert_array_equal(np.concatenate(halves), q)


@pytest.mark.gpu
def test_gpu_apollo_fullsize_rollout_deterministic():
  import torch

  path = os.path.join(ROOT, "models", "apptronik_apollo", "scene_flat.xml")
  runs = []
  for _ in range(2):
    mjm, m, d, c = _setup(path, 4096, 16, 64)
    _roll(m, d, c, 100)
    torch.cuda.synchronize()
    runs.append((np_(d.qpos), np_(d.sensordata)))
  q, s = runs[0]
  assert np.isfinite(q).all() and np.isfinite(s).all()
  assert float(d.qpos[:, 2].min()) > 0.5  # the stand keyframe holds (position actuators)
  np.testing.assert_array_equal(runs[1][0], q)
  np.testing.assert_array_equal(runs[1][1], s)
