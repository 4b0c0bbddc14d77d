"""hipGraph capture and replay of mjw.step (reference forward_test.py:272-288 graph smoke test,
benchmark.py:123-155 capture-once / replay-per-step harness).

The step is captured once on a side stream; each replay is preceded by the (uncaptured) control-noise
launch, with and without a host synchronisation in between, and must equal eager stepping bitwise."""

import os

import numpy as np
import pytest

from tests.common import HUMANOID, ROOT, np_


def _setup(path, nworld, nconmax, njmax, solver=None, key=0):
  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model(path)
  if solver:
    mjw.override_model(mjm, [f"opt.solver={solver}"])
  mjd = mjcf.MjData(mjm)
  if key is not None:
    mjcf.reset_data_keyframe(mjm, mjd, key)
  m = mjw.put_model(mjm, device="cuda")
  d = mjw.put_data(mjm, mjd, nworld=nworld, nconmax=nconmax, njmax=njmax, device="cuda", m=m)
  return m, d


def _graph_vs_eager(path, nworld, nconmax, njmax, solver=None, key=0, nstep=6, sync=False):
  import torch

  import mujoco_warp_amd as mjw

  m, d = _setup(path, nworld, nconmax, njmax, solver, key)
  mjw.ctrl_noise(m, d, 0)
  mjw.step(m, d)
  torch.cuda.synchronize()
  q0 = np_(d.qpos)
  s = torch.cuda.Stream()
  s.wait_stream(torch.cuda.current_stream())
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g, stream=s):
    mjw.step(m, d)
  torch.cuda.synchronize()
  np.testing.assert_array_equal(np_(d.qpos), q0)  # capture records, it does not run
  for i in range(1, nstep):
    mjw.ctrl_noise(m, d, i)
    if sync:
      torch.cuda.synchronize()
    g.replay()
  torch.cuda.synchronize()
  m2, d2 = _setup(path, nworld, nconmax, njmax, solver, key)
  for i in range(nstep):
    mjw.ctrl_noise(m2, d2, i)
    mjw.step(m2, d2)
  torch.cuda.synchronize()
  assert not np.array_equal(np_(d.qpos), q0)
  np.testing.assert_array_equal(np_(d.qpos), np_(d2.qpos))
  np.testing.assert_array_equal(np_(d.qvel), np_(d2.qvel))
  assert int(d.nacon[0]) == int(d2.nacon[0])


@pytest.mark.gpu
@pytest.mark.parametrize("sync", [False, True])
def test_gpu_graph_replay_humanoid(sync):
  _graph_vs_eager(HUMANOID, 301, 24, 64, solver="CG", sync=sync)


@pytest.mark.gpu
def test_gpu_graph_replay_apollo_ccd_sensors():
  """Newton, box-box CCD pre-pass and the sensor kernel inside the captured step."""
  _graph_vs_eager(os.path.join(ROOT, "models", "apptronik_apollo", "scene_flat.xml"), 64, 16, 64, sync=True)


@pytest.mark.gpu
def test_gpu_graph_replay_cloth_sparse():
  """The sparse / flex pipeline (several launches per step) inside the captured step."""
  _graph_vs_eager(os.path.join(ROOT, "models", "cloth", "scene.xml"), 4, 200, 3000, key=None, nstep=3, sync=True)
