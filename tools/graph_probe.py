"""hipGraph capture probe: eager steps vs captured-step replays on the humanoid (prints max |dq|)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mujoco_warp_amd as mjw  # noqa: E402
from mujoco_warp_amd import mjcf  # noqa: E402


def setup(nworld):
  mjm = mjcf.load_model(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "models", "humanoid.xml"))
  mjw.override_model(mjm, ["opt.solver=CG"])
  mjd = mjcf.MjData(mjm)
  mjcf.reset_data_keyframe(mjm, mjd, 0)
  m = mjw.put_model(mjm, device="cuda")
  d = mjw.put_data(mjm, mjd, nworld=nworld, nconmax=24, njmax=64, device="cuda", m=m)
  return m, d


n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
sync_between = len(sys.argv) > 2 and sys.argv[2] == "sync"
m, d = setup(n)
for i in range(2):
  mjw.ctrl_noise(m, d, i)
  mjw.step(m, d)
torch.cuda.synchronize()
q_before = d.qpos.clone()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
  mjw.step(m, d)
torch.cuda.synchronize()
print("capture changed qpos:", float((d.qpos - q_before).abs().max()))
for i in range(2, 7):
  mjw.ctrl_noise(m, d, i)
  if sync_between:
    torch.cuda.synchronize()
  g.replay()
torch.cuda.synchronize()
print("replays moved qpos:", float((d.qpos - q_before).abs().max()))
m2, d2 = setup(n)
for i in range(7):
  mjw.ctrl_noise(m2, d2, i)
  mjw.step(m2, d2)
torch.cuda.synchronize()
print("graph vs eager max |dq|:", float((d.qpos - d2.qpos).abs().max()))
print("graph vs eager max |dctrl|:", float((d.ctrl - d2.ctrl).abs().max()))
