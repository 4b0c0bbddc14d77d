"""Probe: one 8192-world batch on one stream vs two 4096-world halves on two streams (tail overlap)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mujoco_warp_amd as mjw  # noqa: E402
from mujoco_warp_amd import mjcf  # noqa: E402

mjm = mjcf.load_model(os.path.join(ROOT, "models", "humanoid.xml"))
mjw.override_model(mjm, ["opt.solver=CG"])
mjd = mjcf.MjData(mjm)
mjcf.reset_data_keyframe(mjm, mjd, 0)
m = mjw.put_model(mjm, device="cuda")
center = torch.as_tensor(np.asarray(mjm.key_ctrl[0], dtype=np.float32), device="cuda")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
K = int(sys.argv[2]) if len(sys.argv) > 2 else 300
nsplit = int(sys.argv[3]) if len(sys.argv) > 3 else 2


def make(n, off):
  d = mjw.put_data(mjm, mjd, nworld=n, nconmax=24, njmax=64, device="cuda", m=m)
  d.world_offset = off
  return d


def run(datas, streams, k0, k):
  for i in range(k0, k0 + k):
    for d, s in zip(datas, streams):
      with torch.cuda.stream(s):
        mjw.ctrl_noise(m, d, i, center=center)
        mjw.step(m, d)


for label, parts, nstreams in (("one batch, one stream", 1, 1), (f"{nsplit} parts, {nsplit} streams", nsplit, nsplit),
                               (f"{nsplit} parts, one stream", nsplit, 1)):
  per = N // parts
  datas = [make(per, i * per) for i in range(parts)]
  streams = [torch.cuda.Stream() for _ in range(nstreams)]
  streams = [streams[i % nstreams] for i in range(parts)]
  run(datas, streams, 0, 20)
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  run(datas, streams, 20, K)
  torch.cuda.synchronize()
  dt = time.perf_counter() - t0
  print(f"{label:28s}: {N * K / dt / 1e6:.3f} M env-steps/s  ({dt / K * 1e3:.4f} ms/step)", flush=True)
