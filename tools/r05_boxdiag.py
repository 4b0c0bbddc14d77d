"""Diagnostic (GPU box): the BOXES sensor layout of tests/test_sensor_collision.py at z = 0.33 / 0.3 -- device
sensordata and box-box contacts next to the fp64 / fp32 oracles, to find where the fromto's first
multi-contact point differs."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mujoco_warp_amd as mjw  # noqa: E402
from tests.common import gpu_from_state, np_, oracle_from_state  # noqa: E402
from tests.test_sensor_collision import BOXES, _load  # noqa: E402

np.set_printoptions(precision=6, suppress=True, linewidth=220)
for z in (0.33, 0.3):
  mjm = _load(BOXES.format(z=z))
  nworld = 6
  rng = np.random.default_rng(4)
  qpos = np.tile(mjm.qpos0, (nworld, 1))
  q = qpos[1:, 3:7] + rng.normal(0, 0.05, (nworld - 1, 4))
  qpos[1:, 3:7] = q / np.linalg.norm(q, axis=1, keepdims=True)
  z0, u0 = np.zeros((nworld, mjm.nv)), np.zeros((nworld, mjm.nu))
  m, d = gpu_from_state(mjm, qpos, z0, u0)
  _, o64 = oracle_from_state(mjm, qpos, z0, u0)
  _, o32 = oracle_from_state(mjm, qpos, z0, u0, real_bits=32)
  mjw.forward(m, d)
  o64.forward()
  o32.forward()
  torch.cuda.synchronize()
  g = np_(d.sensordata)
  print("z", z, "fromto gpu - fp64 per world", np.abs(g[:, 4:10] - o64.sensordata[:, 4:10]).max(axis=1))
  print(" gpu  fromto", g[:, 4:10])
  print(" fp64 fromto", o64.sensordata[:, 4:10])
  n = int(d.nacon[0])
  wid = np_(d.contact.worldid)[:n]
  for w in range(nworld):
    sel = np.nonzero(wid == w)[0]
    print(" world", w, "gpu contacts pos/dist", [(np_(d.contact.pos[i]).round(5).tolist(), float(d.contact.dist[i])) for i in sel])
    nc = int(o64.ncon[w, 0])
    print("          oracle64 contacts", [(o64.con_pos[w].reshape(-1, 3)[i].round(5).tolist(), float(o64.con_dist[w][i])) for i in range(nc)])
