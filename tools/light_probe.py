"""Debug probe (GPU box): light / camera frames of the sparse path against the oracle on the cloth scene."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests.cloth_common import cloth_model, cloth_states  # noqa: E402
from tests.common import gpu_from_state, np_, oracle_from_state  # noqa: E402


def main():
  import torch

  import mujoco_warp_amd as mjw

  mjm = cloth_model()
  q, v, c = cloth_states(mjm, 2, seed=1)
  m, d = gpu_from_state(mjm, q, v, c, njmax=3000, nconmax=200)
  om, od = oracle_from_state(mjm, q, v, c, njmax=3000, nconmax=200)
  mjw.fwd_position(m, d)
  od.fwd_position()
  torch.cuda.synchronize()
  np.set_printoptions(precision=5, suppress=True)
  print("light modes", mjm.light_mode, "body", mjm.light_bodyid, "target", mjm.light_targetbodyid)
  print("gpu light_xpos", np_(d.light_xpos)[0].ravel(), "\noracle", od.light_xpos[0])
  print("gpu light_xdir", np_(d.light_xdir)[0].ravel(), "\noracle", od.light_xdir[0])
  print("gpu xpos[0:2]", np_(d.xpos)[0, :2].ravel(), "xquat[0:2]", np_(d.xquat)[0, :2].ravel())
  print("gpu subtree_com[0:2]", np_(d.subtree_com)[0, :2].ravel(), "oracle", od.subtree_com[0, :6])
  print("cam gpu", np_(d.cam_xpos)[0].ravel(), "oracle", od.cam_xpos[0])


if __name__ == "__main__":
  main()
