"""Measured errors of the sparse / flex path against the fp64 oracle (GPU box; prints JSON):
normwise qpos / qvel / qacc errors after 1 and 3 steps for `cloth` and `aloha_cloth`, and the CG cost
ratio.  Sets the bars of tests/test_cloth.py::test_gpu_cloth_rollout_parity_and_determinism."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
  import torch

  import mujoco_warp_amd as mjw
  from tests.test_cloth import _setup
  from tests.common import gpu_from_state, np_, oracle_from_state

  out = {}
  for which in ("cloth", "aloha"):
    mjm, qpos, qvel, ctrl, NJMAX, NCONMAX = _setup(which, 2, seed=4)
    m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=NJMAX, nconmax=NCONMAX)
    om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=NJMAX, nconmax=NCONMAX)
    for k in range(3):
      mjw.step(m, d)
      od.step()
      torch.cuda.synchronize()
      r = {}
      for f in ("qpos", "qvel", "qacc", "qacc_smooth"):
        g, o = np_(getattr(d, f)), getattr(od, f)
        r[f] = float((np.abs(g - o).max(axis=1) / (np.abs(o).max(axis=1) + 1e-30)).max())
      r["niter_gpu"] = np_(d.solver_niter).ravel().tolist()
      r["niter_oracle"] = od.solver_niter.ravel().tolist()
      out[f"{which}_step{k + 1}"] = r
  print(json.dumps(out, indent=1))


if __name__ == "__main__":
  main()
