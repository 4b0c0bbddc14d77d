"""Per-step solver iteration / constraint-count distribution of a bench config (driver window: 5 warm-up
+ 20 timed steps by default), to see whether the dense kernel's time follows the mean or the slowest
worlds.  usage: python tools/r05_niter.py [model] [steps]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402
import mujoco_warp_amd as mjw  # noqa: E402
from mujoco_warp_amd import mjcf  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "humanoid"
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 25
cfg = bench.MODELS[model]
sys.argv = ["bench.py", "--model", model]
a = bench.parse()
mjm = mjcf.load_model(os.path.join(bench.ROOT, cfg["path"]))
if a.solver is not None:
  mjw.override_model(mjm, [f"opt.solver={a.solver}"])
mjd = mjcf.MjData(mjm)
center = None
if cfg["key"] is not None:
  mjcf.reset_data_keyframe(mjm, mjd, cfg["key"])
  center = torch.as_tensor(np.asarray(mjm.key_ctrl[cfg["key"]], dtype=np.float32), device="cuda")
m = mjw.put_model(mjm, device="cuda")
d = mjw.put_data(mjm, mjd, nworld=a.nworld, nconmax=a.nconmax, njmax=a.njmax, device="cuda", m=m)
out = []
prev_it = None
for i in range(nsteps):
  mjw.ctrl_noise(m, d, i, center=center)
  e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  e0.record()
  mjw.step(m, d)
  e1.record()
  torch.cuda.synchronize()
  it = d.solver_niter.cpu().numpy().astype(np.int64)
  nefc = d.nefc.cpu().numpy().astype(np.int64)
  r = {"step": i, "ms": round(e0.elapsed_time(e1), 4), "niter_mean": round(float(it.mean()), 2), "niter_p50": int(np.percentile(it, 50)),
       "niter_p99": int(np.percentile(it, 99)), "niter_max": int(it.max()), "niter_sum": int(it.sum()),
       "nefc_mean": round(float(nefc.mean()), 2), "nefc_max": int(nefc.max()), "nworld_gt32rows": int((nefc > 32).sum())}
  if getattr(d.efc, "J_rownnz", None) is not None and d.efc.J_rownnz.numel() >= nefc.size and m.nv > 64:
    nnz = d.efc.J_rownnz.reshape(nefc.size, -1).cpu().numpy().astype(np.int64)
    mask = np.arange(nnz.shape[1])[None, :] < nefc[:, None]
    r["Jnnz_per_world_mean"] = round(float((nnz * mask).sum(1).mean()), 1)
  # how well the previous step's iterations and this step's rows predict this step's iterations (the
  # dense kernel's longest-first order uses the former)
  if prev_it is not None and it.std() > 0 and prev_it.std() > 0:
    r["corr_prev_niter"] = round(float(np.corrcoef(prev_it, it)[0, 1]), 3)
  if it.std() > 0 and nefc.std() > 0:
    r["corr_nefc"] = round(float(np.corrcoef(nefc, it)[0, 1]), 3)
  prev_it = it
  hist = np.bincount(np.minimum(it, 60), minlength=61)
  r["niter_hist"] = hist.tolist()
  out.append(r)
  print(json.dumps({k: v for k, v in r.items() if k != "niter_hist"}), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open(f"gpurun_out/niter_{model}.json", "w"))
