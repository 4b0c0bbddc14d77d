"""Per-wave lifetimes of the humanoid step's two kernels (wave-log build, -DMJW_WAVELOG: no other
instrumentation, so the kernels keep their timing).

Each world's wave logs {start, end} s_memrealtime (100 MHz, chip-wide), its HW_ID / XCC_ID and, for the
dense kernel, its CG iterations (mjw_common.h WLOG_*).  For the last of `nsteps` steps this prints, per
kernel: the span (first start -> last end), the busy time summed over waves, the peak number of
concurrently resident waves (= resident slots), the slot efficiency busy / (span x slots), the time the
kernel spends with fewer than 90 % / 50 % of its slots busy (the tail), and the mean lifetime by
iteration count.
usage: python tools/wave_log.py [nworld] [nsteps] [CG|NEWTON] [out.json]
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PROF = os.path.join(ROOT, "mujoco_warp_amd", "libmjw_amd_wlog.so")
if not os.path.exists(PROF):
  from mujoco_warp_amd import build

  build.build(out=PROF, defines=("MJW_WAVELOG",))
os.environ["MJW_LIB_PATH"] = PROF

import torch  # noqa: E402

import mujoco_warp_amd as mjw  # noqa: E402
from mujoco_warp_amd import _lib, mjcf  # noqa: E402

TICK_NS = 10.0  # s_memrealtime: 100 MHz


def analyse(log, niter=None):
  t0, t1 = log[:, 0].astype(np.int64), log[:, 1].astype(np.int64)
  base = t0.min()
  t0, t1 = t0 - base, t1 - base
  life = (t1 - t0) * TICK_NS
  span = (t1.max()) * TICK_NS
  ev = np.concatenate([np.stack([t0, np.ones_like(t0)], 1), np.stack([t1, -np.ones_like(t1)], 1)])
  ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]  # ends before starts at equal times
  conc = np.cumsum(ev[:, 1])
  slots = int(conc.max())
  times = ev[:, 0]
  dt = np.diff(times) * TICK_NS
  c = conc[:-1]
  busy = float(life.sum())
  out = {
    "worlds": int(len(t0)), "span_us": span / 1e3, "busy_us_sum": busy / 1e3, "resident_slots_peak": slots,
    "slot_efficiency": busy / (span * slots) if span > 0 else None,
    "us_below_90pct_slots": float(dt[c < 0.9 * slots].sum()) / 1e3,
    "us_below_50pct_slots": float(dt[c < 0.5 * slots].sum()) / 1e3,
    "lifetime_us": {"mean": float(life.mean()) / 1e3, "p50": float(np.median(life)) / 1e3, "max": float(life.max()) / 1e3},
    "last_start_us": float(t0.max()) * TICK_NS / 1e3,
    "xcc_count": int(len(np.unique(log[:, 2] >> 32))),
  }
  if niter is not None:
    byit = {}
    for k in np.unique(niter):
      sel = niter == k
      byit[int(k)] = [int(sel.sum()), round(float(life[sel].mean()) / 1e3, 2)]
    out["lifetime_us_by_niter"] = byit
    out["niter_mean"] = float(niter.mean())
    out["niter_max"] = int(niter.max())
    # lifetime model: a + b * niter (least squares)
    A = np.stack([np.ones_like(niter, dtype=float), niter.astype(float)], 1)
    coef = np.linalg.lstsq(A, life / 1e3, rcond=None)[0]
    out["lifetime_fit_us"] = {"fixed": float(coef[0]), "per_iteration": float(coef[1])}
    # start order vs iteration count: were the long worlds started early?
    order = np.argsort(t0)
    q = len(order) // 4
    out["niter_mean_by_start_quartile"] = [float(niter[order[i * q:(i + 1) * q]].mean()) for i in range(4)]
  return out


def main():
  nworld = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
  nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
  solver = sys.argv[3] if len(sys.argv) > 3 else "CG"
  out_path = sys.argv[4] if len(sys.argv) > 4 else None
  mjm = mjcf.load_model(os.path.join(ROOT, "models", "humanoid.xml"))
  mjw.override_model(mjm, [f"opt.solver={solver}"])
  mjd = mjcf.MjData(mjm)
  mjcf.reset_data_keyframe(mjm, mjd, 0)
  m = mjw.put_model(mjm, device="cuda")
  d = mjw.put_data(mjm, mjd, nworld=nworld, nconmax=24, njmax=64, device="cuda", m=m)
  center = torch.as_tensor(np.asarray(mjm.key_ctrl[0], dtype=np.float32), device="cuda")
  L = _lib.lib()
  logs = {k: torch.zeros((nworld, 4), dtype=torch.int64, device="cuda") for k in ("fwd", "dense")}
  for k, fn in (("fwd", L.mjw_prof_wlog_fwd), ("dense", L.mjw_prof_wlog_dense)):
    fn.argtypes = [ctypes.c_void_p]
    _lib.check(fn(ctypes.c_void_p(logs[k].data_ptr())), "wlog")
  for i in range(nsteps):
    mjw.ctrl_noise(m, d, i, center=center)
    mjw.step(m, d)
  torch.cuda.synchronize()
  niter = d.solver_niter.cpu().numpy()
  res = {"nworld": nworld, "nsteps": nsteps, "solver": solver,
         "forward": analyse(logs["fwd"].cpu().numpy().view(np.uint64).astype(np.int64)),
         "dense": analyse(logs["dense"].cpu().numpy().view(np.uint64).astype(np.int64), niter)}
  for fn in (L.mjw_prof_wlog_fwd, L.mjw_prof_wlog_dense):
    fn(ctypes.c_void_p(0))
  s = json.dumps(res, indent=1)
  print(s)
  if out_path:
    with open(out_path, "w") as f:
      f.write(s)


if __name__ == "__main__":
  main()
