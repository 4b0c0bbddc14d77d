"""Shape of the sparse solver's row and column work on a bench config (aloha_cloth by default): after
`warm` steps, the per-world constraint rows, J non-zeros per row, and the entries per dof column of the
transposed index (efc_JT_adr, built by solve_kernel<0>) -- mean, max and the share of the J'f pass's
entries held by the heaviest columns -- plus what each thread of a 256-thread world walks under the
strided column assignment (thread t: columns t, t + 256, ...).
usage: python tools/r06_jt_probe.py [model] [nworld] [warm]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import mujoco_warp_amd as mjw  # noqa: E402
from bench import MODELS  # noqa: E402
from mujoco_warp_amd import mjcf  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "aloha_cloth"
nworld = int(sys.argv[2]) if len(sys.argv) > 2 else 64
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 25
cfg = MODELS[model]
mjm = mjcf.load_model(os.path.join(ROOT, cfg["path"]))
mjd = mjcf.MjData(mjm)
if cfg["key"] is not None:
  mjcf.reset_data_keyframe(mjm, mjd, cfg["key"])
m = mjw.put_model(mjm, device="cuda")
d = mjw.put_data(mjm, mjd, nworld=nworld, nconmax=cfg["nconmax"], njmax=cfg["njmax"], device="cuda", m=m)
center = None if cfg["key"] is None else torch.as_tensor(mjm.key_ctrl[cfg["key"]], dtype=torch.float32, device="cuda")
for i in range(warm):
  mjw.ctrl_noise(m, d, i, center=center)
  mjw.step(m, d)
torch.cuda.synchronize()
nv = mjm.nv
adr = d.efc.JT_adr.reshape(nworld, nv + 1).cpu().numpy().astype(np.int64)
cnt = np.diff(adr, axis=1)
nefc = d.nefc.reshape(-1).cpu().numpy()
nnz = d.efc.J_rownnz.reshape(nworld, -1).cpu().numpy()
rows_nnz = [nnz[w, : min(nefc[w], nnz.shape[1])] for w in range(nworld)]
per_thread = np.zeros((nworld, 256), np.int64)
for t in range(256):
  per_thread[:, t] = cnt[:, t::256].sum(1)
top = np.sort(cnt, axis=1)[:, ::-1]
out = {
  "model": model, "nworld": nworld, "warm": warm, "nv": nv,
  "nefc_mean": float(nefc.mean()),
  "row_nnz_mean": float(np.mean([r.mean() for r in rows_nnz if len(r)])),
  "row_nnz_max": int(max(r.max() for r in rows_nnz if len(r))),
  "entries_mean": float(cnt.sum(1).mean()),
  "col_entries_mean": float(cnt.mean()),
  "col_entries_max": int(cnt.max()),
  "top16_col_entries_mean": [int(x) for x in top[:, :16].mean(0)],
  "top16_share": float(top[:, :16].sum() / max(cnt.sum(), 1)),
  "thread_entries_mean": float(per_thread.mean()),
  "thread_entries_max_mean": float(per_thread.max(1).mean()),
  "heaviest_cols": [int(x) for x in np.argsort(-cnt.sum(0))[:16]],
}
print(json.dumps(out, indent=1))
