"""Per-stage device time of the step (stage kernels launched separately, HIP events)."""
import os, sys, json
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mujoco_warp_amd as mjw
from mujoco_warp_amd import mjcf

nworld = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
solver = sys.argv[3] if len(sys.argv) > 3 else "CG"
mjm = mjcf.load_model(os.path.join(ROOT, "models", "humanoid.xml"))
mjw.override_model(mjm, [f"opt.solver={solver}"])
mjd = mjcf.MjData(mjm); mjcf.reset_data_keyframe(mjm, mjd, 0)
m = mjw.put_model(mjm, device="cuda")
d = mjw.put_data(mjm, mjd, nworld=nworld, nconmax=24, njmax=64, device="cuda", m=m)
center = torch.zeros(mjm.nu, device="cuda")
stages = [("fwd_position", mjw.fwd_position), ("fwd_velocity", mjw.fwd_velocity), ("fwd_actuation", mjw.fwd_actuation),
          ("fwd_acceleration", mjw.fwd_acceleration), ("solve", mjw.solve), ("euler", mjw.euler)]
acc = {n: 0.0 for n, _ in stages}
fused = 0.0
cnt = 0
for i in range(nsteps):
  mjw.ctrl_noise(m, d, i, center=center)
  if i % 50 == 49:
    # measure: staged on a copy of the state, then fused
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(stages) + 1)]
    q0, v0, w0, c0, t0 = d.qpos.clone(), d.qvel.clone(), d.qacc_warmstart.clone(), d.ctrl.clone(), d.time.clone()
    ev[0].record()
    for k, (n, f) in enumerate(stages):
      f(m, d); ev[k + 1].record()
    torch.cuda.synchronize()
    for k, (n, f) in enumerate(stages):
      acc[n] += ev[k].elapsed_time(ev[k + 1])
    d.qpos.copy_(q0); d.qvel.copy_(v0); d.qacc_warmstart.copy_(w0); d.ctrl.copy_(c0); d.time.copy_(t0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); mjw.step(m, d); e1.record(); torch.cuda.synchronize()
    fused += e0.elapsed_time(e1); cnt += 1
    print(f"step {i}: nefc_mean {d.nefc.float().mean():.1f} ncon/world {int(d.nacon[0])/nworld:.2f} niter_mean {d.solver_niter.float().mean():.1f} niter_max {int(d.solver_niter.max())}", flush=True)
  else:
    mjw.step(m, d)
torch.cuda.synchronize()
print(json.dumps({"nworld": nworld, "solver": solver, "fused_ms": fused / cnt, **{k: v / cnt for k, v in acc.items()}}))
