import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import mujoco_warp_amd as mjw
from tests.common import franka_model, franka_states, gpu_from_state, oracle_from_state, np_
mjm = franka_model()
qpos, qvel, ctrl = franka_states(mjm, 16, seed=22)
m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=16, nconmax=4)
_, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=16, nconmax=8)
mjw.forward(m, d); torch.cuda.synchronize(); od.forward()
print("gpu ne", np_(d.ne).astype(int).tolist()); print("orc ne", od.ne[:, 0].tolist())
print("gpu nefc", np_(d.nefc).astype(int).tolist()); print("orc nefc", od.nefc[:, 0].tolist())
print("gpu nacon", int(d.nacon[0]), "orc ncon", od.ncon[:, 0].tolist())
print("gpu types", d.efc.type[:4, :6].cpu().numpy().tolist()); print("orc types", od.efc_type[:4, :6].tolist())
print("eq_active", d.eq_active.cpu().numpy().ravel().tolist(), "neq", m.neq)
