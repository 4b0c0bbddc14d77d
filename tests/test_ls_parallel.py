"""The parallel linesearch (solver.py:325-567, `opt.ls_parallel`, set by <numeric name="ls_parallel" data="1"/>,
io.py:188-190): each solver iteration takes the cheapest of `ls_iterations` step sizes log-spaced over
[ls_parallel_min_step, 1] instead of the exact iterative search.

CPU: the compiler reads the numeric; the oracle's parallel solve picks only log-spaced candidates, never
raises the cost, and with enough candidates lands near the iterative optimum.  GPU: the dense
(register-resident), generic (nv > 32) and sparse kernels against the oracle from the same rows.
"""

import numpy as np
import pytest

from tests.common import HUMANOID, gpu_from_state, np_, oracle_from_state, random_states


def test_compiler_reads_ls_parallel_numeric():
  from mujoco_warp_amd import mjcf

  xml = """<mujoco><custom><numeric name="ls_parallel" data="{v}"/><numeric name="contact_sensor_maxmatch" data="12"/></custom>
  <worldbody><body><freejoint/><geom size=".1"/></body></worldbody></mujoco>"""
  assert mjcf.load_model_from_string(xml.format(v=1)).opt.ls_parallel
  m0 = mjcf.load_model_from_string(xml.format(v=0))
  assert not m0.opt.ls_parallel and m0.opt.contact_sensor_maxmatch == 12


def _humanoid(ls_parallel, iterations=None):
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model(HUMANOID)
  mjm.opt.solver = 1
  mjm.opt.ls_parallel = ls_parallel
  if iterations is not None:
    mjm.opt.ls_iterations = iterations
  return mjm


def _contact_states(mjm, nworld, seed=0):
  qpos, qvel, ctrl = random_states(mjm, nworld, seed=seed, qpos_noise=0.1, qvel_noise=0.5)
  qpos[:, 2] -= 0.25  # into the floor: contact rows
  return qpos, qvel, ctrl


def test_oracle_parallel_step_is_a_log_spaced_candidate():
  """One CG iteration from qacc_smooth (warmstart off): qacc - qacc_smooth = alpha * search with
  search = -M^-1 grad(qacc_smooth); alpha must be one of the log-spaced candidates and the cheapest of them."""
  from tests.parity_models import efc_cost

  mjm = _humanoid(True)
  mjm.opt.iterations = 1
  mjm.opt.disableflags |= 512  # WARMSTART: start from qacc_smooth
  qpos, qvel, ctrl = _contact_states(mjm, 4)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  od.forward()
  n, nv = mjm.opt.ls_iterations, mjm.nv
  cands = np.exp(np.log(1e-6) + np.arange(n) * (-np.log(1e-6)) / (n - 1))
  for w in range(4):
    ne, nf, nefc = int(od.ne[w, 0]), int(od.nf[w, 0]), int(od.nefc[w, 0])
    assert nefc > 0
    J = od.efc_J[w].reshape(od.njmax, nv)[:nefc]
    D, aref, fl = od.efc_D[w, :nefc], od.efc_aref[w, :nefc], od.efc_frictionloss[w, :nefc]
    M = od.qM[w].reshape(nv, nv)
    q0 = od.qacc_smooth[w]
    jar = J @ q0 - aref
    f = np.where(jar < 0, -D * jar, 0.0)
    f[:ne] = -D[:ne] * jar[:ne]
    for r in range(ne, ne + nf):
      rf = fl[r] / D[r]
      f[r] = fl[r] if jar[r] <= -rf else (-fl[r] if jar[r] >= rf else -D[r] * jar[r])
    search = -np.linalg.solve(M, -(J.T @ f))
    dq = od.qacc[w] - q0
    alpha = float(dq @ search / (search @ search))
    np.testing.assert_allclose(dq, alpha * search, rtol=1e-6, atol=1e-9)
    k = int(np.argmin(np.abs(cands - alpha)))
    assert abs(cands[k] - alpha) <= 1e-9 * cands[k], (alpha, cands[k])
    costs = [efc_cost(J, D, aref, od.efc_type[w, :nefc], M, q0, q0 + a * search, fl=fl, nf=nf) for a in cands]
    assert k == int(np.argmin(costs))


def test_oracle_parallel_close_to_iterative_optimum():
  """Many log-spaced candidates and many iterations: the parallel solve reaches the iterative solve's cost
  to 1e-3 relative (the reference's own bar for CG is 2.5 %, solver_test.py:308-322)."""
  from tests.parity_models import efc_cost

  res = {}
  for par in (False, True):
    mjm = _humanoid(par, iterations=200)
    mjm.opt.iterations = 200
    qpos, qvel, ctrl = _contact_states(mjm, 3, seed=1)
    _, od = oracle_from_state(mjm, qpos, qvel, ctrl)
    od.forward()
    res[par] = od
  a, b = res[False], res[True]
  nv = a.qacc.shape[1]
  for w in range(3):
    n = int(a.nefc[w, 0])
    args = (a.efc_J[w].reshape(a.njmax, nv)[:n], a.efc_D[w, :n], a.efc_aref[w, :n], a.efc_type[w, :n], a.qM[w].reshape(nv, nv),
            a.qacc_smooth[w])
    c_it = efc_cost(*args, a.qacc[w], fl=a.efc_frictionloss[w, :n])
    c_par = efc_cost(*args, b.qacc[w], fl=a.efc_frictionloss[w, :n])
    c0 = efc_cost(*args, a.qacc_smooth[w], fl=a.efc_frictionloss[w, :n])
    assert c_par <= c0 + 1e-12
    assert (c_par - c_it) <= 1e-3 * abs(c0 - c_it) + 1e-12, (w, c_it, c_par, c0)


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["dense", "generic", "sparse"])
def test_gpu_ls_parallel_matches_oracle(path):
  """One forward + solve on the device against the oracle with ls_parallel on: the same solver cost (fp64,
  from the oracle's rows) to 1e-5 relative excess and qacc at the solver bar (solver_test.py:32)."""
  import torch

  import mujoco_warp_amd as mjw
  from tests.parity_models import efc_cost

  mjm = _humanoid(True)
  njmax = 64
  if path == "generic":
    njmax = 96  # njmax > 64: the generic LDS-solver kernel
  if path == "sparse":
    mjm.opt.jacobian = 1
  qpos, qvel, ctrl = _contact_states(mjm, 8, seed=2)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=24)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=njmax, nconmax=24)
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  nv = mjm.nv
  for w in range(8):
    n = int(od.nefc[w, 0])
    assert int(d.nefc[w]) == n and n > 0
    args = (od.efc_J[w].reshape(njmax, nv)[:n], od.efc_D[w, :n], od.efc_aref[w, :n], od.efc_type[w, :n], od.qM[w].reshape(nv, nv),
            od.qacc_smooth[w])
    c_or = efc_cost(*args, od.qacc[w], fl=od.efc_frictionloss[w, :n])
    c_gpu = efc_cost(*args, np_(d.qacc[w]), fl=od.efc_frictionloss[w, :n])
    assert (c_gpu - c_or) <= 1e-5 * abs(c_or), (w, c_gpu, c_or)
  err = np.abs(np_(d.qacc) - od.qacc).max(axis=1) / (np.abs(od.qacc).max(axis=1) + 1e-9)
  assert err.max() < 5e-3, err
