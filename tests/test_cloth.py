"""Sparse / flex pipeline (csrc/mjw_sparse.hip) on the reference's cloth benchmark scene
(`benchmarks/cloth/scene.xml`: a 30x30 dim-2 flexcomp towel over a jointless mannequin; nv = 2706,
jacobian="sparse", CG) -- SURVEY.md §8(f) f3.

Reference functions covered: flex kinematics / edge lengths and Jacobians (smooth.py:227-355), the
flex passive forces (passive.py:566-726), flex equality rows (constraint.py:1113-1313), flex-vertex /
flex-element collisions (collision_flex.py:261-529), sparse qM and its L'DL factor
(smooth.py:825-852, 1003-1064), sparse efc_J rows and the CG solve (solver.py).

CPU: compiler sizes, oracle invariants (edge rows vanish at rest, edge Jacobians are time
derivatives, a lowered towel touches the mannequin and stays finite).  GPU (`-m gpu`): every stage
against the fp64 oracle, the CG cost of the device solution evaluated in fp64 against the oracle's
optimum, short rollouts, and determinism across copies of one world.
"""

import numpy as np
import pytest

from tests.cloth_common import (aloha_model, aloha_states, cloth_model, cloth_states, dense_J, dense_qM, flex_vert_adr, gpu_contacts,
                                 oracle_contacts)
from tests.common import assert_close, gpu_from_state, np_, oracle_from_state

NJMAX, NCONMAX = 3000, 200
# aloha_cloth: the towel lies on the table, 2 contacts per triangle (3364) and ~16k rows -- sized so
# that nothing overflows (the reference config's 920 / 6300 would cut both)
ALOHA_NJMAX, ALOHA_NCONMAX = 16384, 4096


def _setup(which, nworld, seed):
  if which == "aloha":
    mjm = aloha_model()
    return (mjm,) + aloha_states(mjm, nworld, seed=seed) + (ALOHA_NJMAX, ALOHA_NCONMAX)
  mjm = cloth_model()
  return (mjm,) + cloth_states(mjm, nworld, seed=seed) + (NJMAX, NCONMAX)


def _normwise(name, got, want, tol):
  e = np.abs(got - want).max(axis=1) / (np.abs(want).max(axis=1) + 1e-30)
  assert e.max() <= tol, f"{name}: normwise error {e.max():.3e} > {tol}"


@pytest.fixture(scope="module")
def mjm():
  return cloth_model()


# ---- CPU ------------------------------------------------------------------------------------------
def test_cloth_compiles_to_the_reference_sizes(mjm):
  # 30 x 30 grid: 900 vertices, 29*30*2 + 29*29 edges, 2*29*29 triangles; one slide-xyz body per
  # vertex plus the mannequin's free joint
  assert (mjm.nflex, mjm.nflexvert, mjm.nflexedge, mjm.nflexelem) == (1, 900, 2581, 1682)
  assert mjm.nv == 900 * 3 + 6 and mjm.nq == 900 * 3 + 7
  assert int(mjm.opt.jacobian) == 1 and int(mjm.opt.solver) == 1
  assert (flex_vert_adr(mjm)[:, 0] >= 0).all()


def test_put_model_selects_the_sparse_path(mjm):
  import mujoco_warp_amd as mjw

  m = mjw.put_model(mjm, device="cpu")
  assert m.is_sparse and m.ntree == 1 + 900 and m.nM == int(np.asarray(mjm.M_rownnz).sum())
  assert m.nflexinc > 0 and m.nplane == 1
  # an interior vertex is touched by 6 triangles (plus bending stencils)
  assert np.diff(m.flexvert_incadr.numpy()).max() >= 6


def test_oracle_edge_rows_vanish_at_rest(mjm):
  om, od = oracle_from_state(mjm, mjm.qpos0[None], np.zeros((1, mjm.nv)), np.zeros((1, mjm.nu)), njmax=NJMAX, nconmax=NCONMAX)
  od.fwd_position()
  np.testing.assert_allclose(od.flexedge_length[0], mjm.flexedge_length0, rtol=1e-12, atol=1e-12)
  ne = int(od.ne[0, 0])
  assert ne == mjm.nflexedge
  np.testing.assert_allclose(od.efc_pos[0, :ne], 0.0, atol=1e-12)


def test_oracle_edge_jacobian_is_the_time_derivative(mjm):
  qpos, qvel, ctrl = cloth_states(mjm, 1, seed=3, dz=0.0)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=NJMAX, nconmax=NCONMAX)
  od.fwd_position()
  L0 = od.flexedge_length[0].copy()
  h = 1e-7
  q2 = qpos.copy()
  q2[0, 7:] += h * qvel[0, 6:]  # slide joints: qpos advances by qvel
  om2, od2 = oracle_from_state(mjm, q2, qvel, ctrl, njmax=NJMAX, nconmax=NCONMAX)
  od2.fwd_position()
  fd = (od2.flexedge_length[0] - L0) / h
  ne = int(od.ne[0, 0])
  J = od.efc_J[0].reshape(NJMAX, mjm.nv)[:ne]
  np.testing.assert_allclose(J @ qvel[0], fd, atol=2e-6)
  np.testing.assert_allclose(od.efc_vel[0, :ne], J @ qvel[0], atol=1e-12)


def test_oracle_lowered_towel_touches_the_mannequin(mjm):
  qpos, qvel, ctrl = cloth_states(mjm, 1, seed=0)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=NJMAX, nconmax=NCONMAX)
  for _ in range(3):
    od.step()
  assert np.isfinite(od.qpos).all() and np.isfinite(od.qvel).all()
  cons = oracle_contacts(od, 0)
  assert sum(c["flex"][1] == 0 for c in cons) > 0  # flex-element contacts with the head
  assert int(od.nefc[0, 0]) > mjm.nflexedge


# ---- GPU ------------------------------------------------------------------------------------------
def _efc_cost(J, D, aref, types_, M, qacc_smooth, qacc):
  """fp64 primal cost of qacc (solver.py: Gauss term + quadratic rows; equality rows always,
  limits / contacts only while J qacc - aref < 0)."""
  dq = qacc - qacc_smooth
  jar = J @ qacc - aref
  active = (types_ == 0) | (jar < 0)
  return 0.5 * dq @ M @ dq + 0.5 * np.sum(D * jar * jar * active)


def _match_rows(d, od, w, gc, oc):
  """(gpu row, oracle row) pairs: equality / friction / limit rows by index, contact rows through
  the matched contacts (gc / oc are the key-sorted contact lists of the two sides)."""
  pairs = [(r, r) for r in range(int(od.ne[w, 0]) + int(od.nf[w, 0]) + int(od.nl[w, 0]))]
  for a, b in zip(gc, oc):
    ga = d.contact.efc_address[a["slot"]].cpu().numpy()
    oa = od.con_efc_address[w, 10 * b["slot"] : 10 * b["slot"] + 10]
    for k in range(len(ga)):
      if ga[k] >= 0 and oa[k] >= 0:
        pairs.append((int(ga[k]), int(oa[k])))
  return pairs


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["cloth", "aloha"])
def test_gpu_cloth_position_stage_parity(which):
  import torch

  import mujoco_warp_amd as mjw

  nworld = 2
  mjm, qpos, qvel, ctrl, NJMAX, NCONMAX = _setup(which, nworld, seed=1)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=NJMAX, nconmax=NCONMAX)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=NJMAX, nconmax=NCONMAX)
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()
  od.fwd_position()
  nv = mjm.nv
  for w in range(nworld):
    for f in ("xpos", "geom_xpos", "flexvert_xpos", "flexedge_length"):
      assert_close(f"{f}[w{w}]", np_(getattr(d, f)[w]).ravel(), getattr(od, f)[w].ravel(), rtol=1e-5, atol=1e-6)
    assert_close(f"flexedge_J[w{w}]", np_(d.flexedge_J[w]).ravel(), od.flexedge_J[w], rtol=1e-3, atol=5e-6)
    assert_close(f"subtree_com[w{w}]", np_(d.subtree_com[w]).ravel(), od.subtree_com[w], rtol=1e-4, atol=1e-5)
    assert_close(f"qM[w{w}]", dense_qM(mjm, np_(d.qM[w])), od.qM[w].reshape(nv, nv), rtol=1e-5, atol=2e-6)
    assert (int(d.ne[w]), int(d.nf[w]), int(d.nl[w]), int(d.nefc[w])) == (int(od.ne[w, 0]), int(od.nf[w, 0]), int(od.nl[w, 0]), int(od.nefc[w, 0]))
    gc, oc = gpu_contacts(d, w), oracle_contacts(od, w)
    assert len(gc) == len(oc) and any(c["flex"][1] == 0 for c in gc)
    assert int(od.ncon[w, 0]) <= NCONMAX
    for a, b in zip(gc, oc):
      assert (a["geom"], a["flex"], a["vert"], a["dim"]) == (b["geom"], b["flex"], b["vert"], b["dim"])
      assert abs(a["dist"] - b["dist"]) < 2e-6
      assert_close(f"con_pos[w{w}]", a["pos"], b["pos"], rtol=1e-5, atol=2e-6)
      assert_close(f"con_frame[w{w}]", a["frame"], b["frame"], rtol=1e-4, atol=2e-5)
    n = int(od.nefc[w, 0])
    Jg, Jo = dense_J(d, w, n, nv), od.efc_J[w].reshape(NJMAX, nv)[:n]
    pairs = _match_rows(d, od, w, gc, oc)
    assert len(pairs) == n
    g_idx, o_idx = np.array([p[0] for p in pairs]), np.array([p[1] for p in pairs])
    np.testing.assert_array_equal(d.efc.type[w].cpu().numpy()[g_idx], od.efc_type[w][o_idx])
    assert_close(f"J[w{w}]", Jg[g_idx], Jo[o_idx], rtol=1e-4, atol=2e-5)
    # aref = -k imp pos - b vel: the mannequin rests on the floor at dist ~0, and solref .003 gives
    # k ~ 1e4 / s^2, so fp32 distance rounding (~1e-7) alone moves aref by ~1e-3
    for f, rt, at in (("pos", 1e-4, 2e-6), ("D", 1e-4, 1e-6), ("vel", 1e-4, 1e-6), ("aref", 2e-3, 2e-3)):
      assert_close(f"efc_{f}[w{w}]", np_(getattr(d.efc, f)[w])[g_idx], getattr(od, "efc_" + f)[w][o_idx], rtol=rt, atol=at)


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["cloth", "aloha"])
def test_gpu_cloth_smooth_forces_and_cg_cost(which):
  """qfrc_passive / qacc_smooth to fp32 accuracy; the device CG solution's fp64 cost within the
  reference's CG tolerance of the oracle optimum (solver_test.py:317 uses 1.025x)."""
  import torch

  import mujoco_warp_amd as mjw

  nworld = 2
  mjm, qpos, qvel, ctrl, NJMAX, NCONMAX = _setup(which, nworld, seed=2)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=NJMAX, nconmax=NCONMAX)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=NJMAX, nconmax=NCONMAX)
  mjw.forward(m, d)
  torch.cuda.synchronize()
  od.forward()
  nv = mjm.nv
  # vertex masses are 1.1e-4 kg, so qacc_smooth = f / m amplifies fp32 force rounding ~1e4x
  assert_close("qfrc_passive", np_(d.qfrc_passive), od.qfrc_passive, rtol=1e-3, atol=5e-7)
  assert_close("qfrc_bias", np_(d.qfrc_bias), od.qfrc_bias, rtol=1e-5, atol=1e-4)
  assert_close("qacc_smooth", np_(d.qacc_smooth), od.qacc_smooth, rtol=1e-2, atol=5e-3)
  # normwise per world, the bar that does not depend on near-zero components: measured 1.1e-5 (cloth)
  # and 5.7e-7 (aloha_cloth) after one step, profiles/r02_cloth_parity_probe.json
  _normwise("qacc_smooth", np_(d.qacc_smooth), od.qacc_smooth, 1e-4)
  for w in range(nworld):
    n = int(od.nefc[w, 0])
    J = od.efc_J[w].reshape(NJMAX, nv)[:n]
    M = od.qM[w].reshape(nv, nv)
    args = (J, od.efc_D[w, :n], od.efc_aref[w, :n], od.efc_type[w, :n], M, od.qacc_smooth[w])
    c_or = _efc_cost(*args, od.qacc[w])
    c_gpu = _efc_cost(*args, np_(d.qacc[w]))
    c_0 = _efc_cost(*args, od.qacc_smooth[w])
    assert c_or <= c_0
    assert c_gpu <= c_or + 0.025 * abs(c_or) + 1e-9, (w, c_gpu, c_or, c_0)


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["cloth", "aloha"])
def test_gpu_cloth_rollout_parity_and_determinism(which):
  import torch

  import mujoco_warp_amd as mjw

  nworld = 2
  mjm, qpos, qvel, ctrl, NJMAX, NCONMAX = _setup(which, nworld, seed=4)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=NJMAX, nconmax=NCONMAX)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=NJMAX, nconmax=NCONMAX)
  for _ in range(3):
    mjw.step(m, d)
    od.step()
  torch.cuda.synchronize()
  # three fp32 CG solves of 2700 dofs / ~3-15k rows each stop at slightly different iterates than the
  # fp64 oracle's (iteration counts differ by a few), and the next step starts from there: measured
  # normwise qpos 1.6e-5 and qvel 8.5e-3 (cloth), 4.7e-7 / 3.4e-4 (aloha_cloth) after 3 steps
  # (tools/cloth_parity_probe.py -> profiles/r02_cloth_parity_probe.json)
  assert_close("qpos", np_(d.qpos), od.qpos, rtol=1e-3, atol=1e-4)
  _normwise("qpos", np_(d.qpos), od.qpos, 1e-4)
  _normwise("qvel", np_(d.qvel), od.qvel, 2e-2)
  # copies of one world stay bitwise equal over a longer rollout, and nothing blows up
  rep = 64 if which == "cloth" else 16
  m2, d2 = gpu_from_state(mjm, np.repeat(qpos[:1], rep, 0), np.repeat(qvel[:1], rep, 0), np.repeat(ctrl[:1], rep, 0), njmax=NJMAX, nconmax=NCONMAX)
  for _ in range(100):
    mjw.step(m2, d2)
  torch.cuda.synchronize()
  q = d2.qpos.cpu().numpy()
  assert np.isfinite(q).all()
  assert (q == q[:1]).all()
  assert int(d2.nacon) <= rep * NCONMAX


@pytest.mark.gpu
def test_gpu_aloha_sharding_is_bitwise_invariant():
  """SURVEY §8(e) on the sparse path: two shards (world_offset 0 / 8) of a 16-world aloha_cloth
  rollout with the benchmark's control noise equal the single 16-world run bitwise -- worlds never
  read each other (the pool is large enough that none overflows)."""
  import torch

  import mujoco_warp_amd as mjw

  mjm = aloha_model()
  nworld, half = 16, 8
  qpos, qvel, ctrl = aloha_states(mjm, nworld, seed=6)
  center = torch.as_tensor(np.asarray(ctrl[0], dtype=np.float32), device="cuda")

  def run(lo, hi):
    m, d = gpu_from_state(mjm, qpos[lo:hi], qvel[lo:hi], ctrl[lo:hi], njmax=ALOHA_NJMAX, nconmax=ALOHA_NCONMAX)
    d.world_offset = lo
    for i in range(10):
      mjw.ctrl_noise(m, d, i, center=center)
      mjw.step(m, d)
    torch.cuda.synchronize()
    return d.qpos.cpu().numpy(), d.qvel.cpu().numpy()

  q_all, v_all = run(0, nworld)
  q0, v0 = run(0, half)
  q1, v1 = run(half, nworld)
  np.testing.assert_array_equal(np.concatenate([q0, q1]), q_all)
  np.testing.assert_array_equal(np.concatenate([v0, v1]), v_all)
  assert np.isfinite(q_all).all()


@pytest.mark.gpu
def test_gpu_aloha_global_contact_pool_overflow():
  """The sparse path shares one pool of naconmax contacts between worlds like the reference
  (collision_core.py:212-231): nacon counts every contact found, each world's block is reserved with
  one atomic, and contacts past the pool are dropped together with their rows."""
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf
  from mujoco_warp_amd.types import ConstraintType

  mjm = aloha_model()
  nworld = 4
  qpos, qvel, ctrl = aloha_states(mjm, nworld, seed=3)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=ALOHA_NJMAX, nconmax=ALOHA_NCONMAX)
  mjw.fwd_position(m, d)
  torch.cuda.synchronize()
  per_world = d.ncon_world[:, 1].cpu().numpy().copy()
  total = int(per_world.sum())
  assert total > 1000
  pool = total // 2 + 17
  d2s = mjw.put_data(mjm, mjcf.MjData(mjm), nworld=nworld, nconmax=ALOHA_NCONMAX, njmax=ALOHA_NJMAX, naconmax=pool, device="cuda", m=m)
  for f in ("qpos", "qvel", "ctrl"):
    getattr(d2s, f).copy_(getattr(d, f))
  m2 = m
  mjw.fwd_position(m2, d2s)
  torch.cuda.synchronize()
  assert int(d2s.nacon[0]) == total  # every contact found is counted
  ncw = d2s.ncon_world.cpu().numpy()
  assert int(ncw[:, 1].sum()) == pool  # the pool is filled exactly
  for w in range(nworld):
    base, kept = int(ncw[w, 0]), int(ncw[w, 1])
    assert kept == max(0, min(per_world[w], pool - base))
    if kept:
      assert (d2s.contact.worldid[base:base + kept].cpu().numpy() == w).all()
    # contact rows only for the kept contacts
    n = int(d2s.nefc[w])
    typ = d2s.efc.type[w, :n].cpu().numpy()
    ids = d2s.efc.id[w, :n].cpu().numpy()
    con = typ == int(ConstraintType.CONTACT_PYRAMIDAL)
    assert (ids[con] < pool).all()


def _mul_m_check(mjm, device):
  import torch

  import mujoco_warp_amd as mjw

  m = mjw.put_model(mjm, device=device)
  d = mjw.make_data(mjm, nworld=3, nconmax=8, njmax=8, device=device, m=m)
  rng = np.random.default_rng(5)
  qm = rng.normal(size=(3, int(m.nM)))
  vec = rng.normal(size=(3, mjm.nv))
  d.qM[:] = torch.as_tensor(qm, dtype=torch.float32, device=device)
  res = torch.zeros((3, mjm.nv), dtype=torch.float32, device=device)
  v = torch.as_tensor(vec, dtype=torch.float32, device=device)
  mjw.mul_m(m, d, res, v)
  skip = torch.tensor([False, True, False], device=device)
  res2 = torch.full((3, mjm.nv), 7.0, dtype=torch.float32, device=device)
  mjw.mul_m(m, d, res2, v, skip=skip)
  qm32 = qm.astype(np.float32).astype(np.float64)
  for w in range(3):
    want = dense_qM(mjm, qm32[w]) @ vec[w].astype(np.float32)
    assert_close(f"mul_m[w{w}]", res[w].cpu().numpy(), want, rtol=1e-5, atol=1e-5 * np.abs(want).max())
  assert (res2[1] == 7.0).all() and torch.equal(res2[0], res[0])


def test_mul_m_sparse_layout(mjm):
  """support.mul_m on the sparse ancestor-row qM (support.py:67-101 gather): equal to the densified
  matrix times the vector, on the CPU device (torch ops only, no kernel)."""
  _mul_m_check(mjm, "cpu")


@pytest.mark.gpu
def test_gpu_mul_m_sparse_layout(mjm):
  _mul_m_check(mjm, "cuda")


def _csr_dense(rownnz, rowadr, colind, J, w, n, nv):
  out = np.zeros((n, nv))
  for r in range(n):
    a, k = int(rowadr[w, r]), int(rownnz[w, r])
    c = colind[w, 0, a:a + k]
    assert (np.diff(c) > 0).all()
    out[r, c] = J[w, 0, a:a + k]
  return out


def test_efc_J_csr_converter(mjm):
  """The ELL -> reference-CSR converter (io.py:940-943 layout) on synthetic slot-major rows (CPU)."""
  import torch

  import mujoco_warp_amd as mjw

  m = mjw.put_model(mjm, device="cpu")
  d = mjw.make_data(mjm, nworld=2, nconmax=8, njmax=16, device="cpu", m=m)
  rng = np.random.default_rng(9)
  nv, njrow = mjm.nv, d.efc.J.shape[1]
  dense = np.zeros((2, 16, nv))
  nefc = [5, 11]
  for w in range(2):
    d.nefc[w] = nefc[w]
    for r in range(nefc[w]):
      k = int(rng.integers(1, njrow + 1))
      cols = rng.choice(nv, size=k, replace=False)
      vals = rng.normal(size=k)
      d.efc.J_rownnz[w, r] = k
      for s in range(k):  # unsorted slots, as a tree walk may emit them
        d.efc.J[w, s, r] = vals[s]
        d.efc.J_colind[w, s, r] = int(cols[s])
        dense[w, r, cols[s]] = np.float32(vals[s])
    d.efc.J_rownnz[w, nefc[w]:] = 3  # stale counts past nefc are ignored
  rownnz, rowadr, colind, J = mjw.efc_J_csr(m, d, njmax_nnz=16 * njrow)
  assert J.shape == (2, 1, 16 * njrow) and rownnz.shape == (2, 16)
  for w in range(2):
    assert int(rownnz[w, nefc[w]:].sum()) == 0
    got = _csr_dense(rownnz.numpy(), rowadr.numpy(), colind.numpy(), J.numpy(), w, nefc[w], nv)
    np.testing.assert_array_equal(got, dense[w, :nefc[w]])


@pytest.mark.gpu
def test_gpu_efc_J_csr_matches_rows(mjm):
  import torch

  import mujoco_warp_amd as mjw

  qpos, qvel, ctrl = cloth_states(mjm, 2, seed=1)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=NJMAX, nconmax=NCONMAX)
  mjw.fwd_position(m, d)
  rownnz, rowadr, colind, J = mjw.efc_J_csr(m, d)
  torch.cuda.synchronize()
  for w in range(2):
    n = int(d.nefc[w])
    got = _csr_dense(rownnz.cpu().numpy(), rowadr.cpu().numpy(), colind.cpu().numpy(), J.cpu().numpy(), w, n, mjm.nv)
    np.testing.assert_array_equal(got, dense_J(d, w, n, mjm.nv))
