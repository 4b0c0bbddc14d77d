"""Pinning the CPU oracle (no GPU): reference known-answer tests + analytic invariants.

KATs restated from mujoco_warp/_src/math_test.py:27-131 (segment/segment closest
points, triangular index maps) and util_misc.halton (util_misc.py:59-73).
"""

import json
import os

import numpy as np
import pytest

from oracle import orc
from tests.common import HUMANOID, humanoid_model, oracle_from_state, random_states


# ---- math_test.py KATs (tests/golden/math_kat.json, extracted by tests/golden/make_golden.py) ----
_KAT = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "math_kat.json")))


@pytest.mark.parametrize("case", _KAT["closest_segment_points"], ids=lambda c: c["name"])
def test_closest_segment_points_kat(case):
  ba, bb = orc.kat_closest_segment_points(case["a0"], case["a1"], case["b0"], case["b1"])
  np.testing.assert_almost_equal(ba, case["best_a"], case["places"])
  np.testing.assert_almost_equal(bb, case["best_b"], case["places"])


@pytest.mark.parametrize("case", _KAT["triangular_index"], ids=lambda c: c["name"])
def test_triangular_index_kat(case):
  if case["fn"] == "upper_tri_index":
    n = case["n"]
    arr = [orc.kat_upper_tri_index(n, i, j) for i in range(n) for j in range(i + 1, n)]
    assert arr == list(range(case["count"]))
  elif case["fn"] == "upper_trid_index":
    n = case["n"]
    arr = [orc.kat_upper_trid_index(n, i, j) for i in range(n) for j in range(i, n)]
    assert arr == list(range(case["count"]))
  else:
    a = case["args"]
    assert orc.kat_upper_trid_index(*a[:3]) == orc.kat_upper_trid_index(*a[3:])


def test_golden_fixture_is_complete():
  assert len(_KAT["closest_segment_points"]) == 7 and len(_KAT["triangular_index"]) == 5


def test_halton_known_values():
  assert orc.halton(1, 2) == 0.5
  assert orc.halton(2, 2) == 0.25
  assert orc.halton(3, 2) == 0.75
  assert abs(orc.halton(1, 3) - 1 / 3) < 1e-15
  assert abs(orc.halton(5, 3) - (2 / 3 + 1 / 9)) < 1e-15
  assert orc.halton(0, 7) == 0.0


def test_ctrl_noise_formula():
  """benchmark.py:41-83 restated independently in numpy."""
  mjm = humanoid_model()
  om = orc.OracleModel(mjm)
  od = orc.OracleData(om, 3, 64, 24)
  for step in range(3):
    before = od.ctrl.copy()
    od.ctrl_noise(step, center=np.zeros(mjm.nu), world_offset=5)
    rate = np.exp(-mjm.opt.timestep / 0.1)
    scale = 0.01 * np.sqrt(1 - rate * rate)
    for w in range(3):
      for a in range(mjm.nu):
        h = orc.halton((step + 1) * (5 + w + 1), a + 2)
        want = np.clip(rate * before[w, a] + scale * (2 * h - 1), -1, 1)
        assert abs(od.ctrl[w, a] - want) < 1e-14


# ---- analytic invariants ----------------------------------------------------------------------
def _single_body(xml_body, option=""):
  from mujoco_warp_amd import mjcf

  xml = f"""<mujoco><option {option}/><worldbody>{xml_body}</worldbody></mujoco>"""
  return mjcf.load_model_from_string(xml)


def test_free_fall_is_ballistic():
  m = _single_body('<body pos="0 0 1"><freejoint/><geom type="sphere" size=".1"/></body>', 'timestep="0.01"')
  om = orc.OracleModel(m)
  od = orc.OracleData(om, 1, 16, 8)
  od.qvel[0, :3] = [1.0, -2.0, 3.0]
  n = 20
  for _ in range(n):
    od.step()
  dt, g = 0.01, -9.81
  # semi-implicit Euler: v_k = v0 + k g dt, z_n = z0 + dt * sum_k v_k
  vz = 3.0 + g * dt * np.arange(1, n + 1)
  z = 1.0 + dt * vz.sum()
  np.testing.assert_allclose(od.qpos[0, :3], [1.0 * dt * n, -2.0 * dt * n, z], rtol=1e-12, atol=1e-12)
  np.testing.assert_allclose(od.qacc[0, :3], [0, 0, g], atol=1e-12)
  assert od.nefc[0, 0] == 0


def test_capsule_inertia_matches_analytic():
  m = _single_body('<body><freejoint/><geom type="capsule" fromto="0 0 -0.2 0 0 0.2" size="0.05"/></body>')
  r, h = 0.05, 0.4
  vol = np.pi * r * r * h + 4 / 3 * np.pi * r**3
  mass = 1000 * vol
  assert abs(m.body_mass[1] - mass) < 1e-12
  mc = 1000 * np.pi * r * r * h
  ms = mass - mc
  ixx = mc * (3 * r * r + h * h) / 12 + 2 * ms * r * r / 5 + ms * h * (3 * r + 2 * h) / 8
  izz = mc * r * r / 2 + 2 * ms * r * r / 5
  np.testing.assert_allclose(sorted(m.body_inertia[1]), sorted([ixx, ixx, izz]), rtol=1e-12)


def test_no_efc_keyframe_is_contact_free():
  mjm = humanoid_model()
  om = orc.OracleModel(mjm)
  od = orc.OracleData(om, 1, 64, 24)
  od.qpos[0] = mjm.key_qpos[2]  # 'no_efc'
  od.forward()
  assert od.nefc[0, 0] == 0 and od.ncon[0, 0] == 0
  np.testing.assert_allclose(od.qacc[0], od.qacc_smooth[0], rtol=1e-6, atol=1e-9)


def test_mass_matrix_spd_and_energy():
  mjm = humanoid_model()
  qpos, qvel, ctrl = random_states(mjm, 4, seed=11)
  om, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  od.fwd_position()
  od.fwd_velocity()
  for w in range(4):
    M = od.qM[w].reshape(mjm.nv, mjm.nv)
    np.testing.assert_allclose(M, M.T, atol=1e-12)
    assert np.linalg.eigvalsh(M).min() > 0
    # kinetic energy from cvel/cinert equals 0.5 qvel' M qvel
    ke_m = 0.5 * qvel[w] @ (M - np.diag(mjm.dof_armature)) @ qvel[w]  # armature is not body inertia
    ke_b = 0.0
    for b in range(1, mjm.nbody):
      ci = od.cinert[w].reshape(-1, 10)[b]
      I = np.array([[ci[0], ci[3], ci[4]], [ci[3], ci[1], ci[5]], [ci[4], ci[5], ci[2]]])
      h = ci[6:9]
      S = np.array([[0, -h[2], h[1]], [h[2], 0, -h[0]], [-h[1], h[0], 0]])
      Mb = np.block([[I, S], [-S, ci[9] * np.eye(3)]])
      v = od.cvel[w].reshape(-1, 6)[b]
      ke_b += 0.5 * v @ Mb @ v
    assert abs(ke_m - ke_b) < 1e-9 * max(1.0, ke_m)


def test_cg_and_newton_reach_same_optimum():
  m_cg = humanoid_model("CG", iterations=200)
  m_nt = humanoid_model("NEWTON", iterations=200)
  qpos, qvel, ctrl = random_states(m_cg, 6, seed=12)
  _, a = oracle_from_state(m_cg, qpos, qvel, ctrl)
  _, b = oracle_from_state(m_nt, qpos, qvel, ctrl)
  a.forward()
  b.forward()
  # both minimise the same convex cost (solver.py); costs agree closely
  np.testing.assert_allclose(a.solver_cost[:, 0], b.solver_cost[:, 0], rtol=1e-5)
  assert (a.nefc[:, 0] > 0).all()


def test_solution_is_stationary():
  """At the Newton solution grad = M qacc - qfrc_smooth - J' f ~ 0 (solver.py:2879-2888)."""
  mjm = humanoid_model("NEWTON", iterations=100)
  qpos, qvel, ctrl = random_states(mjm, 4, seed=13)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  od.forward()
  nv = mjm.nv
  for w in range(4):
    M = od.qM[w].reshape(nv, nv)
    n = int(od.nefc[w, 0])
    J = od.efc_J[w].reshape(-1, nv)[:n]
    grad = M @ od.qacc[w] - od.qfrc_smooth[w] - J.T @ od.efc_force[w, :n]
    assert np.abs(grad).max() < 1e-6 * max(1.0, np.abs(od.qfrc_smooth[w]).max())


def test_fp32_oracle_tracks_fp64():
  mjm = humanoid_model()
  qpos, qvel, ctrl = random_states(mjm, 4, seed=14)
  _, a = oracle_from_state(mjm, qpos, qvel, ctrl, real_bits=64)
  _, b = oracle_from_state(mjm, qpos, qvel, ctrl, real_bits=32)
  a.fwd_position()
  b.fwd_position()
  np.testing.assert_allclose(b.xpos, a.xpos, atol=1e-5)
  np.testing.assert_allclose(b.qM, a.qM, rtol=1e-4, atol=1e-4)


def test_long_rollout_stays_finite():
  mjm = humanoid_model()
  om = orc.OracleModel(mjm)
  od = orc.OracleData(om, 4, 64, 24)
  od.qpos[:] = mjm.key_qpos[0]
  for i in range(300):
    od.ctrl_noise(i, center=np.zeros(mjm.nu))
    od.step(nthread=4)
  assert np.isfinite(od.qpos).all()
  assert (od.ncon[:, 0] > 0).all()  # the humanoid settles onto the floor
