"""Spatial tendons (smooth.py:3172-3465): site paths, sphere / cylinder wrapping with and without sidesites,
pulleys, and the armature bias of their moving Jacobian (smooth.py:1590-1932).

CPU: the wrap geometry on the known answers of the reference's util_misc_test.py:297-513 (transcribed below
as data), for both restatements -- the oracle's C and the compiler's numpy (tendon_geom.py); the reference's
tendon test models (test_data/tendon/*.xml, copied as fixtures into tests/golden/tendon) compile, the two
restatements agree on length and Jacobian, the Jacobian is the derivative of the length, and the armature
bias is armature J (dJ/dt qvel).  GPU: the device path against the oracle on the same models.
"""

import glob
import os

import numpy as np
import pytest

from tests.common import gpu_from_state, np_, oracle_from_state

HERE = os.path.dirname(os.path.abspath(__file__))
TENDON_XML = sorted(glob.glob(os.path.join(HERE, "golden", "tendon", "*.xml")))
MAXVAL, MINVAL = 1e10, 1e-15
SPHERE, CYLINDER = 4, 5
NOWRAP2 = (-1.0, [MAXVAL] * 2, [MAXVAL] * 2)
NOWRAP3 = (-1.0, [MAXVAL] * 3, [MAXVAL] * 3)
S2 = np.sqrt(2.0)
# the reference's "wlen 0 at atol 1e-3" for radius 1 + 5e-4 around endpoints at distance sqrt 2 sits on its
# tolerance edge: the exact arc is r (pi/2 - 2 acos(r / sqrt 2)) = 1.0005e-3, used here instead
ARC = (1.0 + 5e-4) * (np.pi / 2 - 2 * np.arccos((1.0 + 5e-4) / S2))

# util_misc_test.py:297-513 -- (inputs, expected) at its tolerance 1e-3
IS_INTERSECT = [(([0, 0], [1, 0], [0, 1], [1, 1]), False), (([0, 0], [1, 0], [0.5, -1], [0.5, 1]), True),
                (([0, 0], [0, 0], [0, 0], [0, 0]), False)]
LENGTH_CIRCLE = [(([0, 1], [1, 0], 0, 1.0), 0.5 * np.pi), (([0, 1], [1, 0], 1, 1.0), 1.5 * np.pi),
                 (([1, 0], [0, 1], 0, 1.0), 1.5 * np.pi), (([1, 0], [0, 1], 1, 1.0), 0.5 * np.pi)]
WRAP_CIRCLE = [
  (([1, 0, 0, 1], [MAXVAL, MAXVAL], 0.1), NOWRAP2),
  (([1, 0, 0, 1], [0.0, 0.0], 0.1), NOWRAP2),
  (([S2, 0, 0, S2], [MAXVAL, MAXVAL], 1.0 + 5e-4), (ARC, [S2 / 2, S2 / 2], [S2 / 2, S2 / 2])),
  (([S2, 0, 0, S2], [0.0, 0.0], 1.0 + 5e-4), (ARC, [S2 / 2, S2 / 2], [S2 / 2, S2 / 2])),
  (([1.0, 0, 0, 1.0], [0.0, 0.0], 1.0), (0.5 * np.pi, [1.0, 0.0], [0.0, 1.0])),
  (([0, -100, 0, 100], [0.2, 0.0], 0.1), (0.0, [0.1, 0], [0.1, 0])),
  (([0, -100, 0, 100], [-0.2, 0.0], 0.1), (0.0, [-0.1, 0], [-0.1, 0])),
]
WRAP_INSIDE = [
  (([1, 0, 0, 1], 0.7071), (0.0, [0.5, 0.5], [0.5, 0.5])),
  (([0, 0, 1, 0], 1.0), NOWRAP2), (([1, 0, 0, 0], 1.0), NOWRAP2), (([0, 0, 0, 0], 1.0), NOWRAP2),
  (([1, 0, 0, 0], 2.0), NOWRAP2), (([0, 0, 1, 0], 2.0), NOWRAP2), (([1, 1, 1, 1], 0.1 * MINVAL), NOWRAP2),
  (([-1, 0, 1, 0], 0.1), NOWRAP2), (([-1, 0.2, 1, 0.2], 0.1), (0.0, [0, 0.1], [0, 0.1])),
]


def _wrap_cases(wraptype):
  """util_misc_test.py:441-513 (the last two cases run as CYLINDER whatever the parameter: the test rebinds it)."""
  big = [MAXVAL] * 3
  return [
    (([1, 1, 1], [2, 2, 2], [0, 0, 0], 0.1, wraptype, big), NOWRAP3),
    (([0.1, -1.0, 0.0], [0.1, 1.0, 0.0], [0, 0, 0], 0.1, wraptype, big), (0.0, [0.1, 0, 0], [0.1, 0, 0])),
    (([MINVAL, -100.0, 0.0], [MINVAL, 100.0, 0.0], [0, 0, 0], 0.1, wraptype, [0.1 + 10 * MINVAL, 0, 0]), (0.0, [0.1, 0, 0], [0.1, 0, 0])),
    (([0.0, -1.0, 0.0], [0.0, 1.0, 0.0], [0, 0, 0], 0.1, CYLINDER, [0, 0, 0]), NOWRAP3),
    (([1.0, -1.0, 0.0], [1.0, 1.0, 0.0], [0, 0, 0], 0.1, CYLINDER, [0.0, 0.0, 0.0]), (0.0, [0.1, 0, 0], [0.1, 0, 0])),
  ]


def _eq(a, b):
  np.testing.assert_allclose(np.asarray(a, float), np.asarray(b, float), atol=1e-3, rtol=1e-3)


def _check(got, want):
  _eq(got[0], want[0])
  _eq(got[1], want[1])
  _eq(got[2], want[2])


@pytest.mark.parametrize("impl", ["oracle32", "oracle64", "host"])
def test_wrap_geometry_known_answers(impl):
  """The reference runs these in fp32; its second wrap case (the segment x = 0.1 grazing a sphere of radius
  0.1) is exactly tangent, so whether it wraps (length 0) or not (-1) is decided by rounding: fp32 wraps as
  the reference asserts, fp64 may land on either side."""
  from mujoco_warp_amd import tendon_geom as tg
  from oracle import orc

  bits = 32 if impl == "oracle32" else 64
  orcl = impl.startswith("oracle")
  for args, want in IS_INTERSECT:
    got = orc.kat_wrap("is_intersect", args, real_bits=bits) if orcl else tg.is_intersect(*map(np.asarray, args))
    assert bool(got) == want
  for (p0, p1, ind, r), want in LENGTH_CIRCLE:
    got = orc.kat_wrap("length_circle", (p0, p1), ind, r, real_bits=bits) if orcl else tg.length_circle(np.array(p0, float), np.array(p1, float), ind, r)
    _eq(got, want)
  for (end, side, r), want in WRAP_CIRCLE:
    got = orc.kat_wrap("wrap_circle", (end, side), 0, r, real_bits=bits) if orcl else tg.wrap_circle(end, side, r)
    _check(got, want)
  for (end, r), want in WRAP_INSIDE:
    got = orc.kat_wrap("wrap_inside", (end,), 0, r, real_bits=bits) if orcl else tg.wrap_inside(end, r)
    _check(got, want)
  for wt in (SPHERE, CYLINDER):
    for i, ((x0, x1, pos, r, t, side), want) in enumerate(_wrap_cases(wt)):
      if orcl:
        got = orc.kat_wrap("wrap", (x0, x1, pos, np.eye(3), side), t, r, real_bits=bits)
      else:
        got = tg.wrap(np.array(x0, float), np.array(x1, float), np.array(pos, float), np.eye(3), r, t, np.array(side, float))
      if bits == 64 and wt == SPHERE and i == 1 and got[0] == -1.0:
        _check(got, NOWRAP3)  # the tangent case, rounded to "no wrap"
        continue
      _check(got, want)


def _load(path):
  from mujoco_warp_amd import mjcf

  return mjcf.load_model(path)


def _key_state(mjm, nworld=4, seed=0, qvel_sd=0.5):
  rng = np.random.default_rng(seed)
  base = mjm.key_qpos[0] if mjm.nkey else mjm.qpos0
  qpos = np.tile(base, (nworld, 1)) + 0.2 * rng.normal(size=(nworld, mjm.nq)) * (np.arange(nworld) > 0)[:, None]
  qvel = qvel_sd * rng.normal(size=(nworld, mjm.nv))
  return qpos, qvel, np.zeros((nworld, mjm.nu))


def _dense_J(mjm, od, w):
  J = np.zeros((mjm.ntendon, mjm.nv))
  for t in range(mjm.ntendon):
    a, n = mjm.ten_J_rowadr[t], mjm.ten_J_rownnz[t]
    J[t, mjm.ten_J_colind[a:a + n]] = od.ten_J[w, a:a + n]
  return J


@pytest.mark.parametrize("path", TENDON_XML, ids=[os.path.basename(p)[:-4] for p in TENDON_XML])
def test_compile_and_oracle_matches_host(path):
  """Oracle (C) and compiler (numpy) restatements agree on length and Jacobian at the keyframe and three
  perturbed poses; for spatial tendons the Jacobian's sparsity covers every dof on the path's chains."""
  from mujoco_warp_amd import mjcf

  mjm = _load(path)
  qpos, qvel, ctrl = _key_state(mjm)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  od.fwd_position()
  for w in range(len(qpos)):
    k = mjcf._kinematics_qpos0(mjm, qpos[w])
    Jo = _dense_J(mjm, od, w)
    for t in range(mjm.ntendon):
      if mjm.wrap_type[mjm.tendon_adr[t]] == 1:
        continue
      L, J = mjcf._spatial_tendon_qpos0(mjm, k, t)
      np.testing.assert_allclose(od.ten_length[w, t], L, rtol=1e-12, atol=1e-12)
      np.testing.assert_allclose(Jo[t], J, rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("path", TENDON_XML, ids=[os.path.basename(p)[:-4] for p in TENDON_XML])
def test_oracle_jacobian_is_length_derivative(path):
  """ten_J = d ten_length / d qpos (central differences; these models have slide / hinge joints only)."""
  mjm = _load(path)
  assert mjm.nq == mjm.nv
  qpos, qvel, ctrl = _key_state(mjm, nworld=1)
  eps = 1e-6
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  od.fwd_position()
  J = _dense_J(mjm, od, 0)
  fd = np.zeros_like(J)
  for i in range(mjm.nv):
    qp, qm = qpos.copy(), qpos.copy()
    qp[0, i] += eps
    qm[0, i] -= eps
    Ls = []
    for q in (qp, qm):
      _, o = oracle_from_state(mjm, q, qvel, ctrl)
      o.fwd_position()
      Ls.append(o.ten_length[0].copy())
    fd[:, i] = (Ls[0] - Ls[1]) / (2 * eps)
  np.testing.assert_allclose(J, fd, atol=1e-6)


@pytest.mark.parametrize("name", ["site", "pulley_site", "site_fixed"])
def test_oracle_armature_bias_is_jdot(name):
  """qfrc_bias(armature) - qfrc_bias(0) = armature J (dJ/dt qvel), dJ/dt by central differences along qvel
  (site-only paths: the reference leaves Jdot of wrapped segments out, smooth.py:1726-1728)."""
  mjm = _load(os.path.join(HERE, "golden", "tendon", name + ".xml"))
  qpos, qvel, ctrl = _key_state(mjm, nworld=1, seed=3)
  arm = 0.7
  out = {}
  for a in (0.0, arm):
    mjm.tendon_armature = np.full(mjm.ntendon, a)
    _, od = oracle_from_state(mjm, qpos, qvel, ctrl)
    od.fwd_position()
    od.fwd_velocity()
    out[a] = (od.qfrc_bias[0].copy(), _dense_J(mjm, od, 0))
  J = out[arm][1]
  eps = 1e-6
  Js = []
  for s in (1, -1):
    _, o = oracle_from_state(mjm, qpos + s * eps * qvel, qvel, ctrl)
    o.fwd_position()
    Js.append(_dense_J(mjm, o, 0))
  Jdot = (Js[0] - Js[1]) / (2 * eps)
  spatial = np.array([mjm.wrap_type[mjm.tendon_adr[t]] != 1 for t in range(mjm.ntendon)])
  want = arm * J[spatial].T @ (Jdot[spatial] @ qvel[0])
  np.testing.assert_allclose(out[arm][0] - out[0.0][0], want, rtol=1e-6, atol=1e-8)


def test_pulley_scales_following_segments():
  """pulley_site.xml: tendon 0 is pulley(2) + the site path of site.xml's tendon 0, so half its length."""
  from oracle import orc  # noqa: F401  (builds the oracle)

  a = _load(os.path.join(HERE, "golden", "tendon", "site.xml"))
  b = _load(os.path.join(HERE, "golden", "tendon", "pulley_site.xml"))
  qa = _key_state(a, nworld=1)
  _, oa = oracle_from_state(a, *qa)
  _, ob = oracle_from_state(b, *qa)
  oa.fwd_position()
  ob.fwd_position()
  np.testing.assert_allclose(ob.ten_length[0, 0], 0.5 * oa.ten_length[0, 0], rtol=1e-12)
  np.testing.assert_allclose(ob.ten_length[0, 3], oa.ten_length[0, 3] / 3, rtol=1e-12)
  np.testing.assert_allclose(ob.ten_length[0, 1:3], oa.ten_length[0, 1:3], rtol=1e-12)


def test_wrap_model_wraps():
  """wrap.xml at its keyframe: tendon 0 passes the sphere (radius .1 at x .5) -- it wraps, longer than the
  straight site-site distance."""
  mjm = _load(os.path.join(HERE, "golden", "tendon", "wrap.xml"))
  qpos, qvel, ctrl = _key_state(mjm, nworld=1)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  od.fwd_position()
  s0, s1 = mjm.wrap_objid[mjm.tendon_adr[0]], mjm.wrap_objid[mjm.tendon_adr[0] + 2]
  straight = np.linalg.norm(od.site_xpos[0, 3 * s1:3 * s1 + 3] - od.site_xpos[0, 3 * s0:3 * s0 + 3])
  assert od.ten_length[0, 0] > straight + 1e-4


# ---- GPU ------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("path", TENDON_XML, ids=[os.path.basename(p)[:-4] for p in TENDON_XML])
def test_gpu_tendon_models_match_oracle(path, sparse):
  """Forward on the device against the oracle: ten_length / ten_J / ten_velocity, qfrc_bias (armature bias),
  qfrc_passive and qacc, on 8 worlds around the keyframe; dense (world-per-wave) and sparse
  (workgroup-per-world, jacobian = sparse) paths."""
  import torch

  import mujoco_warp_amd as mjw

  mjm = _load(path)
  if sparse:
    mjm.opt.jacobian = 1
  if mjm.ntendon:
    mjm.tendon_armature = np.where(np.arange(mjm.ntendon) % 2 == 0, 0.3, 0.0)
  qpos, qvel, ctrl = _key_state(mjm, nworld=8, seed=5)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=32, nconmax=8)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=32, nconmax=8)
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  for f, tol in (("ten_length", 2e-6), ("ten_J", 2e-5), ("ten_velocity", 2e-5), ("qfrc_bias", 2e-5), ("qfrc_passive", 2e-5)):
    g, o = np_(getattr(d, f)).reshape(8, -1), getattr(od, f).reshape(8, -1)
    scale = max(1.0, float(np.abs(o).max()))
    np.testing.assert_allclose(g, o, atol=tol * scale, err_msg=f)
  err = np.abs(np_(d.qacc) - od.qacc).max() / max(1.0, float(np.abs(od.qacc).max()))
  assert err < 5e-3, err


TENDON_EQ = """<mujoco><worldbody><site name="s0" pos="0 0 .5"/>
<body pos="0 0 0"><joint name="j0" type="hinge" axis="0 1 0"/><geom type="capsule" size=".05" fromto="0 0 0 .3 0 0"/><site name="s1" pos=".3 0 0"/>
<body pos=".3 0 0"><joint name="j1" type="hinge" axis="0 1 0"/><geom type="capsule" size=".05" fromto="0 0 0 .3 0 0"/><site name="s2" pos=".3 0 0"/></body></body>
<body pos="0 .5 0"><joint name="j2" type="slide" axis="1 0 0"/><geom type="sphere" size=".05"/></body></worldbody>
<tendon><spatial name="sp"><site site="s0"/><site site="s1"/><site site="s2"/></spatial>
<fixed name="fx"><joint joint="j2" coef="1"/><joint joint="j0" coef=".5"/></fixed><fixed name="f1"><joint joint="j1" coef="1"/></fixed></tendon>
<equality><tendon tendon1="sp" tendon2="fx" polycoef="0 .7 .2 0 0"/><tendon tendon1="f1" polycoef=".1 0 0 0 0"/></equality></mujoco>"""


def test_oracle_tendon_equality_rows():
  """constraint.py:498-674: one row per active tendon equality, pos = (L1 - L1_0) - poly(L2 - L2_0), J = J1 -
  poly'(L2 - L2_0) J2, after the joint equality rows."""
  from mujoco_warp_amd import mjcf

  mjm = mjcf.load_model_from_string(TENDON_EQ)
  assert mjm.neq == 2 and list(mjm.eq_type) == [3, 3]
  qpos, qvel, ctrl = _key_state(mjm, nworld=3, seed=7)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl)
  od.fwd_position()
  for w in range(3):
    assert int(od.ne[w, 0]) == 2
    J = _dense_J(mjm, od, w)
    L = od.ten_length[w]
    dif = L[1] - mjm.tendon_length0[1]
    c = mjm.eq_data[0]
    pos0 = (L[0] - mjm.tendon_length0[0]) - (c[0] + c[1] * dif + c[2] * dif ** 2)
    np.testing.assert_allclose(od.efc_pos[w, 0], pos0, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(od.efc_J[w].reshape(od.njmax, mjm.nv)[0], J[0] - (c[1] + 2 * c[2] * dif) * J[1], atol=1e-12)
    np.testing.assert_allclose(od.efc_pos[w, 1], (L[2] - mjm.tendon_length0[2]) - 0.1, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
def test_gpu_tendon_equality_matches_oracle(sparse):
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf
  from tests.parity_models import efc_cost

  mjm = mjcf.load_model_from_string(TENDON_EQ)
  if sparse:
    mjm.opt.jacobian = 1
  qpos, qvel, ctrl = _key_state(mjm, nworld=8, seed=8)
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=16, nconmax=4)
  assert bool(m.is_sparse) == sparse
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=16, nconmax=4)
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  from tests.common import dense_efc_J

  for w in range(8):
    n = int(od.nefc[w, 0])
    assert int(d.nefc[w]) == n == 2
    np.testing.assert_allclose(np_(d.efc.pos[w, :n]), od.efc_pos[w, :n], atol=2e-6)
    np.testing.assert_allclose(dense_efc_J(m, d, w)[:n], od.efc_J[w].reshape(16, mjm.nv)[:n], atol=2e-5)
  err = np.abs(np_(d.qacc) - od.qacc).max() / max(1.0, float(np.abs(od.qacc).max()))
  assert err < 5e-3, err
