"""SITE (with and without a reference site), SLIDERCRANK and BODY (adhesion) transmissions (smooth.py:2150-2602).

CPU: the reference's actuation models (test_data/actuation/{site,slidercrank,adhesion}.xml, copied as fixtures
into tests/golden/actuation) compile; the oracle's moment rows are the derivative of the actuator length
wherever the length is a function of qpos (slider-crank; site with a reference site and a translational gear),
equal J' (R gear) for a site without a reference, agree with the compiler's host restatement, and the BODY
moment is minus the mean contact-normal Jacobian over the body's contacts, inside or outside the margin.
GPU: the device path against the oracle (lengths, moment rows, actuator forces, qacc).
"""

import os

import numpy as np
import pytest

from tests.common import gpu_from_state, np_, oracle_from_state

HERE = os.path.dirname(os.path.abspath(__file__))
ACT = os.path.join(HERE, "golden", "actuation")


def _load(name, **kw):
  from mujoco_warp_amd import mjcf

  if name.lstrip().startswith("<mujoco"):
    return mjcf.load_model_from_string(name)
  return mjcf.load_model(os.path.join(ACT, name + ".xml"))


def _oracle(mjm, qpos, forward=False):
  qpos = np.atleast_2d(qpos)
  n = len(qpos)
  _, od = oracle_from_state(mjm, qpos, np.zeros((n, mjm.nv)), np.zeros((n, mjm.nu)))
  od.forward() if forward else od.fwd_position()
  return od


def _states(mjm, nworld, seed=0, sd=0.3):
  rng = np.random.default_rng(seed)
  base = mjm.key_qpos[0] if mjm.nkey else mjm.qpos0
  qpos = np.tile(base, (nworld, 1)) + sd * rng.normal(size=(nworld, mjm.nq)) * (np.arange(nworld) > 0)[:, None]
  return qpos


def _fd_moment(mjm, qpos, eps=1e-6):
  J = np.zeros((mjm.nu, mjm.nv))
  for i in range(mjm.nv):
    qp, qm = qpos.copy(), qpos.copy()
    qp[i] += eps
    qm[i] -= eps
    J[:, i] = (_oracle(mjm, qp).actuator_length[0] - _oracle(mjm, qm).actuator_length[0]) / (2 * eps)
  return J


SITE_TRANSLATIONAL = """<mujoco><worldbody><site name="siteworld" pos=".1 .2 .3" euler="10 20 30"/>
<body><joint type="hinge" axis="1 0 0"/><geom type="sphere" size=".1" pos="0 .1 0"/><site name="site0" pos=".1 0 .05"/>
<body pos="0 .2 0"><joint type="slide" axis="0 1 0"/><joint type="hinge" axis="0 1 0"/><geom type="sphere" size=".1" pos="0 0 .2"/>
<site name="site1" pos=".05 .1 .2"/></body></body></worldbody>
<actuator><motor site="site0" refsite="siteworld" gear="1 2 3 0 0 0"/><motor site="site1" refsite="site0" gear="-1 .5 2 0 0 0"/>
<motor site="site1" refsite="siteworld" gear=".3 -2 1 0 0 0"/></actuator></mujoco>"""


@pytest.mark.parametrize("name", ["slidercrank", "site_translational"])
def test_oracle_moment_is_length_derivative(name):
  mjm = _load(SITE_TRANSLATIONAL if name == "site_translational" else name)
  assert mjm.nq == mjm.nv
  for q in _states(mjm, 3, seed=1):
    od = _oracle(mjm, q)
    np.testing.assert_allclose(od.actuator_moment[0].reshape(mjm.nu, mjm.nv), _fd_moment(mjm, q), atol=1e-6)


def test_site_without_reference_is_jacobian_transpose_wrench():
  """mom = Jp' (R gear[:3]) + Jr' (R gear[3:]) with R the site frame (smooth.py:2285-2328), via the host
  restatement (mjcf._site_moment) at perturbed poses."""
  from mujoco_warp_amd import mjcf

  mjm = _load("site")
  for q in _states(mjm, 3, seed=2):
    od = _oracle(mjm, q)
    k = mjcf._kinematics_qpos0(mjm, q)
    mom = od.actuator_moment[0].reshape(mjm.nu, mjm.nv)
    for a in range(mjm.nu):
      np.testing.assert_allclose(mom[a], mjcf._site_moment(mjm, k, a), rtol=1e-10, atol=1e-12)
    assert np.all(od.actuator_length[0][mjm.actuator_trnid[:, 1] < 0] == 0)


def test_site_reference_rotation_length():
  """site.xml with refsite: length = (R_ref' (x - x_ref)) . gear[:3] + quat_sub(q, q_ref) . gear[3:], quats
  as site_quat * xquat (smooth.py:2366-2384); at qpos0 the world-frame sites coincide in orientation only for
  the first body."""
  from mujoco_warp_amd import mjcf
  from mujoco_warp_amd.mjcf import quat_mul, quat_to_mat, rot_vec

  mjm = _load("site")
  q = mjm.key_qpos[0]
  od = _oracle(mjm, q)
  k = mjcf._kinematics_qpos0(mjm, q)

  def quat_sub(qa, qb):  # math.quat_sub: the rotation vector of qb^-1 qa
    dq = quat_mul(np.array([qb[0], -qb[1], -qb[2], -qb[3]]), qa)
    s = np.linalg.norm(dq[1:])
    ang = 2 * np.arctan2(s, dq[0])
    if ang > np.pi:
      ang -= 2 * np.pi
    return dq[1:] / s * ang if s > 0 else np.zeros(3)

  for a in range(mjm.nu):
    s1, s2 = mjm.actuator_trnid[a]
    if s2 < 0:
      continue
    b1, b2 = mjm.site_bodyid[s1], mjm.site_bodyid[s2]
    x1 = k["xpos"][b1] + rot_vec(k["xquat"][b1], mjm.site_pos[s1])
    x2 = k["xpos"][b2] + rot_vec(k["xquat"][b2], mjm.site_pos[s2])
    R2 = quat_to_mat(quat_mul(k["xquat"][b2], mjm.site_quat[s2]))
    g = mjm.actuator_gear[a]
    want = (R2.T @ (x1 - x2)) @ g[:3] + quat_sub(quat_mul(mjm.site_quat[s1], k["xquat"][b1]), quat_mul(mjm.site_quat[s2], k["xquat"][b2])) @ g[3:]
    np.testing.assert_allclose(od.actuator_length[0, a], want, rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("key", range(4))
def test_oracle_adhesion_body_moment(key):
  """adhesion.xml keyframes (smooth_test.py:360-400 runs the same four): minus the mean of n . (J(pos, b2) -
  J(pos, b1)) over the body's contacts; the keyframes put contacts inside the margin, in the gap and beyond."""
  mjm = _load("adhesion")
  od = _oracle(mjm, mjm.key_qpos[key])
  n = int(od.ncon[0, 0])
  body = mjm.actuator_trnid[0, 0]
  from mujoco_warp_amd import mjcf

  k = mjcf._kinematics_qpos0(mjm, mjm.key_qpos[key])
  acc, cnt = np.zeros(mjm.nv), 0
  for c in range(n):
    g1, g2 = od.con_geom[0, 2 * c:2 * c + 2]
    b1, b2 = mjm.geom_bodyid[g1], mjm.geom_bodyid[g2]
    if body not in (b1, b2):
      continue
    cnt += 1
    pos, nrm = od.con_pos[0, 3 * c:3 * c + 3], od.con_frame[0, 9 * c:9 * c + 3]

    def jp(b):
      J = np.zeros((3, mjm.nv))
      bb = b
      while bb > 0:
        for d in range(mjm.body_dofadr[bb], mjm.body_dofadr[bb] + mjm.body_dofnum[bb]):
          cd = k["cdof"][d]
          J[:, d] = cd[3:] + np.cross(cd[:3], pos - k["subtree_com"][mjm.body_rootid[b]])
        bb = mjm.body_parentid[bb]
      return J

    acc += nrm @ (jp(b2) - jp(b1))
  want = -acc / cnt if cnt else acc
  np.testing.assert_allclose(od.actuator_moment[0], want, atol=1e-9)


def test_put_model_sizes():
  import mujoco_warp_amd as mjw

  m = mjw.put_model(_load("site"), device="cpu")
  assert m.nsitetrn == 6 and m.nbodytrn == 0 and m.nJmom == 1 + 1 + 2 + 2 + 3 + 3
  m = mjw.put_model(_load("adhesion"), device="cpu")
  assert m.nbodytrn == 1 and m.nJmom == m.nv and m.act_maxnnz == m.nv


# ---- GPU ------------------------------------------------------------------------------------------
def _dense_moment(mjm, d, w):
  mom = np.zeros((mjm.nu, mjm.nv))
  rn, ra = d.moment_rownnz[w].cpu().numpy(), d.moment_rowadr[w].cpu().numpy()
  ci, mv = d.moment_colind[w].cpu().numpy(), np_(d.actuator_moment[w])
  for a in range(mjm.nu):
    mom[a, ci[ra[a]:ra[a] + rn[a]]] = mv[ra[a]:ra[a] + rn[a]]
  return mom


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["site", "slidercrank", "adhesion", "adhesion_elliptic", "site_translational", "site_sparse",
                                  "slidercrank_sparse", "site_translational_sparse", "adhesion_sparse", "adhesion_elliptic_sparse"])
def test_gpu_transmissions_match_oracle(name):
  """The device computes the BODY moment from the contact normals; the oracle from the constraint rows as
  the reference does (pyramidal and elliptic cones).  `_sparse`: the same models forced onto the sparse
  path (jacobian="sparse"), whose transmission stage runs the same site / slider-crank rows (mjw_trn.h) and
  fills the BODY rows from the world's contact list after the constraint stage."""
  import torch

  import mujoco_warp_amd as mjw

  base = name.replace("_elliptic", "").replace("_sparse", "")
  mjm = _load(SITE_TRANSLATIONAL if base == "site_translational" else base)
  if name.startswith("adhesion_elliptic"):
    mjm.opt.cone = 1
  if name.endswith("_sparse"):
    mjw.override_model(mjm, ["opt.jacobian=sparse"])
  nworld = 8
  if name.startswith("adhesion"):
    qpos = np.stack([mjm.key_qpos[i % 4] for i in range(nworld)])
  else:
    qpos = _states(mjm, nworld, seed=4)
  rng = np.random.default_rng(5)
  qvel = 0.3 * rng.normal(size=(nworld, mjm.nv))
  ctrl = rng.uniform(0, 1, size=(nworld, mjm.nu))
  m, d = gpu_from_state(mjm, qpos, qvel, ctrl, njmax=32, nconmax=8)
  _, od = oracle_from_state(mjm, qpos, qvel, ctrl, njmax=32, nconmax=8)
  assert m.is_sparse == name.endswith("_sparse")
  mjw.forward(m, d)
  od.forward()
  torch.cuda.synchronize()
  np.testing.assert_allclose(np_(d.actuator_length), od.actuator_length, atol=2e-5 * max(1.0, np.abs(od.actuator_length).max()))
  for w in range(nworld):
    want = od.actuator_moment[w].reshape(mjm.nu, mjm.nv)
    np.testing.assert_allclose(_dense_moment(mjm, d, w), want, atol=2e-5 * max(1.0, np.abs(want).max()), err_msg=f"world {w}")
  np.testing.assert_allclose(np_(d.qfrc_actuator), od.qfrc_actuator, atol=2e-5 * max(1.0, np.abs(od.qfrc_actuator).max()))
  err = np.abs(np_(d.qacc) - od.qacc).max() / max(1.0, float(np.abs(od.qacc).max()))
  assert err < 5e-3, err
