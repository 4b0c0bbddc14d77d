"""reset_data(mask), get_data_into, make_data sizing, the pool-overflow drop and refused callbacks
(reference io.py:859-932, :1243-1455, :1458-1691; collision_core.py:212-231; forward.py:876-881).

The CPU tests run the host-side reset / readback on CPU-resident torch tensors (no kernel launch);
the GPU tests step the HIP path first and compare reset worlds with freshly made ones."""

import numpy as np
import pytest
import torch

MOCAP_EQ_XML = """<mujoco><option timestep="0.002"/><worldbody>
<geom type="plane" size="5 5 .1"/>
<body name="m" mocap="true" pos=".3 .2 1" quat="0 1 0 0"><geom type="sphere" size=".05" contype="0" conaffinity="0"/></body>
<body name="a" pos="0 0 1"><freejoint/><geom type="box" size=".1 .05 .05"/></body>
<body name="c" pos="-.5 0 1"><joint name="h1" type="hinge" axis="1 0 0"/><geom type="capsule" fromto="0 0 0 0 0 -.3" size=".03"/>
  <body name="c2" pos="0 0 -.3"><joint name="h2" type="hinge" axis="1 0 0"/><geom type="sphere" size=".05"/></body>
</body>
</worldbody>
<equality><connect body1="a" anchor="0 0 .05"/><joint joint1="h2" active="false"/></equality>
<actuator><motor joint="h1"/></actuator>
<sensor><framepos objtype="body" objname="a"/></sensor>
</mujoco>"""


def _mocap_model():
  from mujoco_warp_amd import mjcf

  return mjcf.load_model_from_string(MOCAP_EQ_XML)


def _dirty(d):
  for name in ("qpos", "qvel", "ctrl", "qacc_warmstart", "qfrc_applied", "xfrc_applied", "qacc", "sensordata", "energy", "qM", "time"):
    getattr(d, name).fill_(7.0)
  for name in ("ne", "nf", "nl", "nefc", "solver_niter"):
    getattr(d, name).fill_(3)
  d.eq_active.fill_(0)
  d.mocap_pos.fill_(9.0)
  d.mocap_quat.fill_(0.5)
  n = d.nworld
  d.nacon.fill_(n)
  d.contact.worldid[:n] = torch.arange(n, dtype=torch.int32)
  d.contact.dist[:n] = 1.0
  d.contact.dim[:n] = 3
  d.contact.efc_address[:n] = 5


def test_reset_data_mask_mirrors_reference_fields():
  import mujoco_warp_amd as mjw

  mjm = _mocap_model()
  assert mjm.nmocap == 1 and mjm.neq == 2 and list(mjm.eq_active0) == [1, 0]
  m = mjw.put_model(mjm, device="cpu")
  d = mjw.make_data(mjm, nworld=4, nconmax=4, njmax=32, device="cpu", m=m)
  fresh = mjw.make_data(mjm, nworld=4, nconmax=4, njmax=32, device="cpu", m=m)
  _dirty(d)
  mask = torch.tensor([False, True, False, True])
  mjw.reset_data(m, d, mask)
  for w in range(4):
    for name in ("qpos", "qvel", "ctrl", "qacc_warmstart", "qfrc_applied", "xfrc_applied", "qacc", "sensordata", "energy", "qM",
                 "mocap_pos", "mocap_quat", "eq_active", "time", "ne", "nf", "nl", "nefc", "solver_niter"):
      got, want = getattr(d, name)[w], getattr(fresh, name)[w]
      if mask[w]:
        assert torch.equal(got, want), (name, w)
      else:
        assert not torch.equal(got, want), (name, w)
  np.testing.assert_allclose(d.mocap_pos[1, 0].numpy(), [0.3, 0.2, 1.0], rtol=1e-6)
  np.testing.assert_allclose(d.mocap_quat[1, 0].numpy(), [0, 1, 0, 0], atol=1e-7)
  assert d.eq_active[1].tolist() == [1, 0]
  # contacts of reset worlds cleared, others kept; world 0 not reset -> pool counter kept
  assert d.contact.dist.tolist()[:4] == [1.0, 0.0, 1.0, 0.0]
  assert d.contact.efc_address[1].tolist() == [-1] * d.contact.efc_address.shape[1]
  assert d.contact.efc_address[0, 0] == 5
  assert int(d.nacon[0]) == 4
  mjw.reset_data(m, d, torch.tensor([True, False, False, False]))
  assert int(d.nacon[0]) == 0
  mjw.reset_data(m, d)  # all worlds
  for name in ("qpos", "qvel", "mocap_pos", "eq_active", "qM"):
    assert torch.equal(getattr(d, name), getattr(fresh, name)), name
  with pytest.raises(ValueError):
    mjw.reset_data(m, d, torch.ones(3, dtype=torch.bool))


def test_make_data_size_arguments():
  """nccdmax / njmax_nnz / naccdmax keywords and their checks (io.py:859-932)."""
  import mujoco_warp_amd as mjw
  from tests.common import humanoid_model

  mjm = humanoid_model()
  m = mjw.put_model(mjm, device="cpu")
  d = mjw.make_data(mjm, nworld=3, nconmax=8, nccdmax=4, njmax=16, njmax_nnz=100, naccdmax=10, device="cpu", m=m)
  assert (d.naconmax, d.nccdmax, d.naccdmax, d.njmax_nnz) == (24, 4, 10, 100)
  d = mjw.make_data(mjm, nworld=3, nconmax=8, njmax=16, device="cpu", m=m)
  assert (d.nccdmax, d.naccdmax, d.njmax_nnz) == (8, 24, 16 * mjm.nv)
  d = mjw.make_data(mjm, nworld=3, nconmax=8, nccdmax=2, njmax=16, device="cpu", m=m)
  assert d.naccdmax == 6
  with pytest.raises(ValueError, match="nccdmax"):
    mjw.make_data(mjm, nworld=2, nconmax=4, nccdmax=5, naccdmax=4, device="cpu", m=m)
  with pytest.raises(ValueError, match="naccdmax"):
    mjw.make_data(mjm, nworld=2, nconmax=4, naccdmax=9, device="cpu", m=m)
  with pytest.raises(ValueError):
    mjw.make_data(mjm, nworld=0, device="cpu", m=m)


def test_get_data_into_world_selection():
  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  mjm = _mocap_model()
  m = mjw.put_model(mjm, device="cpu")
  d = mjw.make_data(mjm, nworld=3, nconmax=4, njmax=32, device="cpu", m=m)
  for w in range(3):
    d.qpos[w] = float(w)
    d.qvel[w] = 10.0 + w
  d.nefc[:] = torch.tensor([0, 2, 1], dtype=torch.int32)
  d.efc.force[1, :2] = torch.tensor([1.5, 2.5])
  d.nacon.fill_(2)
  d.contact.worldid[:2] = torch.tensor([1, 2], dtype=torch.int32)
  d.contact.dist[:2] = torch.tensor([-0.1, -0.2])
  res = mjcf.MjData(mjm)
  mjw.get_data_into(res, mjm, d, world_id=1)
  np.testing.assert_array_equal(res.qpos, np.ones(mjm.nq))
  np.testing.assert_array_equal(res.qvel, np.full(mjm.nv, 11.0))
  assert res.nefc == 2 and res.efc_force.tolist() == [1.5, 2.5]
  assert res.ncon == 1 and np.allclose(res.contact.dist, [-0.1])
  with pytest.raises(ValueError):
    mjw.get_data_into(res, mjm, d, world_id=3)


@pytest.mark.gpu
def test_gpu_reset_then_step_equals_fresh_worlds():
  """Step humanoid worlds into contact, reset a mask, step again: reset worlds equal fresh ones bitwise."""
  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf
  from tests.common import HUMANOID, np_

  mjm = mjcf.load_model(HUMANOID)
  mjw.override_model(mjm, ["opt.solver=CG"])
  mjd = mjcf.MjData(mjm)
  mjcf.reset_data_keyframe(mjm, mjd, 0)
  m = mjw.put_model(mjm, device="cuda")
  d = mjw.put_data(mjm, mjd, nworld=8, nconmax=24, njmax=64, device="cuda", m=m)
  for i in range(20):
    mjw.ctrl_noise(m, d, i)
    mjw.step(m, d)
  mask = torch.tensor([True, False, True, False, False, True, False, True], device="cuda")
  before = np_(d.qpos)
  mjw.reset_data(m, d, mask)
  fresh = mjw.make_data(mjm, nworld=8, nconmax=24, njmax=64, device="cuda", m=m)
  for _ in range(5):
    mjw.step(m, d)
    mjw.step(m, fresh)
  torch.cuda.synchronize()
  got, want = np_(d.qpos), np_(fresh.qpos)
  mk = mask.cpu().numpy()
  np.testing.assert_array_equal(got[mk], want[mk])
  assert not np.allclose(got[~mk], want[~mk])
  assert np.isfinite(before).all()


@pytest.mark.gpu
def test_gpu_contact_pool_overflow_drops_rows():
  """naconmax smaller than the contacts found: contacts past the pool are dropped together with their
  efc rows (collision_core.py:212-231), so every row's contact id is inside the pool."""
  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf
  from mujoco_warp_amd.types import ConstraintType
  from tests.common import HUMANOID

  mjm = mjcf.load_model(HUMANOID)
  mjw.override_model(mjm, ["opt.solver=CG"])
  mjd = mjcf.MjData(mjm)
  mjcf.reset_data_keyframe(mjm, mjd, 0)
  m = mjw.put_model(mjm, device="cuda")
  full = mjw.put_data(mjm, mjd, nworld=4, nconmax=24, njmax=64, device="cuda", m=m)
  mjw.forward(m, full)
  torch.cuda.synchronize()
  total = int(full.nacon[0])
  assert total >= 8
  small = mjw.put_data(mjm, mjd, nworld=4, nconmax=24, njmax=64, naconmax=total // 2, device="cuda", m=m)
  mjw.forward(m, small)
  torch.cuda.synchronize()
  assert int(small.nacon[0]) == total  # the counter still counts every contact found
  ncontact_rows = 0
  for w in range(4):
    n = int(small.nefc[w])
    typ = small.efc.type[w, :n].cpu().numpy()
    ids = small.efc.id[w, :n].cpu().numpy()
    con = np.isin(typ, (int(ConstraintType.CONTACT_FRICTIONLESS), int(ConstraintType.CONTACT_PYRAMIDAL)))
    assert (ids[con] < total // 2).all()
    ncontact_rows += int(con.sum())
  # the stored contacts keep their rows: dropping past the pool removes rows, never the pool's own
  assert 0 < ncontact_rows < sum(int(full.nefc[w]) for w in range(4))


def test_derive_model_fields_for_reference_binding():
  """io.derive_model_fields: the derived arrays a reference-side binding uploads."""
  import numpy as np

  from mujoco_warp_amd import io
  from tests.common import humanoid_model

  mjm = humanoid_model()
  f = io.derive_model_fields(mjm)
  assert f["nxn"] == 161 and f["nxn_geom_pair"].shape == (161, 2) and f["nxn_ccd"] == 0
  par = np.asarray(mjm.body_parentid)
  # DFS subtree ranges: every body's descendants lie in [b, subtree_end[b])
  for b in range(1, mjm.nbody):
    p = par[b]
    assert p <= b < f["body_subtree_end"][p] and f["body_subtree_end"][b] <= f["body_subtree_end"][p]
    assert f["body_level"][b] == f["body_level"][p] + 1
  # level lists: level_body[level_adr[l]:level_adr[l+1]] are the bodies of depth l
  for lv in range(f["nlevel"]):
    bodies = f["level_body"][f["level_adr"][lv]:f["level_adr"][lv + 1]]
    assert (f["body_level"][bodies] == lv).all()
  assert f["nlimited"] == len(f["jnt_limited_slide_hinge_adr"]) == 21
  assert f["nJmom"] == mjm.nu and f["nv_pad"] == 28
