"""CPU tests of the host side: MJCF compiler, put_model/put_data/make_data, C ABI exports."""

import ctypes
import os
import re

import numpy as np
import pytest

from tests.common import HUMANOID, ROOT, humanoid_model


def test_humanoid_sizes():
  m = humanoid_model()
  assert (m.nq, m.nv, m.nu, m.na, m.nbody, m.njnt, m.ngeom) == (28, 27, 21, 0, 17, 22, 20)
  assert (m.ncam, m.nlight, m.nsite, m.nkey) == (3, 2, 0, 3)
  assert m.opt.timestep == 0.005
  assert m.opt.disableflags & (1 << 15)  # eulerdamp disabled (humanoid.xml:18)


def test_humanoid_nxn_pairs():
  """161 filtered pairs (100 cap-cap, 39 sph-cap, 16 plane-cap, 3 plane-sph, 3 sph-sph)."""
  from mujoco_warp_amd.io import nxn_geom_pairs

  m = humanoid_model()
  pairs, pairid = nxn_geom_pairs(m)
  assert len(pairs) == 161
  t = np.sort(m.geom_type[pairs], axis=1)
  kinds = {}
  for a, b in t:
    kinds[(a, b)] = kinds.get((a, b), 0) + 1
  assert kinds == {(3, 3): 100, (2, 3): 39, (0, 3): 16, (0, 2): 3, (2, 2): 3}
  assert (pairid == -1).all()


def test_humanoid_tree_and_symmetry():
  m = humanoid_model()
  names = m.body_names
  # left/right limbs mirror each other in mass
  for side in ("thigh", "shin", "foot", "upper_arm", "lower_arm", "hand"):
    r, l = names.index(f"{side}_right"), names.index(f"{side}_left")
    assert abs(m.body_mass[r] - m.body_mass[l]) < 1e-12
  for i in range(1, m.nbody):
    assert m.body_parentid[i] < i
  assert m.dof_parentid[0] == -1 and all(m.dof_parentid[i] < i for i in range(m.nv))
  assert 40.0 < m.body_mass.sum() < 42.0
  assert np.all(m.dof_invweight0 > 0) and np.all(m.body_invweight0[1:] > 0)


def test_default_classes_resolved():
  m = humanoid_model()
  j = {n: i for i, n in enumerate(m.jnt_names)}
  np.testing.assert_allclose(m.jnt_range[j["hip_y_right"]], np.deg2rad([-150, 20]))
  assert m.jnt_stiffness[j["abdomen_z"]] == 20 and m.jnt_stiffness[j["ankle_y_right"]] == 6
  assert m.dof_damping[m.jnt_dofadr[j["hip_x_left"]]] == 5 and m.dof_damping[m.jnt_dofadr[j["knee_left"]]] == 0.2
  np.testing.assert_allclose(m.jnt_solimp[j["knee_left"]], [0, 0.99, 0.01, 0.5, 2])
  g = m.geom_names.index("torso")
  np.testing.assert_allclose(m.geom_friction[g], [0.7, 0.005, 0.0001])
  np.testing.assert_allclose(m.geom_solimp[g], [0.9, 0.99, 0.003, 0.5, 2])
  assert m.geom_condim[g] == 1 and m.geom_condim[0] == 3
  # freejoint ignores joint defaults
  assert m.jnt_stiffness[0] == 0 and m.dof_damping[0] == 0 and m.dof_armature[0] == 0 and not m.jnt_limited[0]


def test_put_model_and_make_data_on_cpu():
  import torch

  import mujoco_warp_amd as mjw

  mjm = humanoid_model()
  m = mjw.put_model(mjm, device="cpu")
  assert m.nv_pad == 28 and m.nxn == 161 and m.nlimited == 21 and m.nJmom == 21
  assert m.body_mass.shape == (1, 17) and m.opt.timestep.shape == (1,)
  d = mjw.make_data(mjm, nworld=3, nconmax=24, njmax=64, device="cpu", m=m)
  assert d.qpos.shape == (3, 28) and d.efc.J.shape == (3, 64, 28) and d.qM.shape == (3, 28, 28)
  assert d.contact.dist.shape == (72,) and d.contact.efc_address.shape == (72, 4)
  np.testing.assert_allclose(d.qpos[0].numpy(), mjm.qpos0, atol=1e-6)
  # the C views carry the tensors' pointers
  cm = mjw.io.cmodel(m)
  assert cm.nv == 27 and cm.body_mass == m.body_mass.data_ptr() and cm.body_mass_nb == 1
  cd = mjw.io.cdata(d)
  assert cd.nworld == 3 and cd.qpos == d.qpos.data_ptr()
  # no CPU fallback on the product path
  with pytest.raises(RuntimeError, match="ROCm"):
    mjw.step(m, d)


def test_put_data_keyframe_and_overrides():
  import mujoco_warp_amd as mjw

  mjm = mjw.load_model(HUMANOID)
  mjw.override_model(mjm, ["opt.solver=CG", "opt.iterations=7"])
  assert mjm.opt.solver == 1 and mjm.opt.iterations == 7
  mjd = mjw.MjData(mjm)
  mjw.reset_data_keyframe(mjm, mjd, 0)
  d = mjw.put_data(mjm, mjd, nworld=2, nconmax=24, njmax=64, device="cpu")
  np.testing.assert_allclose(d.qpos[1].numpy(), mjm.key_qpos[0], atol=1e-6)
  with pytest.raises(ValueError):
    mjw.make_data(mjm, nworld=0, device="cpu")


def test_batched_model_fields_accepted():
  import torch

  import mujoco_warp_amd as mjw

  mjm = humanoid_model()
  m = mjw.put_model(mjm, device="cpu")
  m.body_mass = m.body_mass.repeat(4, 1).contiguous()
  m.opt.gravity = torch.tensor([[0, 0, -9.81], [0, 0, -1.62], [0, 0, -3.7], [0, 0, 0]], dtype=torch.float32)
  cm = mjw.io.cmodel(m)
  assert cm.body_mass_nb == 4 and cm.opt_gravity_nb == 4 and cm.body_mass_cnt == 17


def test_unsupported_features_raise():
  """Features outside this build raise NotImplementedError at put_model / the compiler, as the reference's
  io.py:89-144 does (every pair of the collision table is supported since round 4, heightfields included:
  tests/test_hfield.py)."""
  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  for flags in ("<flag override=\"enable\"/>", "<flag fwdinv=\"enable\"/>", "<flag midphase=\"disable\"/>"):
    try:
      m = mjcf.load_model_from_string(f'<mujoco><option>{flags}</option><worldbody><body><freejoint/><geom size=".1"/></body></worldbody></mujoco>')
    except (KeyError, ValueError):
      continue  # the compiler does not know the flag name
    with pytest.raises(NotImplementedError):
      mjw.put_model(m, device="cpu")
  # ellipsoids and cylinders collide with everything of the table now (tests/test_collision_types.py)
  ell = mjcf.load_model_from_string('<mujoco><worldbody><geom type="plane" size="1 1 .1"/><body><freejoint/><geom type="ellipsoid" size=".1 .1 .2"/></body>'
                                    '<body pos=".3 0 0"><freejoint/><geom type="cylinder" size=".1 .1"/></body></worldbody></mujoco>')
  m = mjw.put_model(ell, device="cpu")
  assert m.nxn_ccd == 3  # plane-ellipsoid, plane-cylinder (pre-pass primitives) and ellipsoid-cylinder (convex)


def test_frame_childclass():
  """<frame childclass>: the frame's elements default to the class (an explicit class wins), bodies inside take
  it as their childclass, and an inner frame's childclass overrides the outer one (MJCF frame semantics)."""
  from mujoco_warp_amd import mjcf

  m = mjcf.load_model_from_string("""<mujoco><default><default class="big"><geom size=".3"/><joint damping="2"/></default>
  <default class="small"><geom size=".05"/></default></default>
  <worldbody><frame childclass="big" pos="1 0 0"><geom name="a" type="sphere"/><geom name="b" type="sphere" class="small" pos="0 1 0"/>
  <body><joint type="hinge"/><geom name="c" type="sphere" pos="0 0 1"/><frame childclass="small"><geom name="d" type="sphere" pos="0 0 2"/></frame>
  </body></frame><geom name="e" type="sphere" size=".7" pos="5 0 0"/></worldbody></mujoco>""")
  size = {n: m.geom_size[i, 0] for i, n in enumerate(m.geom_names)}
  assert (size["a"], size["b"], size["c"], size["d"], size["e"]) == (0.3, 0.05, 0.3, 0.05, 0.7)
  np.testing.assert_allclose(m.dof_damping, [2.0])
  np.testing.assert_allclose(m.geom_pos[list(m.geom_names).index("a")], [1, 0, 0])


def test_flexcomp_direct_equals_grid():
  """flexcomp type="direct" (explicit points and triangles) compiles to the same flex tables, vertex bodies
  and bending coefficients as the grid it lists (the grid's own point / triangle order)."""
  from mujoco_warp_amd import mjcf

  body = ('<edge equality="true"/><elasticity young="1e3" poisson="0.2" thickness="0.01" elastic2d="bend"/>'
          '<contact condim="3"/></flexcomp></worldbody></mujoco>')
  grid = mjcf.load_model_from_string('<mujoco><worldbody><geom type="plane" size="1 1 .1"/>'
                                     '<flexcomp name="c" type="grid" count="3 4 1" spacing=".1 .1 .1" pos="0 0 .5" mass=".6" radius=".01" dim="2">'
                                     + body)
  pts = grid.body_pos[grid.flex_vertbodyid] - np.array([0, 0, 0.5])
  tri = grid.flex_elem.reshape(-1, 3)
  direct = mjcf.load_model_from_string('<mujoco><worldbody><geom type="plane" size="1 1 .1"/>'
                                       f'<flexcomp name="c" type="direct" pos="0 0 .5" mass=".6" radius=".01" dim="2" '
                                       f'point="{" ".join(repr(float(x)) for x in pts.reshape(-1))}" element="{" ".join(str(int(x)) for x in tri.reshape(-1))}">'
                                       + body)
  for f in ("flex_edge", "flex_edgeflap", "flex_elem", "flex_elemedge", "body_pos", "body_mass"):
    np.testing.assert_array_equal(getattr(direct, f), getattr(grid, f), err_msg=f)
  for f in ("flexedge_length0", "flex_bending", "flexedge_invweight0"):
    np.testing.assert_allclose(getattr(direct, f), getattr(grid, f), rtol=1e-12, atol=1e-15, err_msg=f)
  assert direct.nflexelem == 2 * 2 * 3 and direct.neq == grid.neq


# ---- C ABI ------------------------------------------------------------------------------------
def test_header_declares_and_library_exports_every_entry_point():
  from mujoco_warp_amd import _lib

  header = open(os.path.join(ROOT, "include", "mjw_amd.h")).read()
  decls = re.findall(r"^(?:int|const char\*)\s+(mjw_[a-z_]+)\(", header, re.M)
  assert set(decls) >= {"mjw_step", "mjw_forward", "mjw_solve", "mjw_fwd_position", "mjw_euler", "mjw_ctrl_noise"}
  L = _lib.lib()
  for name in decls:
    assert hasattr(L, name), name
  assert L.mjw_abi_version() == _lib.ABI_VERSION
  assert L.mjw_sizeof_model() == ctypes.sizeof(_lib.CModel)
  assert L.mjw_sizeof_data() == ctypes.sizeof(_lib.CData)


def test_lds_budget_for_humanoid():
  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import _lib

  m = mjw.put_model(humanoid_model(), device="cpu")
  nbytes = _lib.lib().mjw_lds_bytes(mjw.io.cmodel(m), 64)
  assert 0 < nbytes <= 64 * 1024
