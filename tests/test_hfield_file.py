"""<hfield file=...>: PNG images and MuJoCo's binary format (mjcf._read_hfield_file), and the reference's own
heightfield benchmark scene (benchmarks/apptronik_apollo/scene_hfield.xml: apollo on the 588 x 1121 PNG
terrain `hfield.png`, copied into models/ as input data).

The PNG decoder is checked against an independent decoder (PIL, a test-only dependency) on the reference's
image and on synthetic images in every supported mode; the grid follows MuJoCo's loader (grey = the first
channel, image row 0 -> the last grid row, values / 255, then the [0, 1] normalisation of all elevation data).
Under `-m gpu` the apollo heightfield scene steps on the device with its feet on the terrain, against the oracle.
"""

import os

import numpy as np
import pytest

from tests.common import ROOT, gpu_from_state, np_, oracle_from_state

APOLLO_HF = os.path.join(ROOT, "models", "apptronik_apollo", "scene_hfield.xml")
PNG = os.path.join(ROOT, "models", "apptronik_apollo", "hfield.png")


def test_png_decoder_matches_pil_on_reference_image():
  PIL = pytest.importorskip("PIL.Image")
  from mujoco_warp_amd import mjcf

  h, w, px, depth = mjcf._read_png(PNG)
  ref = np.asarray(PIL.open(PNG))
  assert (h, w, depth) == (588, 1121, 8)
  np.testing.assert_array_equal(px[:, :, 0], ref)


@pytest.mark.parametrize("mode", ["L", "I;16", "RGB", "RGBA", "LA"])
def test_png_decoder_synthetic_modes(tmp_path, mode):
  PIL = pytest.importorskip("PIL.Image")
  from mujoco_warp_amd import mjcf

  rng = np.random.default_rng(0)
  h, w = 37, 53
  # smooth gradients and noise so that PIL's adaptive filtering uses every filter type
  yy, xx = np.mgrid[0:h, 0:w]
  base = (xx * 3 + yy * 5 + rng.integers(0, 40, (h, w))) % 256
  if mode == "L":
    arr = base.astype(np.uint8)
  elif mode == "I;16":
    arr = (base.astype(np.uint16) * 257 + rng.integers(0, 200, (h, w))).astype(np.uint16)
  elif mode == "LA":
    arr = np.stack([base, 255 - base], -1).astype(np.uint8)
  else:
    arr = np.stack([base, (base * 7) % 256, (base * 13) % 256] + ([np.full((h, w), 200)] if mode == "RGBA" else []), -1).astype(np.uint8)
  p = str(tmp_path / "img.png")
  PIL.fromarray(arr, mode=mode).save(p)
  hh, ww, px, depth = mjcf._read_png(p)
  assert (hh, ww) == (h, w)
  np.testing.assert_array_equal(px.reshape(h, w, -1)[:, :, 0], arr.reshape(h, w, -1)[:, :, 0])
  # the heightfield grid: first channel (16-bit: high byte) / 255, rows flipped
  nrow, ncol, data = mjcf._read_hfield_file(p)
  first = arr.reshape(h, w, -1)[:, :, 0].astype(np.int64)
  if depth == 16:
    first >>= 8
  np.testing.assert_allclose(data.reshape(nrow, ncol), first[::-1] / 255.0)


def test_binary_hfield_file(tmp_path):
  from mujoco_warp_amd import mjcf

  grid = np.arange(12, dtype=np.float32).reshape(3, 4) / 11.0
  p = str(tmp_path / "terrain.bin")
  with open(p, "wb") as f:
    f.write(np.array([3, 4], dtype="<i4").tobytes() + grid.astype("<f4").tobytes())
  m = mjcf.load_model_from_string(f"""<mujoco><asset><hfield name="h" file="{p}" size="1 1 .1 .05"/></asset>
    <worldbody><geom type="hfield" hfield="h"/></worldbody></mujoco>""")
  assert (int(m.hfield_nrow[0]), int(m.hfield_ncol[0])) == (3, 4)
  np.testing.assert_allclose(m.hfield_data, grid.reshape(-1), atol=1e-7)


def test_apollo_hfield_scene_compiles():
  import mujoco_warp_amd as mjw

  mjm = mjw.load_model(APOLLO_HF)
  assert int(mjm.nhfield) == 1 and (int(mjm.hfield_nrow[0]), int(mjm.hfield_ncol[0])) == (588, 1121)
  assert mjm.hfield_data.min() == 0.0 and mjm.hfield_data.max() == 1.0
  m = mjw.put_model(mjm, device="cpu")
  assert m.nhfield == 1 and m.nxn_ccd > 0


def test_oracle_apollo_stands_on_terrain():
  import mujoco_warp_amd as mjw

  mjm = mjw.load_model(APOLLO_HF)
  qpos = mjm.key_qpos[0][None].copy()
  _, od = oracle_from_state(mjm, qpos, np.zeros((1, mjm.nv)), np.zeros((1, mjm.nu)), njmax=128, nconmax=32)
  od.ctrl[:] = mjm.key_ctrl[0]
  ncon = []
  for _ in range(40):
    od.step()
    ncon.append(int(od.ncon[0, 0]))
  assert np.isfinite(od.qpos).all()
  assert max(ncon) >= 4 and sum(ncon) > 40  # the feet stand on the heightfield (their box corners)
  assert od.qpos[0, 2] > 0.95  # and hold the robot up


@pytest.mark.gpu
def test_gpu_apollo_hfield_matches_oracle():
  import torch

  import mujoco_warp_amd as mjw

  mjm = mjw.load_model(APOLLO_HF)
  nworld = 4
  rng = np.random.default_rng(2)
  qpos = np.tile(mjm.key_qpos[0], (nworld, 1))
  qpos[1:, :2] += rng.uniform(-0.5, 0.5, (nworld - 1, 2))  # over other terrain cells
  z = np.zeros((nworld, mjm.nv))
  ctrl = np.tile(mjm.key_ctrl[0], (nworld, 1))
  m, d = gpu_from_state(mjm, qpos, z, ctrl, njmax=128, nconmax=32)
  _, od = oracle_from_state(mjm, qpos, z, ctrl, njmax=128, nconmax=32)
  mjw.fwd_position(m, d)
  od.fwd_position()
  torch.cuda.synchronize()
  n = int(d.nacon[0])
  wid = np_(d.contact.worldid)[:n]
  for w in range(nworld):
    sel = np.nonzero(wid == w)[0]
    no = int(od.ncon[w, 0])
    assert len(sel) == no, (w, len(sel), no)
    np.testing.assert_allclose(np.sort(np_(d.contact.dist)[sel]), np.sort(od.con_dist[w][:no]), atol=5e-5)
  for _ in range(10):
    mjw.step(m, d)
  torch.cuda.synchronize()
  assert torch.isfinite(d.qpos).all()
