"""Device self-checks of the dense path's wave primitives (mjw_dense.hip) through the C ABI.

dsum (DPP reduction), xhalf_add (v_permlane32_swap) and spd_inverse (register Cholesky +
v_mfma_f32_32x32x2_f32 X^T X) are checked against numpy on seeded inputs; the MFMA
accumulator layout is exercised with asymmetric-in-rows data (random SPD matrices).
"""

import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(which, x, nout):
  torch = pytest.importorskip("torch")
  if not torch.cuda.is_available():
    pytest.skip("no GPU")
  from mujoco_warp_amd import _lib

  L = _lib.lib()
  n = x.shape[0]
  xin = torch.as_tensor(x, dtype=torch.float32, device="cuda").contiguous()
  out = torch.full((nout,), float("nan"), dtype=torch.float32, device="cuda")
  rc = L.mjw_selftest(which, ctypes.c_void_p(xin.data_ptr()), ctypes.c_void_p(out.data_ptr()), n, None)
  assert rc == 0, L.mjw_last_error()
  torch.cuda.synchronize()
  return out.cpu().numpy()


def test_wave_sum_and_half_swap():
  rng = np.random.default_rng(0)
  n = 256
  x = rng.normal(size=(n, 64)).astype(np.float32)
  x[0] = np.arange(64)  # exact integers: total 2016
  out = _run(0, x, n + n * 64)
  assert out[0] == 2016.0
  np.testing.assert_allclose(out[:n], x.astype(np.float64).sum(1), rtol=1e-5, atol=1e-5)
  half = out[n:].reshape(n, 64)
  want = x + np.roll(x, 32, axis=1)
  np.testing.assert_allclose(half, want, rtol=1e-6, atol=1e-6)
  assert np.array_equal(half[:, :32], half[:, 32:])


def test_spd_inverse_mfma_layout():
  rng = np.random.default_rng(1)
  n = 128
  A = rng.normal(size=(n, 32, 32))
  M = A @ A.transpose(0, 2, 1) / 32 + np.eye(32) * 0.5
  M[1] = np.diag(np.arange(1, 33, dtype=np.float64))  # diagonal: exact row/column placement
  out = _run(1, M.astype(np.float32).reshape(n, -1), n * 1024).reshape(n, 32, 32)
  np.testing.assert_allclose(np.diag(out[1]), 1.0 / np.arange(1, 33), rtol=1e-6)
  assert np.abs(out[1] - np.diag(np.diag(out[1]))).max() == 0.0
  want = np.linalg.inv(M)
  err = np.abs(out - want).max(axis=(1, 2)) / np.abs(want).max(axis=(1, 2))
  assert err.max() < 1e-4, err.max()
  assert np.array_equal(out, out.transpose(0, 2, 1))  # X^T X is bitwise symmetric


def test_spd_inverse_factor_bound_16():
  """spd_inverse with the compile-time factor bound NB = 16 (the nv <= 16 dense kernels, e.g. franka):
  matrices that are the identity past row / column 16 invert exactly as with the full 32 steps."""
  rng = np.random.default_rng(2)
  n = 64
  M = np.tile(np.eye(32), (n, 1, 1))
  for i in range(n):
    k = 1 + i % 16  # every size 1..16
    A = rng.normal(size=(k, k))
    M[i, :k, :k] = A @ A.T / k + np.eye(k) * 0.5
  x = M.astype(np.float32).reshape(n, -1)
  out16 = _run(2, x, n * 1024).reshape(n, 32, 32)
  out32 = _run(1, x, n * 1024).reshape(n, 32, 32)
  want = np.linalg.inv(M)
  err = np.abs(out16 - want).max(axis=(1, 2)) / np.abs(want).max(axis=(1, 2))
  assert err.max() < 1e-4, err.max()
  np.testing.assert_array_equal(out16[:, 16:, 16:], np.tile(np.eye(16), (n, 1, 1)))
  np.testing.assert_array_equal(out16, out32)  # the skipped steps are exact no-ops


@pytest.mark.parametrize("which,nb", [(3, 32), (4, 28)])
def test_ldl_solve(which, nb):
  """ldl_factor + ldl_solve (Newton's Hessian and the implicit-Euler matrix, mjw_dense.h): the solution of
  random SPD systems of every size up to the factor bound, identity-padded to 32 (as the dense kernel
  stages them), against numpy in fp64; a diagonal system is solved exactly up to the reciprocal."""
  rng = np.random.default_rng(3 + which)
  n = 96
  M = np.tile(np.eye(32), (n, 1, 1))
  b = np.zeros((n, 32))
  for i in range(n):
    k = 1 + i % nb
    A = rng.normal(size=(k, k))
    M[i, :k, :k] = A @ A.T / k + np.eye(k) * 0.3
    b[i, :k] = rng.normal(size=k)
  M[0] = np.diag(np.arange(1, 33, dtype=np.float64))
  M[0, nb:, nb:] = np.eye(32 - nb)
  b[0] = 0.0
  b[0, :nb] = np.arange(1, nb + 1)
  x = np.concatenate([M.reshape(n, -1), b], axis=1).astype(np.float32)
  out = _run(which, x, n * 32).reshape(n, 32)
  want = np.linalg.solve(M.astype(np.float32).astype(np.float64), b.astype(np.float32).astype(np.float64)[..., None])[..., 0]
  err = np.abs(out - want).max(axis=1) / np.maximum(np.abs(want).max(axis=1), 1e-30)
  assert err.max() < 1e-4, err.max()
  np.testing.assert_allclose(out[0, :nb], 1.0, rtol=5e-7)
  assert np.all(out[:, nb:] == 0.0)
