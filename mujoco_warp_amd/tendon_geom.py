"""Spatial tendon geometry on the host (fp64 numpy), for the MJCF compiler's qpos0 constants.

The device computes tendon lengths and Jacobians every step (csrc/mjw_tendon.h); the compiler needs the same
quantities once, at qpos0, for tendon_length0, the default spring lengths, tendon_invweight0 and the
actuator constants of tendon transmissions -- what MuJoCo's compiler gets from mj_setConst.  Restates
util_misc.py:30-450 (is_intersect, length_circle, wrap_circle, wrap_inside, wrap) and smooth.py:3126-3465
(site-site segments, site-geom-site wraps, pulley scaling).
"""

from __future__ import annotations

import math

import numpy as np

from .types import MJ_MAXVAL, MJ_MINVAL, WrapType


def _safe_div(x, y):
  return x / (y if y != 0 else MJ_MINVAL)


def _normalize(v):
  n = float(np.linalg.norm(v))
  return (v / n if n > 0 else np.zeros_like(v)), n


def is_intersect(p1, p2, p3, p4) -> bool:
  """util_misc.py:30-56: do segments p1-p2 and p3-p4 (2D) intersect."""
  det = (p4[1] - p3[1]) * (p2[0] - p1[0]) - (p4[0] - p3[0]) * (p2[1] - p1[1])
  if abs(det) < MJ_MINVAL:
    return False
  a = ((p4[0] - p3[0]) * (p1[1] - p3[1]) - (p4[1] - p3[1]) * (p1[0] - p3[0])) / det
  b = ((p2[0] - p1[0]) * (p1[1] - p3[1]) - (p2[1] - p1[1]) * (p1[0] - p3[0])) / det
  return 0 <= a <= 1 and 0 <= b <= 1


def length_circle(p0, p1, ind, radius) -> float:
  """util_misc.py:76-100: arc length from p0 to p1 on the circle, the long way when `ind` says so."""
  p0n, _ = _normalize(np.asarray(p0, float))
  p1n, _ = _normalize(np.asarray(p1, float))
  angle = math.acos(max(-1.0, min(1.0, float(p0n @ p1n))))
  cross = p0[1] * p1[0] - p0[0] * p1[1]
  if (cross > 0 and ind != 0) or (cross < 0 and ind == 0):
    angle = 2 * math.pi - angle
  return radius * angle


_NOWRAP = (-1.0, np.full(2, MJ_MAXVAL), np.full(2, MJ_MAXVAL))


def wrap_circle(end, side, radius):
  """util_misc.py:103-198: 2D wrap of the segment end[0:2]-end[2:4] around a circle at the origin."""
  end = np.asarray(end, float)
  side = np.asarray(side, float)
  valid_side = np.linalg.norm(side) < MJ_MAXVAL
  e0, e1 = end[:2], end[2:]
  sq0, sq1, sqr = e0 @ e0, e1 @ e1, radius * radius
  if sq0 < sqr or sq1 < sqr or radius < MJ_MINVAL:
    return _NOWRAP
  dif = e1 - e0
  dd = dif @ dif
  if dd < MJ_MINVAL:
    return _NOWRAP
  a = min(max(-(dif @ e0) / dd, 0.0), 1.0)
  tmp = a * dif + e0
  if tmp @ tmp > sqr and (not valid_side or side @ tmp >= 0):
    return _NOWRAP
  s0, s1 = math.sqrt(sq0 - sqr), math.sqrt(sq1 - sqr)
  sol00 = np.array([_safe_div(end[0] * sqr + radius * end[1] * s0, sq0), _safe_div(end[1] * sqr - radius * end[0] * s0, sq0)])
  sol01 = np.array([_safe_div(end[2] * sqr - radius * end[3] * s1, sq1), _safe_div(end[3] * sqr + radius * end[2] * s1, sq1)])
  sol10 = np.array([_safe_div(end[0] * sqr - radius * end[1] * s0, sq0), _safe_div(end[1] * sqr + radius * end[0] * s0, sq0)])
  sol11 = np.array([_safe_div(end[2] * sqr + radius * end[3] * s1, sq1), _safe_div(end[3] * sqr - radius * end[2] * s1, sq1)])
  if valid_side:
    good0 = _normalize(sol00 + sol01)[0] @ side
    good1 = _normalize(sol10 + sol11)[0] @ side
  else:
    good0 = -((sol00 - sol01) @ (sol00 - sol01))
    good1 = -((sol10 - sol11) @ (sol10 - sol11))
  if is_intersect(e0, sol00, e1, sol01):
    good0 = -10000.0
  if is_intersect(e0, sol10, e1, sol11):
    good1 = -10000.0
  if good0 > good1:
    p0, p1, ind = sol00, sol01, 0
  else:
    p0, p1, ind = sol10, sol11, 1
  if is_intersect(e0, p0, e1, p1):
    return _NOWRAP
  return length_circle(p0, p1, ind, radius), p0, p1


def wrap_inside(end, radius, maxiter=20, zinit=1.0 - 1.0e-7, tolerance=1.0e-6):
  """util_misc.py:201-323: the tangent point of an inside (sidesite within the geom) wrap, by Newton on
  asin(A z) + asin(B z) - 2 asin(z) + G = 0."""
  end = np.asarray(end, float)
  e0, e1 = end[:2], end[2:]
  len0, len1 = float(np.linalg.norm(e0)), float(np.linalg.norm(e1))
  dif = e1 - e0
  dd = dif @ dif
  if len0 <= radius or len1 <= radius or radius < MJ_MINVAL or len0 < MJ_MINVAL or len1 < MJ_MINVAL:
    return _NOWRAP
  if dd > MJ_MINVAL:
    a = -(dif @ e0) / dd
    if 0 < a < 1 and np.linalg.norm(e0 + a * dif) <= radius:
      return _NOWRAP
  pnt = _normalize(0.5 * (e0 + e1))[0] * radius
  A, B = _safe_div(radius, len0), _safe_div(radius, len1)
  cosG = _safe_div(len0 * len0 + len1 * len1 - dd, 2 * len0 * len1)
  if cosG < -1 + MJ_MINVAL:
    return -1.0, pnt, pnt
  if cosG > 1 - MJ_MINVAL:
    return 0.0, pnt, pnt
  G = math.acos(cosG)
  z = zinit
  f = math.asin(A * z) + math.asin(B * z) - 2 * math.asin(z) + G
  if f > 0:
    return 0.0, pnt, pnt
  it = 0
  while it < maxiter and abs(f) > tolerance:
    sz = z * z
    df = (A / max(MJ_MINVAL, math.sqrt(1 - sz * A * A)) + B / max(MJ_MINVAL, math.sqrt(1 - sz * B * B))
          - 2 / max(MJ_MINVAL, math.sqrt(1 - sz)))
    if df > -MJ_MINVAL:
      return 0.0, pnt, pnt
    z1 = z - _safe_div(f, df)
    if z1 > z:
      return 0.0, pnt, pnt
    z = z1
    f = math.asin(A * z) + math.asin(B * z) - 2 * math.asin(z) + G
    if f > tolerance:
      return 0.0, pnt, pnt
    it += 1
  if it >= maxiter:
    return 0.0, pnt, pnt
  if end[0] * end[3] - end[1] * end[2] > 0:
    vec, ang = e0, math.asin(z) - math.asin(A * z)
  else:
    vec, ang = e1, math.asin(z) - math.asin(B * z)
  vec = _normalize(vec)[0]
  pnt = radius * np.array([math.cos(ang) * vec[0] - math.sin(ang) * vec[1], math.sin(ang) * vec[0] + math.cos(ang) * vec[1]])
  return 0.0, pnt, pnt


def wrap(x0, x1, pos, mat, radius, geomtype, side):
  """util_misc.py:326-450: wrap the segment x0-x1 around a sphere or (infinite) cylinder of `radius` at
  pos / mat; side = a sidesite position or MJ_MAXVAL.  Returns (arc length or -1, wrap point 0, 1)."""
  nowrap = (-1.0, np.full(3, MJ_MAXVAL), np.full(3, MJ_MAXVAL))
  if geomtype not in (WrapType.SPHERE, WrapType.CYLINDER):
    return MJ_MAXVAL, np.full(3, MJ_MAXVAL), np.full(3, MJ_MAXVAL)
  mat = np.asarray(mat, float).reshape(3, 3)
  pos = np.asarray(pos, float)
  p0 = mat.T @ (np.asarray(x0, float) - pos)
  p1 = mat.T @ (np.asarray(x1, float) - pos)
  if np.linalg.norm(p0) < MJ_MINVAL or np.linalg.norm(p1) < MJ_MINVAL:
    return nowrap
  if geomtype == WrapType.SPHERE:
    axis0 = _normalize(p0)[0]
    normal, nrm = _normalize(np.cross(p0, p1))
    if nrm < MJ_MINVAL:
      ab = np.abs(axis0)
      i = 0
      if ab[1] > ab[0] and ab[1] > ab[2]:
        i = 1
      if ab[2] > ab[0] and ab[2] > ab[1]:
        i = 2
      axis1 = np.ones(3)
      axis1[i] = 0
      normal = _normalize(np.cross(axis0, axis1))[0]
    axis1 = _normalize(np.cross(normal, axis0))[0]
  else:
    axis0, axis1 = np.array([1.0, 0, 0]), np.array([0, 1.0, 0])
  end = np.array([p0 @ axis0, p0 @ axis1, p1 @ axis0, p1 @ axis1])
  side = np.asarray(side, float)
  valid_side = np.linalg.norm(side) < MJ_MAXVAL
  if valid_side:
    sidepnt = mat.T @ (side - pos)
    sproj = _normalize(np.array([sidepnt @ axis0, sidepnt @ axis1]))[0] * radius
  else:
    sproj = np.full(2, MJ_MAXVAL)
  if valid_side and np.linalg.norm(sidepnt) < radius:
    wlen, q0, q1 = wrap_inside(end, radius)
  else:
    wlen, q0, q1 = wrap_circle(end, sproj, radius)
  if wlen < 0:
    return nowrap
  r0 = axis0 * q0[0] + axis1 * q0[1]
  r1 = axis0 * q1[0] + axis1 * q1[1]
  if geomtype == WrapType.CYLINDER:
    L0 = math.sqrt((p0[0] - r0[0]) ** 2 + (p0[1] - r0[1]) ** 2)
    L1 = math.sqrt((p1[0] - r1[0]) ** 2 + (p1[1] - r1[1]) ** 2)
    r0[2] = p0[2] + (p1[2] - p0[2]) * _safe_div(L0, L0 + wlen + L1)
    r1[2] = p0[2] + (p1[2] - p0[2]) * _safe_div(L0 + wlen, L0 + wlen + L1)
    wlen = math.sqrt(wlen * wlen + (r1[2] - r0[2]) ** 2)
  return wlen, mat @ r0 + pos, mat @ r1 + pos


def pulley_scale(m):
  """io.py:491-497: 1 / divisor of the last pulley before each wrap of its tendon (else 1)."""
  s = np.ones(m.nwrap)
  for t in range(m.ntendon):
    a, n = m.tendon_adr[t], m.tendon_num[t]
    for p in range(a, a + n):
      if m.wrap_type[p] == WrapType.PULLEY:
        s[p : a + n] = 1.0 / m.wrap_prm[p]
  return s


def tendon_length_jac(m, t, site_xpos, site_body, geom_xpos, geom_xmat, jac_point):
  """Length and dense Jacobian (nv,) of tendon t (smooth.py:3087-3465).  jac_point(point, body) -> (3, nv)
  translational Jacobian of a point rigidly attached to `body`."""
  a, n = int(m.tendon_adr[t]), int(m.tendon_num[t])
  wt, wo, wp_ = m.wrap_type, m.wrap_objid, m.wrap_prm
  if wt[a] == WrapType.JOINT:
    raise ValueError("fixed tendon: length / Jacobian are the wrap coefficients")
  J = np.zeros(m.nv)
  L = 0.0
  scale = pulley_scale(m)

  def seg(p0, b0, p1, b1, sc):
    v, ln = _normalize(p1 - p0)
    if ln < MJ_MINVAL:
      v = np.array([1.0, 0, 0])
    if b0 != b1:
      J[:] += sc * (v @ (jac_point(p1, b1) - jac_point(p0, b0)))
    return ln

  j = 0
  while j < n - 1:
    t0, t1 = wt[a + j], wt[a + j + 1]
    if t0 == WrapType.PULLEY or t1 == WrapType.PULLEY:
      j += 1
      continue
    s0 = wo[a + j]
    p0, b0 = site_xpos[s0], site_body[s0]
    if t1 in (WrapType.SPHERE, WrapType.CYLINDER):
      g, s1 = wo[a + j + 1], wo[a + j + 2]
      p1, b1 = site_xpos[s1], site_body[s1]
      gb = m.geom_bodyid[g]
      sc = scale[a + j + 1]
      side_id = int(round(wp_[a + j + 1]))
      side = site_xpos[side_id] if side_id >= 0 else np.full(3, MJ_MAXVAL)
      wlen, g0, g1 = wrap(p0, p1, geom_xpos[g], geom_xmat[g], m.geom_size[g][0], t1, side)
      if wlen >= 0:
        l0 = seg(p0, b0, g0, gb, sc)
        l1 = seg(g1, gb, p1, b1, sc)
        L += (l0 + wlen + l1) * sc
      else:
        L += seg(p0, b0, p1, b1, sc) * sc
      j += 2
    else:
      s1 = wo[a + j + 1]
      sc = scale[a + j]
      L += seg(p0, b0, site_xpos[s1], site_body[s1], sc) * sc
      j += 1
  return L, J
