"""Builds libmjw_amd.so in-tree with hipcc for gfx950 (`python -m mujoco_warp_amd.build`)."""

import os
import subprocess
import sys

_PKG = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_PKG)
SOURCES = [os.path.join(_PKG, "csrc", n) for n in ("mjw_step.hip", "mjw_dense.hip", "mjw_sensor.hip", "mjw_rk4.hip", "mjw_sparse.hip", "mjw_kat.hip")]
# every header next to the sources (a hand-kept list once missed mjw_trn.h, so sources_hash() and
# needs_build() did not see edits to the transmission code)
HEADERS = sorted(os.path.join(_PKG, "csrc", n) for n in os.listdir(os.path.join(_PKG, "csrc")) if n.endswith(".h"))
HEADERS += [os.path.join(_ROOT, "include", "mjw_amd.h")]
OUT = os.path.join(_PKG, "libmjw_amd.so")
ARCH = os.environ.get("MJW_OFFLOAD_ARCH", "gfx950")


def sources_hash():
  """Short sha256 over the kernel sources and headers: binds a committed rocprof summary to the build it
  was taken on (bench.py reports PMC traffic only when the hashes agree)."""
  import hashlib

  h = hashlib.sha256()
  for p in sorted(SOURCES + HEADERS):
    with open(p, "rb") as f:
      h.update(os.path.basename(p).encode() + b"\0" + f.read())
  return h.hexdigest()[:16]


def needs_build():
  if not os.path.exists(OUT):
    return True
  t = os.path.getmtime(OUT)
  return any(os.path.getmtime(p) > t for p in SOURCES + HEADERS)


def build(force=False, verbose=False, out=None, defines=(), extra_flags=()):
  """Compile SOURCES into `out` (default libmjw_amd.so); `defines` e.g. ("MJW_PROFILE",); `extra_flags`
  e.g. ("-gline-tables-only",) for a PC-sampling build (same code, source line tables)."""
  OUT_ = out or OUT
  if out is None and not force and not needs_build():
    return OUT
  # one object per translation unit, compiled in parallel, then linked
  flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=on", "-fPIC", "-I", os.path.join(_ROOT, "include")]
  flags += [f"-D{x}" for x in defines] + list(extra_flags)
  tag = "_".join(defines).lower() + ("_x" if extra_flags else "")
  objs, procs = [], []
  for src in SOURCES:
    obj = os.path.join(_PKG, "csrc", os.path.basename(src) + tag + ".o")
    cmd = ["hipcc"] + flags + ["-c", src, "-o", obj]
    if verbose:
      print(" ".join(cmd))
    procs.append(subprocess.Popen(cmd))
    objs.append(obj)
  if any(p.wait() != 0 for p in procs):
    raise RuntimeError("hipcc failed")
  cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT_] + objs
  if verbose:
    print(" ".join(cmd))
  subprocess.run(cmd, check=True)
  for o in objs:
    os.remove(o)
  return OUT_


if __name__ == "__main__":
  print(build(force="--force" in sys.argv, verbose=True))
