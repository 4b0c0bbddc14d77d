"""Builds A/B variants of libmjw_amd.so that differ in one translation unit's -D switches.

The other sources are compiled once; each variant's TU is compiled with its defines, all in parallel, and
linked to mujoco_warp_amd/libmjw_amd_<name>.so (bench / tests load one with MJW_LIB_PATH).
usage: python tools/build_variants.py SOURCE name=DEF1,DEF2 [name=...]
  e.g. python tools/build_variants.py mjw_sparse.hip jt1=MJW_SP_JTPF=1 tree0=MJW_SP_TREE=0
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mujoco_warp_amd import build  # noqa: E402

src_name = sys.argv[1]
variants = [a.split("=", 1) for a in sys.argv[2:]]
flags = [f"--offload-arch={build.ARCH}", "-O3", "-std=c++17", "-ffp-contract=on", "-fPIC", "-I", os.path.join(ROOT, "include")]
tmp = tempfile.mkdtemp(prefix="mjw_var_")
procs, common = [], []
for src in build.SOURCES:
  if os.path.basename(src) == src_name:
    continue
  obj = os.path.join(tmp, os.path.basename(src) + ".o")
  procs.append(subprocess.Popen(["hipcc"] + flags + ["-c", src, "-o", obj]))
  common.append(obj)
var_objs = {}
src = [s for s in build.SOURCES if os.path.basename(s) == src_name][0]
for name, defs in variants:
  obj = os.path.join(tmp, f"{src_name}.{name}.o")
  d = [f"-D{x}" for x in defs.split(",") if x]
  procs.append(subprocess.Popen(["hipcc"] + flags + d + ["-c", src, "-o", obj]))
  var_objs[name] = obj
if any(p.wait() != 0 for p in procs):
  raise SystemExit("hipcc failed")
for name, obj in var_objs.items():
  out = os.path.join(ROOT, "mujoco_warp_amd", f"libmjw_amd_{name}.so")
  subprocess.run(["hipcc", f"--offload-arch={build.ARCH}", "-shared", "-fPIC", "-o", out] + common + [obj], check=True)
  print(out)
