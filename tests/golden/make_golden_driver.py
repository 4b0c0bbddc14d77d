"""Extract the MJCF scenes of the reference's collision driver test into tests/golden/driver_fixtures.json
(data only: the scene literals of CollisionTest._FIXTURES, collision_driver_test.py:151-508).

Run in the build container, where the reference tree is readable as text:
    python tests/golden/make_golden_driver.py /root/reference
The test file is parsed with `ast` as text; nothing is imported or executed.  The reference checks these
scenes against MuJoCo C at run time (test_collision, :546-580: every MuJoCo contact found among the
MJWarp contacts, equal counts except mesh-plane), so the file holds inputs only; tests/test_collision_types.py
runs them on the oracle (analytic checks) and on the HIP path against the oracle.
"""

import ast
import json
import os
import sys


def main(ref):
  path = os.path.join(ref, "mujoco_warp", "_src", "collision_driver_test.py")
  tree = ast.parse(open(path).read())
  out = {}
  for node in ast.walk(tree):
    if isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "_FIXTURES" for t in node.targets):
      for k, v in zip(node.value.keys, node.value.values):
        out[k.value] = v.value
  dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "driver_fixtures.json")
  with open(dst, "w") as f:
    json.dump({"source": "mujoco_warp/_src/collision_driver_test.py CollisionTest._FIXTURES", "scenes": out}, f, indent=1)
  print(f"{len(out)} scenes -> {dst}")


if __name__ == "__main__":
  main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
