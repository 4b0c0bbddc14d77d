"""Extract the reference's own known-answer vectors into tests/golden/*.json (data only).

Run in the build container, where the reference tree is readable as text:
    python tests/golden/make_golden.py /root/reference
It parses the literal inputs/expected outputs of
  mujoco_warp/_src/math_test.py:27-126  (closest segment-segment points, triangular index maps)
and writes tests/golden/math_kat.json.  No reference code is imported or executed; the tests
read only the JSON (the reference does not exist on the GPU box).
"""

import ast
import json
import os
import re
import sys


def _vecs(src):
  return [ast.literal_eval(v) for v in re.findall(r"wp\.vec3\((\[[^\]]*\])\)", src)]


def main(ref):
  path = os.path.join(ref, "mujoco_warp", "_src", "math_test.py")
  text = open(path).read()
  cases = []
  # each closest-points test: four wp.vec3 inputs then two assertSequenceAlmostEqual(expected, places)
  for m in re.finditer(r"  def (test_\w+)\(self\):(.*?)(?=\n  def |\nclass |\Z)", text, re.S):
    name, body = m.group(1), m.group(2)
    if "closest_segment_to_segment_points" not in body:
      continue
    v = _vecs(body)
    exp = re.findall(r"assertSequenceAlmostEqual\(best_([ab]), (\[[^\]]*\]), (\d+)\)", body)
    want = {k: (ast.literal_eval(e), int(p)) for k, e, p in exp}
    line = text[: m.start()].count("\n") + 1
    cases.append(dict(name=name, source=f"math_test.py:{line}", a0=v[0], a1=v[1], b0=v[2], b1=v[3],
                      best_a=want["a"][0], best_b=want["b"][0], places=min(want["a"][1], want["b"][1])))
  tri = []
  for m in re.finditer(r"  def (test_upper_trid?_index\w*)\(self\):(.*?)(?=\n  def |\nclass |\Z)", text, re.S):
    name, body = m.group(1), m.group(2)
    line = text[: m.start()].count("\n") + 1
    r = re.search(r"list\(range\(0, (\d+)\)\)", body)
    n = re.search(r"for i in range\((\d+)\)", body)
    if r and n:
      tri.append(dict(name=name, source=f"math_test.py:{line}", fn="upper_trid_index" if "trid" in name else "upper_tri_index",
                      n=int(n.group(1)), count=int(r.group(1))))
    s = re.search(r"upper_trid_index\((\d+), (\d+), (\d+)\), upper_trid_index\((\d+), (\d+), (\d+)\)", body)
    if s:
      tri.append(dict(name=name + "_symmetric", source=f"math_test.py:{line}", fn="upper_trid_index_sym",
                      args=[int(x) for x in s.groups()]))
  out = dict(generated_by="tests/golden/make_golden.py", reference="mujoco_warp/_src/math_test.py",
             closest_segment_points=cases, triangular_index=tri)
  dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "math_kat.json")
  with open(dst, "w") as f:
    json.dump(out, f, indent=1)
  print(f"wrote {dst}: {len(cases)} closest-point cases, {len(tri)} index cases")


if __name__ == "__main__":
  main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
