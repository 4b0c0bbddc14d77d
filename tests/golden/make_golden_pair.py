"""Extract the reference's explicit-<pair> known-answer tests into tests/golden/pair_kat.json (data only).

Run in the build container, where the reference tree is readable as text:
    python tests/golden/make_golden_pair.py /root/reference
The test files are parsed with `ast` as text; no reference code is imported or executed.  Sources:
  mujoco_warp/_src/collision_driver_test.py  test_contact_pair: each fixture's MJCF literal, the asserted
                                             nxn_pairid[:, 0] (all equal to a value, or an explicit array),
                                             d.nacon and the asserted contact fields (includemargin, dim,
                                             friction, solref, solreffriction, solimp) of one contact
  mujoco_warp/_src/io_test.py                test_margin_pair_box_box: a box-box <pair> with a margin, which
                                             put_model must refuse (NotImplementedError)
The tests read only the JSON (the reference does not exist on the GPU box).
"""

import ast
import json
import os
import sys


def _lit(node):
  if isinstance(node, ast.Call) and ast.unparse(node.func) == "np.array":
    return _lit(node.args[0])
  return ast.literal_eval(node)


def _fixture_xml(call):
  for kw in call.keywords:
    if kw.arg == "xml":
      return kw.value.value
  return None


def contact_pair_cases(src):
  tree = ast.parse(src)
  fn = next(n for n in ast.walk(tree) if isinstance(n, ast.FunctionDef) and n.name == "test_contact_pair")
  cases, cur = [], None
  for st in fn.body:
    if isinstance(st, ast.Assign) and isinstance(st.value, ast.Call) and ast.unparse(st.value.func) == "test_data.fixture":
      cur = dict(xml=_fixture_xml(st.value), contact={})
      cases.append(cur)
      continue
    if cur is None or not isinstance(st, ast.Expr) or not isinstance(st.value, ast.Call):
      continue
    call = st.value
    fn_name = ast.unparse(call.func)
    text = ast.unparse(call)
    if fn_name == "self.assertTrue" and "nxn_pairid" in text:
      # ((m.nxn_pairid.numpy()[:][:, 0] == V).all())
      cmp = call.args[0].func.value
      cur["pairid_all"] = _lit(cmp.comparators[0])
    elif fn_name == "np.testing.assert_equal" and "nxn_pairid" in text:
      cur["pairid"] = _lit(call.args[1])
    elif fn_name == "self.assertEqual" and "d.nacon" in text:
      cur["nacon"] = _lit(call.args[1])
    elif fn_name in ("self.assertEqual", "np.testing.assert_allclose") and "d.contact." in text:
      sub = call.args[0]  # d.contact.<field>.numpy()[i]
      field = sub.value.func.value.attr
      cur["contact_index"] = _lit(sub.slice)
      cur["contact"][field] = _lit(call.args[1])
  return cases


def margin_pair_box_box(src):
  tree = ast.parse(src)
  fn = next(n for n in ast.walk(tree) if isinstance(n, ast.FunctionDef) and n.name == "test_margin_pair_box_box")
  for n in ast.walk(fn):
    if isinstance(n, ast.Call) and ast.unparse(n.func) == "mujoco.MjModel.from_xml_string":
      return n.args[0].value
  raise RuntimeError("test_margin_pair_box_box: no MJCF literal")


def main(ref):
  src_dir = os.path.join(ref, "mujoco_warp", "_src")
  with open(os.path.join(src_dir, "collision_driver_test.py")) as f:
    cases = contact_pair_cases(f.read())
  with open(os.path.join(src_dir, "io_test.py")) as f:
    refuse = margin_pair_box_box(f.read())
  out = dict(
    source="mujoco_warp/_src/collision_driver_test.py::test_contact_pair, io_test.py::test_margin_pair_box_box",
    contact_pair=cases,
    refuse_margin_box_box=refuse,
  )
  path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pair_kat.json")
  with open(path, "w") as f:
    json.dump(out, f, indent=1)
  print(f"{len(cases)} contact_pair cases -> {path}")


if __name__ == "__main__":
  main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
