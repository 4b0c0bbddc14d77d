"""Extract the reference's collision known-answer tests into tests/golden/collision_kat.json (data only).

Run in the build container, where the reference tree is readable as text:
    python tests/golden/make_golden_collision.py /root/reference
The test files are parsed with `ast` as text; no reference code is imported or executed.  Sources:
  mujoco_warp/_src/collision_gjk_test.py            GJKTest: MJCF scene literal, optional geom poses
                                                    (wp.vec3 / wp.mat33 literals), _geom_dist arguments
                                                    and the assertEqual / assertAlmostEqual / assertLess
                                                    checks on dist, ncon, witness points and normal
  mujoco_warp/_src/collision_primitive_core_test.py sphere / box / capsule / cylinder vs triangle cases:
                                                    literal inputs and their checks on dist / normal
  mujoco_warp/_src/broadphase_test.py               NXN broadphase pair counts (d.ncollision): scene,
                                                    keyframe(s), broadphase_filter, disableflags and the
                                                    expected count of every assertion
The tests read only the JSON (the reference does not exist on the GPU box).
"""

import ast
import json
import os
import re
import sys


def _lit(node, env):
  """Literal value of an AST node: constants, +/- numbers, lists/tuples, np.array([...]), np.eye(3),
  wp.vec3(...) / wp.mat33(...) of literals, names bound earlier in the same test, and simple + - * /
  arithmetic of those (e.g. `0.5 - sphere_radius`)."""
  if isinstance(node, ast.Constant):
    return node.value
  if isinstance(node, ast.UnaryOp) and isinstance(node.op, ast.USub):
    return -_lit(node.operand, env)
  if isinstance(node, (ast.List, ast.Tuple)):
    return [_lit(e, env) for e in node.elts]
  if isinstance(node, ast.Name):
    if node.id in env:
      return env[node.id]
    raise ValueError(node.id)
  if isinstance(node, ast.BinOp):
    a, b = _lit(node.left, env), _lit(node.right, env)
    ops = {ast.Add: lambda x, y: x + y, ast.Sub: lambda x, y: x - y, ast.Mult: lambda x, y: x * y, ast.Div: lambda x, y: x / y}
    f = ops[type(node.op)]
    if isinstance(a, list) and isinstance(b, list):
      return [f(x, y) for x, y in zip(a, b)]
    if isinstance(a, list) or isinstance(b, list):
      raise ValueError("mixed vector arithmetic")
    return f(a, b)
  if isinstance(node, ast.Call):
    fn = ast.unparse(node.func)
    if fn in ("wp.vec3", "wp.mat33", "np.array"):
      args = [_lit(a, env) for a in node.args]
      if len(args) == 1 and isinstance(args[0], list):
        return [float(x) for x in args[0]]
      return [float(x) for x in args]
    if fn == "np.linalg.norm":
      v = _lit(node.args[0], env)
      return sum(x * x for x in v) ** 0.5
    if fn == "np.eye" and _lit(node.args[0], env) == 3:
      return [1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0]
  raise ValueError(ast.unparse(node))


def _quantity(node, outs):
  """A checked quantity: dist / ncon / x1[i] / x2[i] / normal[i] / dist[i] (by the test's own names)."""
  if isinstance(node, ast.Name) and node.id in outs:
    return [outs[node.id], None]
  if isinstance(node, ast.Subscript) and isinstance(node.value, ast.Name) and node.value.id in outs:
    return [outs[node.value.id], int(_lit(node.slice, {}))]
  return None


def _checks(fn, outs, env):
  """assert* calls comparing a quantity with a literal (either order)."""
  out = []
  for node in ast.walk(fn):
    if not (isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute)):
      continue
    name = node.func.attr
    args = node.args
    if name in ("assertEqual", "assertAlmostEqual", "assertLess", "assertGreater") and len(args) >= 2:
      q, val, flip = _quantity(args[0], outs), None, False
      if q is None:
        q, flip = _quantity(args[1], outs), True
        other = args[0]
      else:
        other = args[1]
      if q is None:
        continue
      try:
        val = _lit(other, env)
      except ValueError:
        continue
      places = 7
      if len(args) > 2:
        places = int(_lit(args[2], env))
      for kw in node.keywords:
        if kw.arg == "places":
          places = int(_lit(kw.value, env))
      op = {"assertEqual": "eq", "assertAlmostEqual": "almost", "assertLess": "lt", "assertGreater": "gt"}[name]
      if flip and op in ("lt", "gt"):
        op = {"lt": "gt", "gt": "lt"}[op]
      c = dict(quantity=q[0], index=q[1], op=op, value=val, line=node.lineno)
      if op == "almost":
        c["places"] = places
      out.append(c)
    elif name == "assert_allclose" or (isinstance(node.func, ast.Attribute) and ast.unparse(node.func).endswith("assert_allclose")):
      q = _quantity(args[0], outs)
      if q is None:
        continue
      try:
        val = _lit(args[1], env)
      except ValueError:
        continue
      atol = 1e-7
      for kw in node.keywords:
        if kw.arg == "atol":
          atol = float(_lit(kw.value, env))
      out.append(dict(quantity=q[0], index=q[1], op="allclose", value=val, atol=atol, line=node.lineno))
  return out


def gjk_cases(ref):
  path = os.path.join(ref, "mujoco_warp", "_src", "collision_gjk_test.py")
  text = open(path).read()
  lines = text.splitlines()
  tree = ast.parse(text)
  cases, skipped = [], []
  for cls in [n for n in tree.body if isinstance(n, ast.ClassDef)]:
    for fn in [n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name.startswith("test_")]:
      if fn.decorator_list:  # parameterized helper-level tests (support functions, hfield) need Warp internals
        skipped.append(fn.name)
        continue
      xml, overrides, env, call, targets = None, [], {}, None, None
      for st in ast.walk(fn):
        if isinstance(st, ast.Call) and ast.unparse(st.func) == "test_data.fixture":
          for kw in st.keywords:
            if kw.arg == "xml":
              xml = _lit(kw.value, env)
            if kw.arg == "overrides":
              overrides = _lit(kw.value, env)
      for st in fn.body:
        if isinstance(st, ast.Assign) and len(st.targets) == 1:
          t = st.targets[0]
          if isinstance(t, ast.Name):
            try:
              env[t.id] = _lit(st.value, env)
            except ValueError:
              pass
          elif isinstance(t, ast.Tuple) and isinstance(st.value, ast.Call) and ast.unparse(st.value.func) == "_geom_dist":
            call, targets = st.value, [e.id if isinstance(e, ast.Name) else "_" for e in t.elts]
      if xml is None or call is None:
        skipped.append(fn.name)
        continue
      pos = [_lit(a, env) for a in call.args[2:]]
      kw = {k.arg: k.value for k in call.keywords}
      args = dict(gid1=pos[0], gid2=pos[1], multiccd=bool(pos[2]) if len(pos) > 2 else False, margin=0.0)
      if len(pos) > 3:
        args["margin"] = float(pos[3])
      for k, v in kw.items():
        if k in ("multiccd",):
          args[k] = bool(_lit(v, env))
        elif k == "margin":
          args[k] = float(_lit(v, env))
        elif k in ("pos1", "pos2", "mat1", "mat2"):
          args[k] = _lit(v, env)
      # the helper returns (dist, ncon, x1, x2); the test's names for them
      outs = {n: q for n, q in zip(targets, ("dist", "ncon", "x1", "x2")) if n != "_"}
      if "x1" in outs.values() and "x2" in outs.values() and "normal" in ast.unparse(fn):
        outs["normal"] = "normal"  # normal = (x1 - x2) / |x1 - x2| (test_box_box_contact)
      checks = _checks(fn, outs, env)
      # a trailing "# dist = <value> - MJC 64 bit precision" comment records MuJoCo C's fp64 answer
      for c in checks:
        m = re.search(r"#\s*dist\s*=\s*([-+0-9.eE]+)\s*-\s*MJC 64 bit", lines[c["line"] - 1])
        if m:
          c["mjc64"] = float(m.group(1))
      cases.append(dict(name=fn.name, source=f"collision_gjk_test.py:{fn.lineno}", xml=xml, overrides=overrides, **args, checks=checks))
  return cases, skipped


def triangle_cases(ref):
  path = os.path.join(ref, "mujoco_warp", "_src", "collision_primitive_core_test.py")
  tree = ast.parse(open(path).read())
  kinds = {"SphereTriangleTest": "sphere", "BoxTriangleTest": "box", "CapsuleTriangleTest": "capsule", "CylinderTriangleTest": "cylinder"}
  cases = []
  for cls in [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name in kinds]:
    kind = kinds[cls.name]
    for fn in [n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name.startswith("test_")]:
      env, outs = {"collision_primitive_core.MJ_MAXVAL": 1e10}, {}
      call = None
      for st in fn.body:
        if isinstance(st, ast.Assign) and len(st.targets) == 1:
          t = st.targets[0]
          if isinstance(t, ast.Name):
            try:
              env[t.id] = _lit(st.value, env)
            except ValueError:
              pass
          elif isinstance(t, ast.Tuple) and isinstance(st.value, ast.Call) and ast.unparse(st.value.func).startswith("self._run_"):
            call = st.value
            outs = {e.id: q for e, q in zip(t.elts, ("dist", "pos", "normal")) if isinstance(e, ast.Name) and e.id != "_"}
      if call is None:
        continue
      vals = [_lit(a, env) for a in call.args]
      if kind == "sphere":
        rec = dict(center=vals[0], radius=vals[1], t=vals[2:5], tri_radius=vals[5])
      elif kind == "box":
        rec = dict(center=vals[0], rot=vals[1], size=vals[2], t=vals[3:6], tri_radius=vals[6])
      else:
        rec = dict(center=vals[0], axis=vals[1], radius=vals[2], half=vals[3], t=vals[4:7], tri_radius=vals[7])
      env2 = dict(env)
      env2["collision_primitive_core.MJ_MAXVAL"] = 1e10
      checks = _checks(fn, outs, env2)
      # `assertLess(dist[0], collision_primitive_core.MJ_MAXVAL)`: an attribute, resolved here
      for node in ast.walk(fn):
        if isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute) and node.func.attr in ("assertLess", "assertGreater"):
          if "MJ_MAXVAL" in ast.unparse(node.args[1]):
            q = _quantity(node.args[0], outs)
            checks.append(dict(quantity=q[0], index=q[1], op="lt", value=1e10, line=node.lineno))
      cases.append(dict(name=f"{cls.name}.{fn.name}", kind=kind, source=f"collision_primitive_core_test.py:{fn.lineno}", **rec, checks=checks))
  return cases


_FILTER = {"PLANE": 1, "SPHERE": 2, "AABB": 4, "OBB": 8}  # types.BroadphaseFilter
_DISABLE = {"FILTERPARENT": 1 << 10}  # types.DisableBit


def _flags(node, env):
  """BroadphaseFilter / DisableBit expressions: X.NAME, names bound to them, `|` combinations."""
  if isinstance(node, ast.BinOp) and isinstance(node.op, ast.BitOr):
    return _flags(node.left, env) | _flags(node.right, env)
  if isinstance(node, ast.Attribute):
    base = ast.unparse(node.value)
    if base.endswith("BroadphaseFilter"):
      return _FILTER[node.attr]
    if base.endswith("DisableBit"):
      return _DISABLE[node.attr]
    if base in ("self", "BroadphaseTest"):
      return env[node.attr]
  if isinstance(node, ast.Name):
    return env[node.id]
  if isinstance(node, ast.Constant):
    return int(node.value)
  raise ValueError(ast.unparse(node))


def broadphase_cases(ref):
  """broadphase_test.py: NXN broadphase pair counts (d.ncollision) per scene / keyframe / filter."""
  path = os.path.join(ref, "mujoco_warp", "_src", "broadphase_test.py")
  tree = ast.parse(open(path).read())
  cls = [n for n in tree.body if isinstance(n, ast.ClassDef)][0]
  env = {}
  for st in cls.body:  # class-level filter combinations
    if isinstance(st, ast.Assign) and isinstance(st.targets[0], ast.Name):
      env[st.targets[0].id] = _flags(st.value, env)
  cases = []
  for fn in [n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name.startswith("test_")]:
    local = dict(env)
    params = [{}]
    for dec in fn.decorator_list:
      if not isinstance(dec, ast.Call):
        continue
      name = ast.unparse(dec.func)
      argnames = [a.arg for a in fn.args.args[1:]]
      if name.endswith("parameters"):
        params = [dict(zip(argnames, [(_flags(e, local) if isinstance(e, (ast.Attribute, ast.BinOp)) else _lit(e, local)) for e in t.elts]))
                  for t in dec.args]
      elif name.endswith("product"):
        for kw in dec.keywords:
          if kw.arg == "filter":
            params = [dict(filter=_flags(e, local)) for e in kw.value.elts]
    for prm in params:
      xmlvars, keyof, filt, disable, contype0, pending = {}, {}, None, 0, None, None
      for st in fn.body:
        if isinstance(st, ast.Assign) and isinstance(st.targets[0], ast.Name) and isinstance(st.value, (ast.Attribute, ast.BinOp)):
          try:  # local filter names (plane = BroadphaseFilter.PLANE, plane_sphere = plane | sphere)
            local[st.targets[0].id] = _flags(st.value, local)
          except (ValueError, KeyError):
            pass
        if isinstance(st, ast.Assign) and isinstance(st.targets[0], ast.Name):
          if isinstance(st.value, ast.Constant) and isinstance(st.value.value, str):
            xmlvars[st.targets[0].id] = st.value.value
          elif isinstance(st.value, ast.JoinedStr):  # f-string scene with the test parameters
            parts = [v.value if isinstance(v, ast.Constant) else str(prm[ast.unparse(v.value)]) for v in st.value.values]
            xmlvars[st.targets[0].id] = "".join(parts)
        if isinstance(st, ast.Assign) and isinstance(st.value, ast.Call) and ast.unparse(st.value.func) == "test_data.fixture":
          kw = {k.arg: k.value for k in st.value.keywords}
          xml = xmlvars[kw["xml"].id]
          key = int(_lit(kw["keyframe"], {})) if "keyframe" in kw else 0
          if "overrides" in kw:
            disable = int(prm[ast.unparse(kw["overrides"].values[0])])
          names = [e.id for e in st.targets[0].elts if isinstance(e, ast.Name)]
          for n in names:
            keyof[n] = key
          contype0 = None
          pending = dict(xml=xml, keys=[key])
        if isinstance(st, ast.Assign) and isinstance(st.targets[0], ast.Attribute) and ast.unparse(st.targets[0]).endswith("opt.broadphase_filter"):
          filt = _flags(st.value, local) if not isinstance(st.value, ast.Name) else prm.get(st.value.id, local.get(st.value.id))
        if isinstance(st, ast.Assign) and isinstance(st.targets[0], ast.Subscript) and ast.unparse(st.targets[0]).endswith("geom_contype[:3]"):
          contype0 = int(_lit(st.value, {}))
        if isinstance(st, ast.Assign) and isinstance(st.value, ast.Call) and ast.unparse(st.value.func) == "mjw.make_data":
          # two worlds whose geom frames come from two keyframes' mjData (np.vstack of mjdA / mjdB)
          pass
        if isinstance(st, ast.Assign) and ast.unparse(st.targets[0]).endswith("geom_xpos") and "vstack" in ast.unparse(st.value):
          srcs = [n.id for n in ast.walk(st.value) if isinstance(n, ast.Name) and n.id.startswith("mjd")]
          pending = dict(xml=pending["xml"], keys=[keyof[n] for n in srcs])
        if isinstance(st, ast.Expr) and isinstance(st.value, ast.Call):
          call = st.value
          fname = ast.unparse(call.func)
          if (fname.endswith("assert_allclose") or fname.endswith("assertEqual")) and "ncollision" in ast.unparse(call.args[0]):
            want = int(_lit(call.args[1], dict(local, **prm)))
            if fname.endswith("assert_allclose") and not isinstance(call.args[1], ast.Constant) and not isinstance(call.args[1], ast.Name):
              continue
            case = dict(name=f"{fn.name}", source=f"broadphase_test.py:{call.lineno}", xml=pending["xml"], keys=pending["keys"],
                        filter=filt if filt is not None else prm.get("filter", 1 | 2 | 8), disableflags=disable, ncollision=want)
            if contype0 is not None:
              case["geom_contype_first3"] = contype0
            if fn.name == "test_broadphase" and case["filter"] is None:
              case["filter"] = prm["filter"]
            cases.append(case)
  return cases


def main(ref):
  gjk, skipped = gjk_cases(ref)
  tri = triangle_cases(ref)
  bp = broadphase_cases(ref)
  out = dict(generated_by="tests/golden/make_golden_collision.py",
             reference=["mujoco_warp/_src/collision_gjk_test.py", "mujoco_warp/_src/collision_primitive_core_test.py",
                        "mujoco_warp/_src/broadphase_test.py"],
             gjk=gjk, gjk_not_extracted=skipped, triangle=tri, broadphase=bp)
  dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "collision_kat.json")
  with open(dst, "w") as f:
    json.dump(out, f, indent=1)
  print(f"wrote {dst}: {len(gjk)} gjk cases ({len(skipped)} not extracted: {skipped}), {len(tri)} triangle cases, "
        f"{len(bp)} broadphase cases")


if __name__ == "__main__":
  main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
