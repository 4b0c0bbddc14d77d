"""Per-field error report of the HIP path against the fp64 oracle on the C3 / C4 / C5 models (GPU box);
the report itself lives in tests/parity_models.py.
usage: python tools/parity_models.py [out.json] [model ...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tests.parity_models import report  # noqa: E402


def main():
  path = sys.argv[1] if len(sys.argv) > 1 else None
  names = sys.argv[2:] or ["franka", "franka_dense", "apollo", "cloth", "aloha"]
  res = {}
  for n in names:
    res[n] = report(n)
    print(n, json.dumps(res[n])[:400], flush=True)
  js = json.dumps(res, indent=1)
  if path:
    with open(path, "w") as f:
      f.write(js)
  print(js)


if __name__ == "__main__":
  main()
