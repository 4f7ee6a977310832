"""A/B tooling only: run a script with product module attributes overridden.

    python3 tools/flag_ab.py liteasr_amd.kernels.DW_DIRECT_MIN_TILES=0 [more=...] -- bench.py [args...]

Each override is MODULE.ATTR=VALUE (VALUE parsed as a Python literal); the modules are imported
and patched before the script runs as __main__ (the product has no environment switches for
these; the tests pin each on/off pair bit for bit or against the oracle)."""

import ast
import importlib
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    if "--" not in sys.argv:
        raise SystemExit(__doc__)
    k = sys.argv.index("--")
    sets, rest = sys.argv[1:k], sys.argv[k + 1:]
    sys.path.insert(0, ROOT)
    for s in sets:
        name, val = s.split("=", 1)
        mod, attr = name.rsplit(".", 1)
        m = importlib.import_module(mod)
        assert hasattr(m, attr), name
        setattr(m, attr, ast.literal_eval(val))
    sys.argv = rest
    sys.path.insert(0, os.path.dirname(os.path.abspath(rest[0])))
    runpy.run_path(rest[0], run_name="__main__")


if __name__ == "__main__":
    main()
