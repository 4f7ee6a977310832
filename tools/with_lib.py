"""A/B tooling only: run a script against another build of libliteasr_hip.so.

    python3 tools/with_lib.py LIB script.py [args...]

The product loader (liteasr_amd/_native.py) has a single path, the in-tree library.  This
wrapper points that module's LIB_PATH at LIB before the script imports anything that loads
it, then runs the script as __main__ (LITEASR_HIP_LIB is set to LIB only as a label for the
tools that print which library they ran)."""

import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    if len(sys.argv) < 3:
        raise SystemExit(__doc__)
    lib, script = os.path.abspath(sys.argv[1]), sys.argv[2]
    if not os.path.exists(lib):
        raise SystemExit(f"with_lib: {lib} does not exist")
    sys.path.insert(0, ROOT)
    from liteasr_amd import _native

    if _native._lib is not None:
        raise SystemExit("with_lib: the library is already loaded")
    _native.LIB_PATH = lib
    os.environ["LITEASR_HIP_LIB"] = lib
    sys.argv = sys.argv[2:]
    sys.path.insert(0, os.path.dirname(os.path.abspath(script)))
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
