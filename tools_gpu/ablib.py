"""A/B runner (measurement tooling, not product code): run a script or module with another build of the
library loaded in place of openke/release/libputranse_hip.so.

  python tools_gpu/ablib.py LIB.so bench.py --workload c3 ...
  python tools_gpu/ablib.py LIB.so -m pytest tests/test_gpu_pu.py -m gpu ...

The product loader (openke/_native.py) reads no environment variable; this wrapper calls
_native.use_alternative_library() before the script imports anything that loads the library."""
import os
import runpy
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "openke-putranse_amd"))
sys.path.insert(0, REPO)


def main():
    if len(sys.argv) < 3:
        sys.exit(__doc__)
    lib = sys.argv[1]
    from openke import _native
    _native.use_alternative_library(lib)
    if sys.argv[2] == "-m":
        mod = sys.argv[3]
        sys.argv = [mod] + sys.argv[4:]
        runpy.run_module(mod, run_name="__main__", alter_sys=True)
    else:
        script = sys.argv[2]
        sys.argv = [script] + sys.argv[3:]
        runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
