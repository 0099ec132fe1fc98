#!/usr/bin/env python
"""Run a script or module with another build of the library in place of the in-tree libvrq.so
(timing sweeps of probe variants under tools/probes/; never the product path).

  python tools/with_lib.py tools/probes/k1r/lib_x.so bench.py --config c3 --nq 64
  python tools/with_lib.py tools/probes/k1r/lib_x.so -m pytest tests -m gpu -k mfma
"""
import os
import runpy
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

from vectorragquantization_amd import _native as N  # noqa: E402

if __name__ == "__main__":
    lib, rest = sys.argv[1], sys.argv[2:]
    N.use_library(os.path.abspath(lib))
    if rest[0] == "-m":
        sys.argv = [rest[1]] + rest[2:]
        runpy.run_module(rest[1], run_name="__main__", alter_sys=True)
    else:
        sys.argv = rest
        sys.path.insert(0, os.path.dirname(os.path.abspath(rest[0])))
        runpy.run_path(rest[0], run_name="__main__")
