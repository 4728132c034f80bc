#!/usr/bin/env python
"""Build a TIMING-PROBE variant of the native extension into a scratch directory.

The probes skip work inside the MNIST step kernels (wrong numerics) to time what that work
costs; they exist only as compile-time macros of csrc/kernels/convnet_step2.hip
(DAMD_PROBE_HACC=1|2, DAMD_PROBE_HCONV=1), never in the product build.  Usage:

    python scripts/probe_build.py /tmp/probe DAMD_PROBE_HACC=1
    PYTHONPATH=/tmp/probe_pkg ...   # see the printed instructions

The variant's _C.so lands in OUT/distributed_amd_probe/ ; load it only from a probe script
(bench.py refuses to run with any DAMD_PROBE_* set, so a probe number never reaches a
benchmark line).
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from distributed_amd import _build  # noqa: E402


def main():
    if len(sys.argv) < 3:
        print(__doc__)
        sys.exit(2)
    out = Path(sys.argv[1]).resolve() / "distributed_amd_probe"
    out.mkdir(parents=True, exist_ok=True)
    defines = [d for d in sys.argv[2:] if d.startswith("DAMD_PROBE_")]
    if not defines:
        sys.exit("only DAMD_PROBE_* defines are accepted")
    so = _build._build_C(verbose=True, defines=defines, out_dir=out)
    print("probe extension:", so)


if __name__ == "__main__":
    main()
