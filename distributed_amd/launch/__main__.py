"""CLI: python -m distributed_amd.launch --nproc N [--port-base P] [--max-restarts R]
[--timeout S] script.py [args...]  — every rank gets its TF_CONFIG (README.md:84-113)."""
import argparse
import sys

from . import launch_script


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m distributed_amd.launch")
    ap.add_argument("--nproc", "--nproc-per-node", type=int, required=True, dest="nproc")
    ap.add_argument("--port-base", type=int, default=None)
    ap.add_argument("--max-restarts", type=int, default=0)
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    res = launch_script([a.script] + a.args, a.nproc, a.port_base, a.max_restarts, a.timeout)
    if not res.ok:
        sys.stderr.write(f"[distributed_amd.launch] failed: returncodes={res.returncodes} "
                         f"after {res.attempts} attempt(s)\n")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
