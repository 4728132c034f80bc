"""bench.py with the HIP device in spin-wait scheduling (hipSetDeviceFlags(hipDeviceScheduleSpin)
before torch initialises the device): does the host wake-up in torch.cuda.synchronize cost
the short timed run anything?  usage: python scripts/bench_spin.py <bench.py args>"""
import ctypes
import os
import runpy
import sys

import torch  # noqa: F401  (loads torch's libamdhip64 without initialising the device)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = next(l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l)
rc = ctypes.CDLL(lib).hipSetDeviceFlags(ctypes.c_uint(1))
print("hipSetDeviceFlags(spin) ->", rc, lib, file=sys.stderr, flush=True)
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
sys.path.insert(0, ROOT)
runpy.run_path(sys.argv[0], run_name="__main__")
