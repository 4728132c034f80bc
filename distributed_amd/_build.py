"""Build the native extensions in-tree with hipcc for gfx950 (MI355X).

Two modules are produced next to this file:

* ``_C``   -- HIP kernels + RCCL communicator + hipGraph step executor (hipcc,
  ``--offload-arch=gfx950``).  It links only libamdhip64 / librccl, which torch has
  already loaded (same sonames), never libtorch.
* ``_h5``  -- Keras-HDF5 checkpoint writer/reader over the libhdf5 C API (g++).

The build is incremental (per-object mtime check) and parallel.  No hipify, no
torch.utils.cpp_extension: explicit ``hipcc -c`` / ``hipcc -shared`` lines.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
HIPCC = str(ROCM / "bin" / "hipcc")
ARCH = os.environ.get("DAMD_OFFLOAD_ARCH", "gfx950")
HDF5_PREFIX = Path(os.environ.get("DAMD_HDF5_PREFIX", "/opt/conda"))
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _pybind_includes():
    import pybind11

    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def _deps_newer(obj: Path, srcs) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(Path(s).stat().st_mtime > t for s in srcs)


def _headers():
    return list((CSRC / "include").glob("*.h")) + list((CSRC / "runtime").glob("*.h"))


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def _common_flags(defines=()):
    inc = ["-I", str(CSRC / "include"), "-I", str(CSRC / "runtime")]
    for p in _pybind_includes():
        inc += ["-I", p]
    return ["-O3", "-fPIC", "-std=c++17", "-Wno-unused-result", "-DNDEBUG"] + inc + [f"-D{d}" for d in defines]


def hip_kernel_cmd(src: Path, obj: Path, defines=(), device_asm: bool = False):
    """The hipcc line of one kernel source.  ``device_asm``: the gfx950 device assembly of
    the very same compilation (``--cuda-device-only -S``) instead of the object -- what
    scripts/check_publish_isa.py reads (it also checks that its instruction stream equals
    the shipped object's)."""
    # kernarg preloading: the first 16 argument dwords arrive in SGPRs, so a kernel's first
    # dependent load does not wait on a kernarg-segment fetch (DAMD_KERNARG_PRELOAD=0 turns
    # it off for A/B runs)
    pre = ["-mllvm", "-amdgpu-kernarg-preload-count=16"] if os.environ.get("DAMD_KERNARG_PRELOAD", "1") != "0" else []
    mode = ["--cuda-device-only", "-S"] if device_asm else ["-c"]
    return [HIPCC, f"--offload-arch={ARCH}"] + mode + [str(src), "-o", str(obj)] + _common_flags(defines) + pre


def _build_C(verbose=False, jobs=None, defines=(), out_dir: Path | None = None) -> Path:
    """``defines``/``out_dir``: a diagnostic variant (e.g. the wrong-numerics timing probes
    of convnet_step2.hip, scripts/probe_build.py) built into its own directory with its own
    objects -- never over the product extension."""
    if defines and out_dir is None:
        raise ValueError("a build with extra defines needs its own out_dir")
    out = (out_dir or PKG) / f"_C{EXT}"
    srcs = sorted((CSRC / "kernels").glob("*.hip")) + sorted((CSRC / "runtime").glob("*.cpp")) + [
        CSRC / "bindings.cpp",
        CSRC / "ops_bindings.cpp",
    ]
    common = _common_flags(defines)
    objdir = (out_dir / "obj") if out_dir is not None else BUILD / "obj"
    objdir.mkdir(parents=True, exist_ok=True)
    hdrs = _headers()
    jobs_list = []
    for s in srcs:
        o = objdir / (s.name + ".o")
        if _deps_newer(o, [s] + hdrs):
            if s.suffix == ".hip":
                cmd = hip_kernel_cmd(s, o, defines)
            else:
                cmd = [HIPCC, "-x", "hip", f"--offload-arch={ARCH}", "-c", str(s), "-o", str(o)] + common + [
                    "-fvisibility=hidden"
                ]
            jobs_list.append(cmd)
    objs = [objdir / (s.name + ".o") for s in srcs]
    if jobs_list:
        n = jobs or min(8, os.cpu_count() or 4, len(jobs_list))
        with cf.ThreadPoolExecutor(n) as ex:
            list(ex.map(lambda c: _run(c, verbose), jobs_list))
    # relink also when the object SET changed (a source added or deleted): mtimes alone
    # would keep a deleted kernel file's object inside the library
    manifest = (out_dir / "C.objs") if out_dir is not None else BUILD / "C.objs"
    listing = "\n".join(o.name for o in objs)
    if _deps_newer(out, objs) or not manifest.exists() or manifest.read_text() != listing:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(out)] + [str(o) for o in objs] + [
            "-L",
            str(ROCM / "lib"),
            "-lrccl",
            "-lamdhip64",
            f"-Wl,-rpath,{ROCM / 'lib'}",
        ]
        _run(cmd, verbose)
        manifest.write_text(listing)
    return out


H5_SOURCES = [CSRC / "io" / "keras_h5.cpp", CSRC / "io" / "h5tree.cpp"]


def hdf5_flags():
    return ["-I", str(CSRC / "io"), "-I", str(HDF5_PREFIX / "include"), "-L", str(HDF5_PREFIX / "lib"), "-lhdf5",
            f"-Wl,-rpath,{HDF5_PREFIX / 'lib'}"]


def _build_h5(verbose=False) -> Path | None:
    out = PKG / f"_h5{EXT}"
    if not H5_SOURCES[0].exists():
        return None
    if not (HDF5_PREFIX / "include" / "hdf5.h").exists():
        raise RuntimeError(f"libhdf5 headers not found under {HDF5_PREFIX}")
    if _deps_newer(out, H5_SOURCES + [CSRC / "io" / "h5tree.h"]):
        inc = []
        for p in _pybind_includes():
            inc += ["-I", p]
        cmd = ["g++", "-O2", "-fPIC", "-shared", "-std=c++17", "-fvisibility=hidden", *map(str, H5_SOURCES), "-o",
               str(out), *inc, *hdf5_flags()]
        _run(cmd, verbose)
    return out


def build_h5_selftest(out: Path, sanitize: bool = True, verbose: bool = False) -> Path:
    """Standalone host executable of the HDF5 tree I/O self-test (ASan + UBSan)."""
    san = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"] if sanitize else []
    # link libhdf5 through a private directory holding only that library: putting the conda
    # lib dir on the search path would also pull in its older libstdc++
    libdir = Path(out).parent / "h5lib"
    libdir.mkdir(parents=True, exist_ok=True)
    so = sorted((HDF5_PREFIX / "lib").glob("libhdf5.so.[0-9]*"), key=lambda p: len(p.name))[0]
    link = libdir / so.name
    if not link.exists():
        link.symlink_to(so.resolve())
    cmd = ["g++", "-O1", "-g", "-std=c++17", *san, str(CSRC / "tests" / "h5_selftest.cpp"),
           str(CSRC / "io" / "h5tree.cpp"), "-o", str(out), "-I", str(CSRC / "io"), "-I", str(HDF5_PREFIX / "include"),
           str(link), f"-Wl,-rpath,{libdir}"]
    _run(cmd, verbose)
    return out


def build(verbose: bool = False, jobs: int | None = None):
    c = _build_C(verbose, jobs)
    h = _build_h5(verbose)
    return c, h


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
