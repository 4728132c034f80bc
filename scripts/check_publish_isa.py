#!/usr/bin/env python
"""Static check of the cross-device publish order in the gfx950 code of every kernel.

Why: the sharded MNIST exchange (csrc/kernels/convnet_step2.hip) and the peer all-reduce
(csrc/kernels/peer_allreduce.hip) announce data stored into another GPU's uncached staging
by a system-scope flag store.  A peer that sees the flag reads the data at once, so every
store the flag announces must have been ACKNOWLEDGED first.  On gfx950 that takes an
explicit ``s_waitcnt vmcnt(0)`` in every wave that issued payload: a workgroup barrier
does not wait for outstanding vector-memory stores (the round-4 bug: the small message of
the sharded exchange was published after a bare ``__syncthreads()``).

What is checked, per kernel function, on the device assembly:

* every system-scope store (``global_store*``/``global_atomic*`` with ``sc0 sc1``) -- a
  flag -- is preceded by a publish marker (``DAMD_PUBLISH_WG()`` / ``DAMD_PUBLISH_WAVE()``,
  csrc/include/damd_common.h: assembly comments, no code), so no publish site is
  unclassified;
* own-wave drain (both kinds): after the last ordinary vector store / atomic ahead of the
  flag there is an ``s_waitcnt`` with ``vmcnt(0)``;
* workgroup publish (payload issued by every wave, flag raised by a few lanes): at the last
  ``s_barrier`` ahead of the flag no store was outstanding, i.e. the drain precedes the
  barrier -- in every wave, since all waves run the same instruction stream.

The markers exist only in the assembly (``hipcc --cuda-device-only -S`` with the build's
exact flags, distributed_amd/_build.py:hip_kernel_cmd).  To make sure that what is checked
is what ships, the instruction stream of each function in that assembly is compared with
the disassembly of the gfx950 code object inside ``build/obj/<src>.o`` (extracted from
its ``.hip_fatbin`` section with clang-offload-bundler): the mnemonic sequences must be
identical.  The scan is linear in code-layout order; a layout that interleaves blocks so
that the check cannot see the order fails closed (reported), it never passes silently.

Exit status 0 = every publish is ordered; 1 = a violation or a mismatch (printed).
"""
from __future__ import annotations

import argparse
import re
import subprocess
import sys
import tempfile
from dataclasses import dataclass, field
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

LLVM = Path("/opt/rocm/lib/llvm/bin")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

STORE_RE = re.compile(r"^(global|buffer|flat|scratch)_(store|atomic)")
PADDING = {"...", "v_cndmask_b32_e32 v0, s0, v0, vcc"}
MARK_RE = re.compile(r";\s*damd\.publish\s+(wg|wave)")


@dataclass
class Fn:
    name: str
    items: list = field(default_factory=list)  # (kind, mnemonic, text)

    def mnemonics(self):
        # s_nop excluded: the assembler pads the kernarg-preload prologue with s_nop fill
        # that the -S output does not show (hazard s_nops appear on both sides anyway)
        return [m for k, m, _ in self.items if k == "insn" and m != "s_nop"]


def parse_asm(text: str) -> dict:
    """Device assembly (-S): functions -> instructions and markers in layout order."""
    fns, cur = {}, None
    in_text = False
    for raw in text.splitlines():
        line = raw.rstrip()
        s = line.strip()
        if s.startswith(".section") or s.startswith(".text"):
            in_text = s.startswith(".text") or ".text" in s
            continue
        m = re.match(r"^([A-Za-z_.$][\w.$]*):", line)
        if m and not line.startswith("."):
            lab = m.group(1)
            if not lab.startswith(".L") and in_text and not lab.startswith("__hip_cuid"):
                cur = fns.setdefault(lab, Fn(lab))
            continue
        if cur is None:
            continue
        if s.startswith(".Lfunc_end") or s.startswith(".size"):
            cur = None if s.startswith(".size") else cur
            continue
        mk = MARK_RE.search(s)
        if mk:
            cur.items.append(("mark", mk.group(1), s))
            continue
        if not s or s.startswith(";") or s.startswith(".") or s.startswith("//"):
            continue
        code = s.split(";")[0].split("//")[0].strip()
        if not code or code.endswith(":"):
            continue
        mn = code.split()[0]
        cur.items.append(("insn", mn, code))
    return fns


def parse_objdump(text: str) -> dict:
    fns, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <([^>]+)>:$", line)
        if m:
            cur = fns.setdefault(m.group(1), Fn(m.group(1)))
            continue
        if cur is None:
            continue
        s = line.strip()
        if not s or s.startswith("Disassembly"):
            continue
        code = s.split("//")[0].strip()
        if not code:
            continue
        cur.items.append(("insn", code.split()[0], code))
    return fns


def check_fn(fn: Fn) -> list:
    """Violations of the publish order in one function (empty = ok)."""
    errs = []
    last_store = -1      # index of the last ordinary (payload) vector store / atomic
    last_drain = -1      # index of the last s_waitcnt with vmcnt(0)
    barrier_dirty = None  # at the last s_barrier: was a store outstanding?  (None = no barrier yet)
    marker = None
    for i, (kind, mn, text) in enumerate(fn.items):
        if kind == "mark":
            marker = mn
            continue
        if mn == "s_waitcnt" and ("vmcnt(0)" in text or re.fullmatch(r"s_waitcnt\s+0", text)):
            last_drain = i
        elif mn == "s_barrier":
            barrier_dirty = last_store > last_drain
        elif STORE_RE.match(mn):
            if " sc0" in f" {text}" and " sc1" in f" {text}":
                where = f"{fn.name}: #{i} `{text}`"
                if marker is None:
                    errs.append(f"unclassified system-scope store (no DAMD_PUBLISH_* marker): {where}")
                    continue
                if last_store > last_drain:
                    errs.append(f"flag store with this wave's payload stores not drained (no s_waitcnt vmcnt(0) "
                                f"after the last store): {where}")
                if marker == "wg":
                    if barrier_dirty is None:
                        errs.append(f"workgroup publish without a preceding s_barrier: {where}")
                    elif barrier_dirty:
                        errs.append(f"workgroup publish: stores still outstanding at the s_barrier ahead of the "
                                    f"flag (other waves' payload may be in flight): {where}")
            else:
                last_store = i
                marker = None  # a marker classifies the flag stores right after it only
    return errs


def flag_count(fn: Fn) -> int:
    return sum(1 for k, mn, t in fn.items if k == "insn" and STORE_RE.match(mn) and " sc0" in f" {t}"
               and " sc1" in f" {t}")


def objdump_of(obj: Path, tmp: Path) -> str:
    fb = tmp / (obj.name + ".fatbin")
    co = tmp / (obj.name + ".gfx950.co")
    subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", str(obj), str(tmp / "x.o")],
                   check=True, capture_output=True)
    subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fb}",
                    f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
    r = subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", str(co)], check=True,
                       capture_output=True, text=True)
    return r.stdout


def check_source(src: Path, tmp: Path, require_obj: bool) -> tuple:
    from distributed_amd import _build

    asm_path = tmp / (src.name + ".s")
    r = subprocess.run(_build.hip_kernel_cmd(src, asm_path, device_asm=True), capture_output=True, text=True)
    if r.returncode != 0:
        return [f"{src.name}: device assembly build failed:\n{r.stderr[-2000:]}"], 0, False
    fns = parse_asm(asm_path.read_text())
    errs, nflags = [], 0
    for fn in fns.values():
        nflags += flag_count(fn)
        errs += [f"{src.name}: {e}" for e in check_fn(fn)]
    obj = _build.BUILD / "obj" / (src.name + ".o")
    compared = False
    if obj.exists() and obj.stat().st_mtime >= src.stat().st_mtime:
        dis = parse_objdump(objdump_of(obj, tmp))
        for name, fn in fns.items():
            if name not in dis:
                errs.append(f"{src.name}: function {name} missing from the shipped object")
                continue
            a, b = fn.mnemonics(), dis[name].mnemonics()
            # the disassembly runs on over the alignment padding after a function (zero
            # words: "..." or their decoding `v_cndmask_b32_e32 v0, s0, v0, vcc`, s_nop fill)
            tail = [t for k, m, t in dis[name].items if k == "insn" and m != "s_nop"][len(a):]
            if b[:len(a)] == a and all(t in PADDING or t.startswith("s_nop") or t.startswith("s_code_end")
                                       for t in tail):
                b = a
            if a != b:
                k = next((i for i, (x, y) in enumerate(zip(a, b)) if x != y), min(len(a), len(b)))
                errs.append(f"{src.name}: {name}: checked assembly differs from the shipped object at instruction "
                            f"{k} ({a[k:k + 3]} vs {b[k:k + 3]}; {len(a)} vs {len(b)} instructions)")
        compared = True
    elif require_obj:
        errs.append(f"{src.name}: no up-to-date object {obj} to compare with (run the build first)")
    return errs, nflags, compared


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("sources", nargs="*", help="kernel sources (default: every csrc/kernels/*.hip)")
    ap.add_argument("--require-object", action="store_true",
                    help="fail when build/obj holds no up-to-date object to compare with")
    a = ap.parse_args(argv)
    srcs = [Path(s) for s in a.sources] or sorted((ROOT / "csrc" / "kernels").glob("*.hip"))
    bad = 0
    with tempfile.TemporaryDirectory() as td:
        for s in srcs:
            errs, nflags, compared = check_source(s.resolve(), Path(td), a.require_object)
            print(f"{s.name}: {nflags} system-scope flag stores, "
                  f"{'asm == shipped object' if compared else 'object not compared'}: "
                  f"{'OK' if not errs else 'FAIL'}")
            for e in errs:
                print("  " + e)
            bad += bool(errs)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
