#!/usr/bin/env python3
"""Build check (CPU): no in-flight vector-memory load's destination VGPRs are touched before a vmcnt wait.

VERDICT r05 item 3 / ADVICE r05 (attention.hip `gload16_asm`): the head-resident attention kernels load their first
Q fragments with inline-asm `global_load_dwordx4` ahead of the K/V LDS-DMA and wait for them later with an explicit
`s_waitcnt vmcnt(n)`.  hipcc treats an asm output as defined when the asm statement ends, so if register allocation
ever copied, split or reused those VGPRs between the load and its wait, the late data would land in registers that
hold something else (round 5's memory fault was put down to exactly that, for a since-removed prefetch).  This script
checks the SHIPPED code object, not the source:

  1. pull the gfx950 code objects out of libpdm.so's `.hip_fatbin` (one offload bundle per translation unit);
  2. disassemble them with llvm-objdump;
  3. for every VMEM load with a VGPR destination (global_/buffer_/flat_/scratch_load_*, not the LDS-DMA forms) walk
     every control-flow path from the instruction after the load (both sides of each conditional branch, loops
     visited once) until the path reaches an `s_waitcnt` with a vmcnt field, and fail if any instruction on the way
     reads or writes one of the load's destination registers.

Compiler-emitted loads pass by construction (hipcc waits before it touches a load's result); the check is what
guards the asm ones, whose waits the compiler does not know about.  Usage:

  python tools/check_asm_loads.py [path/to/libpdm.so] [--kernels REGEX] [-v]
exit status 0 = clean, 1 = violations (listed), 2 = tools or library missing.
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

FUNC_RE = re.compile(r"^([0-9a-f]+) <(.+)>:$")
INST_RE = re.compile(r"^\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-F]+):")
TGT_RE = re.compile(r"<(.+)\+0x([0-9a-f]+)>\s*$")
VREG_RE = re.compile(r"(?<![a-z_])v(?:\[(\d+):(\d+)\]|(\d+))(?![0-9a-z_])")
LOAD_RE = re.compile(r"^(global|buffer|flat|scratch)_load_")


def code_objects(lib, tmp):
    """The gfx950 code object of every offload bundle in lib's .hip_fatbin section."""
    fat = os.path.join(tmp, "fatbin.bin")
    subprocess.check_call([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat])
    data = open(fat, "rb").read()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
    out = []
    for i in range(len(offs) - 1):
        part = os.path.join(tmp, f"b{i}.bundle")
        with open(part, "wb") as f:
            f.write(data[offs[i]:offs[i + 1]])
        co = os.path.join(tmp, f"b{i}.co")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--targets={TARGET}",
                            f"--input={part}", f"--output={co}"], capture_output=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            out.append(co)
    return out


def parse(asm_text):
    """{kernel: [(mnemonic, operands, branch target index or None)]}, branch targets resolved to indices."""
    funcs, cur, addr0 = {}, None, 0
    raw = {}
    for ln in asm_text.splitlines():
        m = FUNC_RE.match(ln)
        if m:
            cur = m.group(2)
            addr0 = int(m.group(1), 16)
            raw[cur] = []
            continue
        if cur is None:
            continue
        m = INST_RE.match(ln)
        if not m:
            continue
        mnem, ops, addr = m.group(1), m.group(2), int(m.group(3), 16)
        t = TGT_RE.search(ln)
        tgt = addr0 + int(t.group(2), 16) if (t and mnem.startswith(("s_branch", "s_cbranch")) and t.group(1) == cur) else None
        raw[cur].append((addr, mnem, ops, tgt))
    for name, ins in raw.items():
        index = {a: i for i, (a, _, _, _) in enumerate(ins)}
        funcs[name] = [(mn, ops, index.get(tg) if tg is not None else None) for (_, mn, ops, tg) in ins]
    return funcs


def vregs(ops):
    s = set()
    for m in VREG_RE.finditer(ops):
        if m.group(3) is not None:
            s.add(int(m.group(3)))
        else:
            s.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return s


def load_dest(mnem, ops):
    """Destination VGPRs of a VMEM load (None for LDS-DMA forms, which write LDS, and for non-loads)."""
    if not LOAD_RE.match(mnem) or " lds" in f" {ops}" or mnem.startswith("global_load_lds"):
        return None
    first = ops.split(",")[0]
    d = vregs(first)
    return d or None


def check_function(name, ins):
    """Violations [(load index, load text, offending index, offending text)] and stats of the waits reached."""
    bad, waits = [], []
    for i, (mn, ops, _) in enumerate(ins):
        dest = load_dest(mn, ops)
        if not dest:
            continue
        seen, stack = set(), [i + 1]
        while stack:
            j = stack.pop()
            if j in seen or j >= len(ins):
                continue
            seen.add(j)
            mj, oj, tj = ins[j]
            if mj == "s_waitcnt" and "vmcnt(" in oj:
                waits.append(oj)
                continue
            if mj.startswith("s_endpgm"):
                continue
            touched = vregs(oj) & dest
            dj = load_dest(mj, oj)
            if touched and dj and not (vregs(oj) - dj) & dest:
                # another vector-memory load re-targeting the registers (a loop's next iteration): loads return in
                # issue order, so the later data lands last -- the compiler relies on the same ordering
                touched = set()
            if touched:
                bad.append((i, f"{mn} {ops}", j, f"{mj} {oj}"))
                continue
            if mj.startswith("s_setpc") or mj.startswith("s_swappc"):
                bad.append((i, f"{mn} {ops}", j, f"{mj} {oj} (indirect control flow: cannot follow)"))
                continue
            if mj == "s_branch":
                if tj is not None:
                    stack.append(tj)
                continue
            if mj.startswith("s_cbranch"):
                if tj is not None:
                    stack.append(tj)
            stack.append(j + 1)
    return bad, waits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(REPO, "panopticdiffusionmodels_amd", "libpdm.so"))
    ap.add_argument("--kernels", default=".", help="regex over mangled kernel names (default: every kernel)")
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args()
    if not os.path.exists(a.lib) or not os.path.exists(f"{LLVM}/llvm-objdump"):
        print(f"missing {a.lib} or {LLVM}/llvm-objdump", file=sys.stderr)
        return 2
    sel = re.compile(a.kernels)
    nload = nfunc = 0
    asm_loads = 0
    violations = []
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(a.lib, tmp):
            text = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], capture_output=True, text=True,
                                  check=True).stdout
            for name, ins in parse(text).items():
                if not sel.search(name):
                    continue
                nfunc += 1
                nl = sum(1 for mn, ops, _ in ins if load_dest(mn, ops))
                nload += nl
                bad, waits = check_function(name, ins)
                violations += [(name,) + b for b in bad]
                if "attention" in name:
                    asm_loads += sum(1 for mn, ops, _ in ins if mn == "global_load_dwordx4" and ops.endswith("off"))
                if a.v and nl:
                    print(f"{name}: {nl} VGPR loads, {len(waits)} vmcnt waits reached, {len(bad)} violations")
    print(f"checked {nload} VGPR-destination VMEM loads in {nfunc} kernels "
          f"({asm_loads} plain 'global_load_dwordx4 ..., off' in attention kernels); violations: {len(violations)}")
    for name, i, lt, j, jt in violations[:50]:
        print(f"  {name}: load #{i} `{lt}` -> instruction #{j} `{jt}` touches its destination before a vmcnt wait")
    return 1 if violations else 0


if __name__ == "__main__":
    sys.exit(main())
