#!/usr/bin/env python3
"""Dump the disassembly of the kernels whose mangled name matches REGEX from libpdm.so's code objects
(dev tool: python tools/dump_kernel_isa.py REGEX [lib] > out.s)."""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import check_asm_loads as c  # noqa: E402

pat = re.compile(sys.argv[1])
lib = sys.argv[2] if len(sys.argv) > 2 else os.path.join(c.REPO, "panopticdiffusionmodels_amd", "libpdm.so")
with tempfile.TemporaryDirectory() as tmp:
    for co in c.code_objects(lib, tmp):
        text = subprocess.run([f"{c.LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                              text=True, check=True).stdout
        on = False
        for ln in text.splitlines():
            m = c.FUNC_RE.match(ln)
            if m:
                on = bool(pat.search(m.group(2)))
            if on:
                print(ln)
