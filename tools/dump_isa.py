"""Disassemble one kernel of libdbsr_hip.so (the gfx950 code objects of its fat binary).
Usage: python tools/dump_isa.py <kernel-symbol-regex> [lib] > out.s"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_audit import LLVM, code_objects   # noqa: E402


def main():
    pat = re.compile(sys.argv[1])
    lib = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                            'deep-rawburst-sr_amd', 'libdbsr_hip.so')
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix='.co', delete=False) as f:
            f.write(co)
        txt = subprocess.run([os.path.join(LLVM, 'llvm-objdump'), '-d', '--no-show-raw-insn', f.name],
                             capture_output=True, text=True).stdout
        os.unlink(f.name)
        on = False
        for line in txt.splitlines():
            m = re.match(r'^[0-9a-f]+ <(.*)>:', line)
            if m:
                on = bool(pat.search(m.group(1)))
            if on:
                print(line)


if __name__ == '__main__':
    main()
