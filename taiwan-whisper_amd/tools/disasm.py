"""Disassembly of one gfx950 kernel of a built object / library:  python disasm.py <file> <symbol substring>"""
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_regs import LLVM, device_objects  # noqa: E402


def main():
    path, pat = sys.argv[1], sys.argv[2]
    with tempfile.TemporaryDirectory() as d:
        for dev in device_objects(path, d):
            syms = subprocess.run([f"{LLVM}/llvm-readelf", "-sW", dev], capture_output=True, text=True).stdout.split("\n")
            for line in syms:
                parts = line.split()
                if len(parts) >= 8 and parts[3] == "FUNC" and pat in parts[7]:
                    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", f"--disassemble-symbols={parts[7]}",
                                          dev], capture_output=True, text=True).stdout
                    print(out)
                    return


if __name__ == "__main__":
    main()
