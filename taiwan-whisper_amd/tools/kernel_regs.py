"""Register / scratch report of the gfx950 kernels in a built object or library (.o / .so): unbundles the HIP fat
binary and reads the code-object metadata.  usage: python kernel_regs.py <file> [name-substring]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def device_objects(path, out_dir):
    """The gfx950 code objects of every offload bundle in the file's .hip_fatbin (a library holds one per source)."""
    fat = os.path.join(out_dir, "fat.bin")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fat], check=True)
    data = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    devs = []
    for i, a in enumerate(starts):
        b = starts[i + 1] if i + 1 < len(starts) else len(data)
        part = os.path.join(out_dir, f"b{i}.bin")
        open(part, "wb").write(data[a:b])
        dev = os.path.join(out_dir, f"dev{i}.o")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"], capture_output=True)
        if r.returncode == 0 and os.path.getsize(dev) > 0:
            devs.append(dev)
    return devs


def main():
    path, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    with tempfile.TemporaryDirectory() as d:
        notes = "".join(subprocess.run([f"{LLVM}/llvm-readelf", "--notes", dev], capture_output=True, text=True).stdout
                        for dev in device_objects(path, d))
    for m in re.finditer(r"\.name:\s+(\S+)(.*?)(?=\n\s+- \.|\Z)", notes, re.S):
        name, body = m.group(1), m.group(2)
        if pat not in name:
            continue
        get = lambda k: (re.search(rf"\.{k}:\s+(\d+)", body) or [None, "-"])[1]
        print(f"{name[:90]:90s} scratch {get('private_segment_fixed_size'):>4s} vgpr {get('vgpr_count'):>3s} "
              f"sgpr {get('sgpr_count'):>3s} lds {get('group_segment_fixed_size')}")


if __name__ == "__main__":
    main()
