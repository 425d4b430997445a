"""Per-kernel VGPR / AGPR / LDS / scratch of a built gfx950 library (the code
object metadata tests/test_codeobject.py checks), filtered by a regex.

usage: python tools/kernel_resources.py [regex] [--lib path/to/lib.so]
"""
import argparse
import os
import re
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def kernel_notes(lib):
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fatbin.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", lib,
                        os.path.join(d, "lib.stripped")], check=True)
        blob = open(fat, "rb").read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        starts = [m.start() for m in re.finditer(re.escape(magic), blob)]
        notes = ""
        for i, st in enumerate(starts):
            part, co = os.path.join(d, f"b{i}.bin"), os.path.join(d, f"b{i}.o")
            with open(part, "wb") as f:
                f.write(blob[st:starts[i + 1] if i + 1 < len(starts) else len(blob)])
            subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
            notes += subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                                    capture_output=True, text=True).stdout
    out = {}
    for ent in re.split(r"\n\s+- \.agpr_count:", notes)[1:]:
        field = lambda k: re.search(rf"\.{k}:\s+(\S+)", ent)  # noqa: E731
        if field("name") is None or field("vgpr_count") is None:
            continue
        out[field("name").group(1)] = (int(field("vgpr_count").group(1)), int(ent.split("\n", 1)[0].strip()),
                                       int(field("group_segment_fixed_size").group(1)),
                                       int(field("private_segment_fixed_size").group(1)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pattern", nargs="?", default=".")
    ap.add_argument("--lib", default=os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd", "kvecc", "libkvecc.so"))
    args = ap.parse_args()
    for name, (v, a, lds, scr) in sorted(kernel_notes(args.lib).items()):
        if re.search(args.pattern, name):
            print(f"vgpr {v:3d} agpr {a:3d} lds {lds:6d} scratch {scr:4d}  {name}")


if __name__ == "__main__":
    main()
