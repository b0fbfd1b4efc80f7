"""Register, scratch and occupancy metadata of the built kernels (gfx950 code objects inside
the library's object files), for checking that a change keeps each variant's waves per SIMD.

    python scripts/kernel_regs.py [FILTER [BUILD_DIR]]

Prints per kernel: VGPRs (arch + acc), SGPRs, scratch bytes per lane, LDS (static) bytes."""
from __future__ import annotations

import glob
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(obj: str, tmp: str) -> list[str]:
    fat = os.path.join(tmp, os.path.basename(obj) + ".fatbin")
    out = os.path.join(tmp, os.path.basename(obj) + ".gfx950.co")
    if subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(tmp, "x.o")],
                      capture_output=True).returncode != 0:
        return []
    r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--input={fat}", f"--output={out}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--unbundle"], capture_output=True)
    return [out] if r.returncode == 0 and os.path.getsize(out) > 0 else []


def main() -> None:
    filt = sys.argv[1] if len(sys.argv) > 1 else ""
    bdir = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "rust-ray-tracing-in-a-weekend_amd", "build")
    objs = sorted(glob.glob(os.path.join(bdir, "*.o")))
    with tempfile.TemporaryDirectory() as tmp:
        for obj in objs:
            for co in code_objects(obj, tmp):
                notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
                for blk in notes.split("  - .agpr_count")[1:]:
                    name = re.search(r"\.name:\s+(\S+)", blk)
                    if not name or (filt and filt not in name.group(1)):
                        continue
                    def f(key):
                        m = re.search(rf"\.{key}:\s+(\d+)", blk)
                        return int(m.group(1)) if m else -1
                    print(f"{os.path.basename(obj):28s} vgpr {f('vgpr_count'):4d} sgpr {f('sgpr_count'):4d} "
                          f"scratch {f('private_segment_fixed_size'):4d} lds {f('group_segment_fixed_size'):6d} "
                          f"{name.group(1)[:90]}")


if __name__ == "__main__":
    main()
