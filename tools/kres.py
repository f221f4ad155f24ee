"""Register use of every kernel in a hipcc object (.o with a .hip_fatbin section) or a code object:

    python tools/kres.py globalign_amd/_lib/ga_lane.o [name-filter]

prints name, VGPRs, AGPRs, SGPRs, VGPR / SGPR spills, LDS (static) per kernel (from the code object's
AMDGPU metadata note).
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def device_object(path, tmp):
    out = os.path.join(tmp, "dev.o")
    fat = os.path.join(tmp, "fat.bin")
    r = subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", path, os.path.join(tmp, "x.o")],
                       capture_output=True)
    if r.returncode != 0:
        return path  # already a code object
    subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={out}"])
    return out


def main():
    path = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    with tempfile.TemporaryDirectory() as tmp:
        notes = subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", device_object(path, tmp)], text=True)
    kernels, cur = [], None
    for ln in notes.splitlines():
        s = ln.strip()
        if s.startswith("- .agpr_count:") or (s.startswith("- ") and cur is None and ":" in s):
            cur = {}
            kernels.append(cur)
            s = s[2:]
        elif s.startswith("- "):
            cur = {}
            kernels.append(cur)
            s = s[2:]
        m = re.match(r"\.(\w+):\s+(.*)", s)
        if m and cur is not None:
            cur.setdefault(m.group(1), m.group(2))
    for k in kernels:
        name = k.get("name", "")
        if not name or flt not in name:
            continue
        print(f"{k.get('vgpr_count', '?'):>4} v {k.get('agpr_count', '?'):>3} a {k.get('sgpr_count', '?'):>4} s "
              f"spill v{k.get('vgpr_spill_count', '?')} s{k.get('sgpr_spill_count', '?')} "
              f"lds {k.get('group_segment_fixed_size', '?'):>6}  {name}")


if __name__ == "__main__":
    main()
