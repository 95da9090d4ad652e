"""List register spills / scratch of every kernel in the built library's gfx950 code objects.

    python tools/spills.py [--all]      (reads picotron_amd/lib/obj/*.o; exit 1 if any kernel spills)

Each object's .hip_fatbin bundle is unbundled to its gfx950 code object and the AMDGPU metadata
notes are read (llvm-readelf --notes): .vgpr_spill_count, .sgpr_spill_count and
.private_segment_fixed_size (scratch bytes per lane) per kernel."""
import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernels(obj):
    with tempfile.TemporaryDirectory() as td:
        fb, co = os.path.join(td, "f.bin"), os.path.join(td, "k.co")
        r = subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(td, "o")],
                           capture_output=True)
        if r.returncode:   # no device code in this object (host-only source)
            return []
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={fb}", f"--output={co}", "--unbundle"], check=True, capture_output=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    out = []
    for blk in notes.split("\n      - ")[1:]:
        def g(k):
            m = re.search(r"\." + k + r":\s+(\S+)", blk)
            return m.group(1) if m else "0"
        if ".symbol:" not in blk:
            continue
        out.append({"name": g("name"), "vgpr": int(g("vgpr_count")), "agpr": int(g("agpr_count")),
                    "vspill": int(g("vgpr_spill_count")), "sspill": int(g("sgpr_spill_count")),
                    "scratch": int(g("private_segment_fixed_size")), "lds": int(g("group_segment_fixed_size"))})
    return out


def main():
    show_all = "--all" in sys.argv
    bad = 0
    for obj in sorted(glob.glob(os.path.join(ROOT, "picotron_amd", "lib", "obj", "*.o"))):
        for k in kernels(obj):
            spill = k["vspill"] or k["scratch"]   # SGPR spills go to VGPR lanes (v_writelane), not memory
            bad += bool(spill)
            if spill or show_all or k["sspill"]:
                print(f"{os.path.basename(obj):18s} vgpr={k['vgpr']:3d} agpr={k['agpr']:3d} vspill={k['vspill']:3d} "
                      f"sspill={k['sspill']:3d} scratch={k['scratch']:4d} lds={k['lds']:6d} {k['name'][:120]}")
    print(f"{bad} kernel(s) with VGPR spills or scratch memory")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
