"""Host-only: resource metadata (VGPRs, spills, scratch, LDS) of the scene-specialised kernels
hiprtc builds for the preset scenes (no GPU needed). Usage: python tools/jit_meta.py [scene ...]"""
import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "surely-raytracing_amd"))
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
KEYS = ("vgpr_count", "vgpr_spill_count", "sgpr_count", "sgpr_spill_count", "agpr_count",
        "private_segment_fixed_size", "group_segment_fixed_size", "max_flat_workgroup_size")


def meta(code_path):
    notes = subprocess.run([READELF, "--notes", code_path], capture_output=True, text=True).stdout
    return {k: int(m.group(1)) for k in KEYS if (m := re.search(rf"\.{k}:\s+(\d+)", notes))}


def main(names):
    tmp = tempfile.mkdtemp()
    for name in names:
        dump = os.path.join(tmp, f"{name}.co")
        os.environ["RT_JIT_DUMP"] = dump
        import surely_rt as rt
        blob, cam = rt.preset_blob(name, width=32, spp=4)
        state, _ = rt.jit_check(blob)
        print(name, state, meta(dump) if state == 1 else "-")


if __name__ == "__main__":
    main(sys.argv[1:] or ["cornell_box", "cornell_smoke", "final_scene"])
