"""Diagnostics: the scene-specialised kernel of final_scene as the GPU box compiles it for the
device (rt_scene_jit_info reports the runtime's view of its resources) and as the host-only
check compiles it; both code objects land in gpurun_out/ for llvm-readelf --notes."""
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "surely-raytracing_amd"))
out = REPO / "gpurun_out"
out.mkdir(exist_ok=True)
os.environ["RT_JIT_DUMP"] = str(out / "fs_device.co")
import surely_rt as rt  # noqa: E402

blob, cam = rt.preset_blob("final_scene", width=32, spp=1, depth=4)
ds = rt.DeviceScene(blob)
ds.render(cam, rt.make_opts(cam))
print("device render:", ds.jit_info(), flush=True)
ds.close()
os.environ["RT_JIT_DUMP"] = str(out / "fs_check.co")
print("jit_check:", rt.jit_check(blob)[0])
