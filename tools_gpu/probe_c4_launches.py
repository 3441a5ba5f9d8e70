import torch, sys, os
sys.path.insert(0, "surely-raytracing_amd")
import surely_rt as rt
print("torch mem_get_info", torch.cuda.mem_get_info(), flush=True)
blob, cam = rt.preset_blob("final_scene", width=800, spp=5000)
ds = rt.DeviceScene(blob)
import numpy as np
acc, st = ds.render(cam, rt.make_opts(cam, seed=1, sj_begin=0, sj_count=70))
print("launches", st.launches, "out_bytes", st.out_bytes, "ms", st.ms_kernel, flush=True)
