"""Fill the code-object cache (build/jit_cache, rt_jit.cpp cache_path) with the scene-specialised
kernels of the benchmark scenes, host-only (hiprtc cross-compiles for gfx950 without a GPU).

PyTorch is imported first, as bench.py does, so the kernels are built by the hiprtc a benchmark
process binds to (PyTorch's bundled compiler); with the cache every process -- the benchmark, the
tests, a rocprofv3 profile -- then loads these same binaries instead of compiling with whichever
libhiprtc it happened to load. Usage: python tools/jit_cache_fill.py [scene ...]"""
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "surely-raytracing_amd"))

# the scenes of BASELINE configs c2 (and c5: same scene), c3, c4 and the smoke test
SCENES = [("cornell_box", {}), ("cornell_smoke", {}), ("final_scene", {})]


def main(names):
    import torch  # noqa: F401  (the benchmark's compiler; see the module docstring)
    import surely_rt as rt

    os.environ["RT_JIT_CACHE_WRITE"] = "1"
    cache = REPO / "build" / "jit_cache"
    cache.mkdir(parents=True, exist_ok=True)
    todo = [(n, kw) for n, kw in SCENES if not names or n in names]
    for name, kw in todo:
        t0 = time.time()
        blob, _ = rt.preset_blob(name, width=32, spp=4, **kw)
        state, _ = rt.jit_check(blob)
        print(f"jit cache: {name}: state {state}, {time.time() - t0:.1f} s", flush=True)
    print(f"jit cache: {len(list(cache.glob('*.co')))} code objects in {cache}")


if __name__ == "__main__":
    main(sys.argv[1:])
