#!/usr/bin/env python3
"""bench.py — Msamples/s of the per-pixel render loop on MI355X (BASELINE.json metric).

Workload (BASELINE configs[1]): the reference's cornell_box scene
(main.rs:417-512) with mixture-PDF light sampling, 800x800, 1000 spp -> 961 effective
(nearest_square, render.rs:38-41), max depth 50, render seed 1.

A "step" = one full frame: every rank renders its cyclic share of the 800 rows
(row r -> rank r % N, no data-path collective) into a device buffer, then the frame is
gathered to rank 0 by the product's C-ABI gather (rt_gather_frame: ncclGather over RCCL/xGMI;
the field "gather" names it; the one-GPU gloo rehearsal uses torch.distributed.gather). Scene upload, RCCL init and the
op-count pass are outside the timed region. value = W*H*spp_eff*steps / max-over-ranks time.

Also reported (one JSON line on rank 0):
  roofline     FP64 VALU roofline of rt_trace: counted algorithmic flops per launch / the
               kernel's average duration (HIP events recorded by the library around each
               rt_trace launch on the bench stream, rt_scene_trace_ms), vs 78.6 TF; render_ms =
               the whole render call (rt_trace + rt_reduce, torch.cuda.Event on that stream).
  hbm          the north star's "achieved HBM GB/s" of the path kernel (BVH traversal at C4):
               rocprofv3 PMC FETCH_SIZE + WRITE_SIZE bytes per rt_trace launch, from the committed
               profile of this exact workload (profiles/pmc_traffic_<config>.json; PMC counters
               cannot be read inside this process), over this run's kernel time, vs 8 TB/s.
  cpu_baseline the f64 CPU oracle (a restatement of the reference; the Rust original cannot be
               built here) on this host's cores, timed on a bounded stratum subset of the same
               frame (rank 0, N = 1 only).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--width 800] [--spp 1000]
       torchrun --nproc-per-node N bench.py --gpus N ...
At --gpus N > 1 without torchrun (WORLD_SIZE unset) the script starts its N ranks itself
(self_launch: one child process per GPU, torchrun's environment, rank 0's line relayed).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "surely-raytracing_amd"))

METRIC = "Msamples/sec (pixels*spp/s), Cornell box 800x800 @ 1/2/4/8 MI355X"
# BASELINE.json configs that fit one GPU. c2 is the headline the metric is quoted on;
# c3/c4 use the same harness (their lines are reported under the same unit, tagged by workload).
CONFIGS = {
    "c2": dict(name="BASELINE configs[1]", scene="cornell_box", width=800, spp=1000, depth=50),
    "c3": dict(name="BASELINE configs[2]", scene="cornell_smoke", width=800, spp=1000, depth=10),
    "c4": dict(name="BASELINE configs[3]", scene="final_scene", width=800, spp=5000, depth=40),
    # configs[4] is quoted on 8 GPUs (the book3 Cornell scene at 16:9); on N GPUs
    # every rank renders its cyclic share of the 2160 rows, as for the other configs
    "c5": dict(name="BASELINE configs[4]", scene="cornell_box", width=3840, spp=10000, depth=50,
               aspect=16.0 / 9.0),
}


# The one-GPU share probe of the C2 frame (tools_gpu/scaling_probe.py, round 3): full-frame
# kernel time / (N x slowest share's kernel time). A projection, reported beside a measured N > 1
# line, never in place of one.
SCALING_PROJECTION = {("BASELINE configs[1]", 2): 0.983, ("BASELINE configs[1]", 4): 0.974,
                      ("BASELINE configs[1]", 8): 0.939}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS),
                    help="BASELINE config (c2 = the headline; c3/c4 = the other 1-GPU configs)")
    ap.add_argument("--scene", default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target CPU-baseline work (bounded sample)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-count", action="store_true", help="skip the op-count pass")
    ap.add_argument("--launch-check", action="store_true",
                    help="check the N-rank launch over gloo without a GPU (no render)")
    a = ap.parse_args()
    c = CONFIGS[a.config]
    for k in ("scene", "width", "spp", "depth"):
        if getattr(a, k) is None:
            setattr(a, k, c[k])
    a.aspect = c.get("aspect", 0.0) if a.scene == c["scene"] else 0.0
    a.config_name = c["name"] if (a.scene, a.width, a.spp, a.depth) == (
        c["scene"], c["width"], c["spp"], c["depth"]) else "custom"
    return a


def host_parallelism():
    """The reference's thread count: rayon's global pool uses std::thread::available_parallelism()
    (render.rs:153-160), i.e. the CPUs this process may run on (sched_getaffinity), lowered to a
    cgroup v2 CPU quota when one is set (cpu.max). Returns (threads, how it was determined)."""
    try:
        n = len(os.sched_getaffinity(0))
        how = f"sched_getaffinity: {n}"
    except AttributeError:
        n = os.cpu_count() or 1
        how = f"os.cpu_count: {n}"
    try:
        quota, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if quota != "max":
            q = max(1, -(-int(quota) // int(period)))
            how += f", cgroup cpu.max quota {quota}/{period} -> {q}"
            n = min(n, q)
    except (OSError, ValueError):
        pass
    if n > 512:  # the GPU box's process guard counts tasks (1024 at once); never expected here
        how += f", capped at 512 of {n}"
        n = 512
    return max(1, n), how


def cpu_baseline(blob, cam, seed, target_s):
    """f64 CPU oracle on a bounded sample of the same frame: full image, a subset of the
    sqrt_spp stratum rows (each sample keeps the full-spp jitter), 3-row chunks over a thread
    pool (render.rs:171)."""
    sys.path.insert(0, str(REPO / "tests"))
    import oracle_lib as O
    import surely_rt as rt

    threads, how = host_parallelism()
    done_samples, elapsed, sj = 0, 0.0, 0
    S = cam.sqrt_spp
    while sj < S and elapsed < target_s:
        opts = rt.make_opts(cam, seed=seed, sj_begin=(S // 2 + sj) % S, sj_count=1)
        t0 = time.perf_counter()
        O.render(blob, cam, opts, precision=64, threads=threads)
        elapsed += time.perf_counter() - t0
        done_samples += cam.image_width * cam.image_height * S
        sj += 1
    return {
        "value": done_samples / elapsed / 1e6,
        "unit": "Msamples/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{sj} of {S} stratum rows (s_j) over the full {cam.image_width}x"
                   f"{cam.image_height} frame = {done_samples} samples in {elapsed:.1f} s; "
                   "f64 C restatement of the reference (oracle/rt_oracle.c), 3-row chunks, one "
                   f"thread per available core as rayon's pool ({how})"),
    }


def self_launch(n: int, argv) -> int:
    """`python3 bench.py --gpus N` without torchrun (WORLD_SIZE unset, N > 1): start N child
    processes of this same script, one per GPU, with RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT set as torchrun would, relay rank 0's stdout (its JSON line) and
    return non-zero if any rank fails. The parent never imports torch nor touches the GPU, and
    it starts children (no exec), so this is safe on the GPU box. A rank that fails ends the
    others (they would wait in a barrier forever): exact child PIDs, SIGTERM then SIGKILL; a
    SIGTERM / SIGINT / SIGHUP to the launcher is forwarded to the ranks the same way."""
    import socket
    import subprocess
    import threading

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", str(Path(__file__).resolve())]
                                      + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else None))

    def relay(stream):
        for line in iter(stream.readline, b""):
            sys.stdout.write(line.decode(errors="replace"))
            sys.stdout.flush()

    import signal

    def forward(signum, _frame):  # a launcher stopped by its caller stops its ranks first
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)
        deadline = time.time() + 20
        while time.time() < deadline and any(p.poll() is None for p in procs):
            time.sleep(0.2)
        for p in procs:
            if p.poll() is None:
                p.kill()
        raise SystemExit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(sig, forward)
    t = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    t.start()
    failed = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad and failed is None:
            failed = bad[0]
            print(f"bench.py self-launch: rank {bad[0][0]} exited with {bad[0][1]}; "
                  "ending the other ranks", file=sys.stderr, flush=True)
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            deadline = time.time() + 20
            while time.time() < deadline and any(p.poll() is None for p in procs):
                time.sleep(0.2)
            for p in procs:
                if p.poll() is None:
                    p.kill()
        if all(c is not None for c in (p.poll() for p in procs)):
            break
        time.sleep(0.2)
    t.join(timeout=10)
    if failed is not None:
        return failed[1] if failed[1] > 0 else 1
    return 0


def launch_check(args):
    """--launch-check: the self-launch's rank plumbing without a GPU (gloo): every rank joins the
    process group from the environment the launcher set, takes the max over ranks as the bench
    does, and rank 0 prints one JSON line. Used by the CPU test of the launcher."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if os.environ.get("RT_LAUNCH_CHECK_FAIL_RANK") == str(rank):
        raise SystemExit(3)  # the launcher's failure path: the other ranks wait in rendezvous
    if os.environ.get("RT_LAUNCH_CHECK_HOLD") == "1":
        time.sleep(120)  # the launcher's signal path: ranks still running when it is stopped
    dist.init_process_group("gloo")
    dist.barrier()
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    objs = [None] * world if rank == 0 else None
    dist.gather_object({"rank": rank, "local_rank": int(os.environ["LOCAL_RANK"])}, objs, dst=0)
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "max_over_ranks": t.item(),
                          "ranks": objs}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the driver's plain `python3 bench.py --gpus N`: become the launcher of N ranks
        raise SystemExit(self_launch(args.gpus, sys.argv[1:]))
    if args.launch_check:
        return launch_check(args)
    import torch
    import torch.distributed as dist

    import surely_rt as rt
    from surely_rt import roofline
    from surely_rt.parallel import (GATHER_RCCL, RcclFrameGather, cyclic_rows, gather_choice,
                                    gather_frame, max_rows, rank_report)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # RT_BENCH_REHEARSAL=1: the N > 1 code path on a one-GPU box (gloo, every rank on the same
    # card, the gather through host memory); the driver's multi-GPU runs use RCCL, one GPU a rank
    rehearse = os.environ.get("RT_BENCH_REHEARSAL") == "1"
    local = local % torch.cuda.device_count() if rehearse else local
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    blob, cam = rt.preset_blob(args.scene, width=args.width, spp=args.spp, depth=args.depth,
                               aspect=args.aspect)
    W, H, spp = cam.image_width, cam.image_height, cam.samples_per_pixel
    ds = rt.DeviceScene(blob, device=local)
    b, s, n = cyclic_rows(H, rank, world)
    m = max_rows(H, world)
    local_buf = torch.zeros((m, W, 3), dtype=torch.float32, device=f"cuda:{local}")
    opts = rt.make_opts(cam, seed=args.seed, row_begin=b, row_step=s, n_rows=n,
                        flags=rt.RT_FLAG_OVERWRITE, device=local)
    stream = torch.cuda.current_stream()
    # The frame gather to rank 0 (surely_rt.parallel.gather_choice): at N > 1 with a GPU per rank
    # the product's C-ABI gather, rt_gather_frame (one ncclGather + the de-interleave kernel on
    # rank 0, librtgather.so); torch.distributed only carries its communicator id. The one-GPU
    # rehearsal keeps torch.distributed.gather over gloo.
    gather_name = gather_choice(world, rehearse)
    # RT_BENCH_RCCL1=1: the N > 1 gather code on one GPU (a one-rank RCCL communicator in this
    # torch process), the rehearsal of the driver's multi-GPU path that a one-GPU box allows
    if world == 1 and os.environ.get("RT_BENCH_RCCL1") == "1":
        gather_name = GATHER_RCCL
    rccl = None
    if gather_name == GATHER_RCCL:
        uid = [RcclFrameGather.unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        rccl = RcclFrameGather(uid[0], world, rank, device=local)
        if rank == 0:
            scratch = torch.empty((world * m, W, 3), dtype=torch.float32, device=f"cuda:{local}")
            frame_buf = torch.empty((H, W, 3), dtype=torch.float32, device=f"cuda:{local}")

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        ds.render_device(cam, opts, local_buf.data_ptr(), stream.cuda_stream)
        if ev is not None:
            ev[1].record(stream)
        if rccl is not None:
            rccl.gather(local_buf.data_ptr(), W, H, scratch.data_ptr() if rank == 0 else 0,
                        frame_buf.data_ptr() if rank == 0 else 0, stream.cuda_stream)
            out = frame_buf if rank == 0 else None
        else:
            out = gather_frame(local_buf.cpu() if rehearse else local_buf, H, rank, world)
        if ev is not None:
            ev[2].record(stream)  # the gather has completed on this stream
        return out

    # ---- op counts for the roofline (outside the timed region; deterministic)
    ops = None
    if not args.no_count:
        copts = rt.make_opts(cam, seed=args.seed, row_begin=b, row_step=s, n_rows=n,
                             flags=rt.RT_FLAG_OVERWRITE | rt.RT_FLAG_COUNT_OPS, device=local)
        st = ds.render_device(cam, copts, local_buf.data_ptr(), stream.cuda_stream, stats=True)
        ops = st.op_counts()

    # one product render with stats (outside the timed region): the bytes the path kernel
    # stores per launch (f64 segment partials + tail samples: its workspace)
    pst = ds.render_device(cam, opts, local_buf.data_ptr(), stream.cuda_stream, stats=True)
    out_bytes_launch = pst.out_bytes / max(1, pst.launches)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    events = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3))
              for _ in range(args.steps)]
    t0 = time.perf_counter()
    frame = None
    for k in range(args.steps):
        frame = step(events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    local_elapsed = elapsed
    t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearse else f"cuda:{local}")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    step_gpu_ms = sum(e[0].elapsed_time(e[1]) for e in events) / max(1, args.steps)
    gather_ms = sum(e[1].elapsed_time(e[2]) for e in events) / max(1, args.steps)
    # the roofline's kernel: rt_trace alone (HIP events the library records around its launches
    # on this stream), excluding the per-pixel reduction that step_gpu_ms also contains
    trace = ds.trace_ms(args.steps)
    kernel_ms = sum(trace) / max(1, len(trace))

    # the product kernel that ran: scene-specialised (world walker generated from the scene,
    # compiled by hiprtc at the first render, outside the timed region) or the interpreter
    # N > 1: every rank's kernel, render and gather times to rank 0 (outside the timed region)
    ranks = None
    if world > 1:
        ranks = rank_report({"trace_ms": kernel_ms, "render_ms": step_gpu_ms,
                             "gather_ms": gather_ms, "step_ms": local_elapsed / args.steps * 1e3,
                             "rows": n}, rank, world)
    jstate, jmsg = ds.jit_info()
    walker = ("scene-specialised (rt_jit.cpp, hiprtc)" if jstate == 1
              else f"interpreter ({jmsg.splitlines()[0] if jmsg else 'jit state %d' % jstate})")
    if rank == 0:
        total = W * H * spp * args.steps
        value = total / elapsed / 1e6
        res = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (procedural reference scene, no input data)",
            "config": {
                "workload": f"{args.scene} {W}x{H}, {args.spp}->{spp} spp, depth {cam.max_depth}"
                            f" ({args.config_name})",
                "width": W, "height": H, "spp_effective": spp, "max_depth": cam.max_depth,
                "seed": args.seed, "parallelism": f"cyclic rows x{world}, gather to rank 0",
                "walker": walker,
                "precision": "rays, hits and every path decision f64 (the reference's); radiance "
                             "weights f32, sums f64 (DESIGN.md §2)",
            },
            "gather": gather_name,
        }
        if ranks is not None:
            res["ranks"] = ranks
            res["ranks"]["note"] = ("per rank: rt_trace ms (HIP events), render ms (rt_trace + "
                                    "rt_reduce), gather ms (the frame gather to rank 0, events "
                                    "on the rank's stream), step ms (host clock), rows")
            proj = SCALING_PROJECTION.get((args.config_name, world))
            if proj is not None:
                res["scaling_projection"] = {
                    "efficiency": proj, "source": "profiles/r03_scaling_probe_adaptive.log",
                    "kind": "projection, not a measurement: one GPU renders each rank's cyclic "
                            "share in turn; efficiency = full frame / (N x slowest share)"}
        if ops is not None:
            # flops of the rank-0 launch (its share of rows) over its kernel time; kernel_ms is
            # per render, i.e. summed over the render's launches (stratum-row chunks)
            fl = roofline.flops(ops)
            ach = fl / (kernel_ms * 1e-3) / 1e12
            # PMC HBM bytes per rt_trace launch, measured by tools_gpu/profile_round.sh at N = 1
            # for this exact workload (null otherwise: a rank's launch at N > 1 is a different size)
            prof = None
            tf = REPO / "profiles" / f"pmc_traffic_{args.config}.json"
            if world == 1 and args.config_name != "custom" and tf.exists():
                try:
                    prof = json.loads(tf.read_text())
                except Exception:
                    prof = None
            # a profile of another kernel build is stale: its bytes are not this kernel's
            stale = None
            if prof and prof.get("kernel_source_sha16") != roofline.kernel_source_sha16():
                stale = (f"profiles/{tf.name} was collected on kernel sources "
                         f"{prof.get('kernel_source_sha16')}, this tree is "
                         f"{roofline.kernel_source_sha16()}: traffic not reported")
                prof = None
            traffic = prof.get("hbm_bytes_per_launch") if prof else None
            res["roofline"] = {
                "bound": "valu", "achieved": round(ach, 3),
                "peak": roofline.PEAK_FP64_VECTOR_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / roofline.PEAK_FP64_VECTOR_TFLOPS, 4),
                "traffic": traffic,
                "traffic_source": (f"profiles/{tf.name} (rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE "
                                   "passes of this workload, per rt_trace launch; not this run)"
                                   if traffic is not None else None),
                "kernel": "rt_trace", "kernel_ms": round(kernel_ms, 3),
                "launches_per_render": pst.launches,
                "render_ms": round(step_gpu_ms, 3),
                "flops_per_launch": fl / max(1, pst.launches),
                "flops_per_sample": round(fl / ops["samples"], 1),
                # the path's only mandatory HBM traffic is the framebuffer, W*H*12 B
                # of f32 RGB per frame (written by rt_reduce). rt_trace's own stores are the f64
                # partial-sum workspace, a design choice reported separately.
                "algorithmic_bytes_per_frame": W * n * 12,
                "workspace_bytes_per_launch": out_bytes_launch,
            }
            if stale:
                res["roofline"]["traffic_note"] = stale
            if traffic is not None:
                res["roofline"]["traffic_per_algorithmic_byte"] = round(
                    traffic * pst.launches / (W * n * 12), 1)
            if traffic is not None:
                launch_s = kernel_ms * 1e-3 / max(1, pst.launches)
                res["hbm"] = {
                    "achieved": round(traffic / launch_s / 1e9, 2),
                    "peak": roofline.PEAK_HBM_GBPS, "unit": "GB/s",
                    "frac": round(traffic / launch_s / 1e9 / roofline.PEAK_HBM_GBPS, 5),
                    "fetch_bytes_per_launch": prof.get("fetch_bytes"),
                    "write_bytes_per_launch": prof.get("write_bytes"),
                    "note": "measured PMC bytes (profile above) / this run's rt_trace time; the "
                            "kernel is FP64-VALU bound, HBM is not its roof",
                }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(blob, cam, args.seed, args.cpu_seconds)
            res["speedup_vs_cpu"] = round(value / res["cpu_baseline"]["value"], 1)
        assert frame is not None and frame.shape == (H, W, 3)
        print(json.dumps(res), flush=True)
    ds.close()
    if rccl is not None:
        rccl.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
