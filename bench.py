"""bench.py — BASELINE.json's headline: Mpaths/s (path segments traced per second) and ms/frame
for scenes/cornell.json at 800x800, depth 8, stream compaction on (BASELINE configs[1]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--pipeline fused|staged]
                    [--shard pixels|samples] [--no-cpu-baseline] [--no-configs]

A "step" is one pathtrace() frame's worth of work per GPU: one sample for every pixel, all
bounces, accumulated into the HBM-resident image (the reference's per-frame 7.68 MB D->H copy is
outside `value`; the API-faithful single-frame time including it is `api`).

N GPUs: one process per GPU.  `python bench.py --gpus N` without WORLD_SIZE starts
`torch.distributed.run --nproc-per-node N` as a child process (before touching any GPU) and exits
with its code; under torchrun WORLD_SIZE must equal --gpus.  Default sharding is by PIXEL TILE
(the north star's partition): rank r traces the interleaved row bands
(y // rows) % N == r of every frame, for N x K frames, so per-GPU work is K frames' worth of
paths (weak scaling) and the whole job is N x K samples per pixel.  The only exchange is one
gather of the ranks' disjoint tiles into rank 0's framebuffer (RCCL over xGMI), inside the timed
region; the result is bit-identical to one GPU tracing the same N x K frames.  `--shard samples`
instead gives each rank whole frames (a contiguous block of iterations) and sums the full
framebuffers with one RCCL reduce.

Timing: W untimed frames, then barrier + device sync, K steps, device sync + barrier; the MAX over
ranks of the elapsed time; value = segments traced by all ranks / that time.  The timed frames run
as the library runs them: one hipGraph per multi-frame pass, replayed back to back.  On one GPU the
same frames are then replayed eagerly with HIP start/stop events on every kernel
(hipExtLaunchKernel, on the library's stream): the dominant kernel's average launch duration for
`roofline` (algorithmic bytes / duration).  Then, still on one GPU: `api` times single
pt_trace() calls as main.cpp:463 makes them (F = 1, image copied to host memory every frame),
`configs` adds BASELINE configs[2..4] as sub-records (own workload string and roofline each), and
rank 0 times the CPU oracle (oracle/, the port of the reference path with stream_compaction/cpu.cu's
compactWithScan) on a bounded sample for `cpu_baseline`.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "project3-cuda-path-tracer-2025_amd")
SCENE = os.path.join(REPO, "scenes", "cornell.json")
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E, MI355X_MICROARCH.md chip table
REF_MS_PER_FRAME = 42.204      # reference README.md:136, RTX 3060 Laptop, compaction on
STATE_BYTES = 48               # one path in flight: 3 x float4 (origin|pixel, dir|bounces, rgb|-)
IMAGE_RMW_BYTES = 24           # terminated path: read + write its pixel's float3 (1-frame pass)
PLANE_STORE_BYTES = 12         # terminated path of an F-frame pass: float3 store to its frame's plane
QUEUE_ENTRY_BYTES = 64         # mesh scenes: a ray queued for k_bvh_bounce (written by k_bounce, read back)
# mesh scenes: a traversal handed over by k_bvh_bounce: its state (queue slot + saved node 8 B, best hit 16 B,
# 4 B per stack entry) written and read back by k_bvh_tail_trav, its final hit (16 B) written there, slot and
# hit read again by k_bvh_tail_shade (24 B), and the queue entry re-read (the ray, 32 B, by the traversal; all
# 64 B by the shading): 24 + 24 + 16 + 24 + 32 + 64 = 184 B + 8 B per stack entry
HANDOVER_BYTES = 184
HANDOVER_STACK_BYTES = 8
N_CUS = 256                    # MI355X compute units

# BASELINE.json configs[2..4] as sub-records of the N=1 line: (tag, scene, res, depth, sort, pipeline, steps, warmup
# [, options]), then the reference's large-mesh scenes (cornell_obj_cyrene.json:266, README.md:206; 262k / 1.0M
# triangle stand-ins) on the pair layout and, for comparison, on the node-array traversal they took until round 5
VAR_NODE_ARRAY = 186 | 64      # the default variant + VAR_BVH_NODES (no pair layout, no traversal queue)
SUB_CONFIGS = [
    ("configs[2]", "cornell_glass_test.json", None, None, True, "fused", 48, 4),
    ("configs[2] staged", "cornell_glass_test.json", None, None, True, "staged", 48, 4),
    ("configs[2] sort off", "cornell_glass_test.json", None, None, False, "fused", 48, 4),
    ("configs[3]", "cornell_obj_bnnuy.json", None, None, False, "fused", 48, 4),
    ("configs[4]", "cornell_obj_khaslana.json", (1600, 1600), 12, False, "fused", 32, 2),
    ("mesh 262k", "cornell_obj_cyrene.json", None, None, False, "fused", 24, 2),
    ("mesh 262k node array", "cornell_obj_cyrene.json", None, None, False, "fused", 8, 1, {"variant": VAR_NODE_ARRAY}),
    ("mesh 1.0M", "cornell_obj_phainon.json", None, None, False, "fused", 24, 2),
    ("mesh 1.0M node array", "cornell_obj_phainon.json", None, None, False, "fused", 8, 1, {"variant": VAR_NODE_ARRAY}),
]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--pipeline", choices=["fused", "staged"], default="fused")
    ap.add_argument("--scene", default=SCENE)
    ap.add_argument("--sort", action="store_true", help="material sort (MATERIAL_SORTING, configs[2])")
    ap.add_argument("--res", default="", help="WxH override (configs[4]: 1600x1600)")
    ap.add_argument("--depth", type=int, default=-1, help="trace depth override (configs[4]: 12)")
    ap.add_argument("--variant", type=int, default=-1, help="kernel variant bits (A/B; default: the library's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the configs[2..4] sub-records")
    ap.add_argument("--no-api", action="store_true", help="skip the single-frame pt_trace() timing")
    ap.add_argument("--no-spread", action="store_true", help="skip the per-pass median / p90 timing")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--shard", choices=["pixels", "samples"], default="pixels",
                    help="N>1: pixels = interleaved row bands of every frame per rank (default); "
                         "samples = whole frames per rank")
    ap.add_argument("--dump-image", default="", help="rank 0 saves the final accumulated image (.npy)")
    ap.add_argument("--inproc", action="store_true",
                    help="ONE process driving --gpus N devices behind one pathtrace() (pt_options.num_devices: "
                         "the path the drop-in and pt_render take), instead of one process per GPU")
    ap.add_argument("--inproc-devices", default="",
                    help="--inproc device list, e.g. 0,0 to rehearse on one GPU (default 0..N-1)")
    ap.add_argument("--combine", choices=["peer", "rccl"], default="peer", help="--inproc: how shards reach device 0")
    ap.add_argument("--no-inproc", action="store_true",
                    help="N>1 under torchrun: skip rank 0's follow-up --inproc run of the same N")
    return ap.parse_args()


def launch_ranks(args) -> int:
    """`--gpus N` without a launcher: run torch.distributed.run as a CHILD process (never an exec,
    and before this process touches any GPU), one rank per GPU, and return its exit code."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def shard_rows(height: int, world: int) -> int:
    """Row-band height: the largest of 8/4/2/1 that splits the image evenly over the ranks."""
    for rows in (8, 4, 2, 1):
        if height % (rows * world) == 0:
            return rows
    return 1


def inproc_main(args):
    """`--gpus N --inproc`: one process, one PathTracer over N devices (pt_options.num_devices),
    every frame split into interleaved row bands across them and combined into device 0's image
    after each call (k_gather_shards over xGMI peer access, or RCCL).  Weak scaling like the
    torchrun line: K steps of N frames each, so every device traces K frames' worth of paths."""
    sys.path.insert(0, PKG)
    import ptamd   # noqa: E402  (no torch: the library's own HIP runtime)
    n = args.gpus
    devices = [int(x) for x in args.inproc_devices.split(",")] if args.inproc_devices else list(range(n))
    n = len(devices)
    scene = ptamd.SceneFile(args.scene)
    tr = ptamd.PathTracer(scene, devices=devices, combine=args.combine)
    per_step = n
    it = 1
    if args.warmup:
        tr.trace_frames(it, args.warmup * per_step)
        it += args.warmup * per_step
    tr.synchronize()
    tr.reset_stats()
    tr.prepare_frames(args.steps * per_step)
    tr.synchronize()
    t0 = time.perf_counter()
    tr.trace_frames(it, args.steps * per_step)        # every shard's passes, then one combine
    tr.synchronize()
    el = time.perf_counter() - t0
    it += args.steps * per_step
    st = tr.stats()
    assert st["frames_total"] == args.steps * per_step
    # the API call (one frame per pathtrace(), image copied to host), as main.cpp:463 makes it: each
    # shard speculates its next frame and copies its own row bands over its own link; then the same
    # calls with the speculation off
    def api_calls(first):
        ts = []
        for k in range(25):
            t1 = time.perf_counter()
            tr.trace(first + k, copy_image=True)
            if k >= 5:
                ts.append(1e3 * (time.perf_counter() - t1))
        ts.sort()
        return round(ts[len(ts) // 2], 4)
    api_ms = api_calls(it)
    tr.set_speculation(False)
    api_ms_nospec = api_calls(it + 25)
    tr.free()
    out = {"metric": "Mpaths/s (rays x bounces / s), 800x800 cornell depth 8", "mode": "inproc",
           "value": round(st["segments_total"] / el / 1e6, 2), "unit": "Mpaths/s", "n_gpus": n,
           "devices": devices, "combine": args.combine, "steps": args.steps, "warmup": args.warmup,
           "frames_per_step": per_step, "ms_per_step": round(1e3 * el / args.steps, 4),
           "ms_per_frame": round(1e3 * el / (args.steps * per_step), 4),
           "api_ms_per_frame": api_ms, "api_ms_per_frame_no_speculation": api_ms_nospec,
           "parallelism": f"one process, pt_options.num_devices={n}: interleaved 8-row bands per device, "
                          f"one combine into device 0 per call ({args.combine})"}
    print(json.dumps(out), flush=True)


def inproc_child(args, world):
    """Rank 0 of a torchrun job, after the other ranks have exited: the same N GPUs once more, as
    ONE process behind one pathtrace() (--inproc), so the scaling run also times the path the
    reference's callers get.  A child process with a time limit: its failure is recorded, not fatal."""
    cmd = [sys.executable, os.path.abspath(__file__), "--gpus", str(world), "--inproc", "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--scene", args.scene]
    # PT_BENCH_INPROC_DEVICES (e.g. "0,0"): the device list for a rehearsal with ranks sharing one GPU
    if os.environ.get("PT_BENCH_INPROC_DEVICES"):
        cmd += ["--inproc-devices", os.environ["PT_BENCH_INPROC_DEVICES"]]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE",
                                                              "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID")}
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    except subprocess.TimeoutExpired:
        return {"error": "timed out after 240 s"}
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"error": f"exit {p.returncode}", "stderr": p.stderr[-600:]}
    return json.loads(lines[-1])


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if args.inproc:
        if env_world is not None and int(env_world) > 1:
            print("bench.py: --inproc is one process; do not start it under torchrun", file=sys.stderr)
            sys.exit(2)
        inproc_main(args)
        return
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    import torch                     # first: ptamd then shares torch's HIP runtime
    import torch.distributed as dist
    sys.path.insert(0, PKG)
    import ptamd
    from ptamd import dist as pdist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RCCL (backend "nccl") in production; PT_BENCH_BACKEND=gloo rehearses the multi-rank logic
    # with several ranks sharing one GPU (the framebuffer combine then goes through host memory)
    backend = os.environ.get("PT_BENCH_BACKEND", "nccl")
    n_dev = torch.cuda.device_count()
    if world > 1 and backend == "nccl" and world > n_dev:
        # one rank per GPU: RCCL ranks stacked on one device would time a different job
        print(f"bench.py: {world} RCCL ranks but {n_dev} visible GPUs (PT_BENCH_BACKEND=gloo rehearses "
              "ranks that share a GPU)", file=sys.stderr)
        sys.exit(2)
    device = local % max(1, n_dev)
    if world > 1:
        torch.cuda.set_device(device)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)

    res = tuple(int(x) for x in args.res.split("x")) if args.res else None
    scene = ptamd.SceneFile(args.scene, res=res, depth=args.depth if args.depth >= 0 else None)
    pipeline = ptamd.PIPELINE_STAGED if args.pipeline == "staged" else ptamd.PIPELINE_FUSED
    pixels = world > 1 and args.shard == "pixels"
    rows = shard_rows(scene.height, world) if pixels else 8
    shard = dict(shard_mode=ptamd.SHARD_PIXELS, shard_rank=rank, shard_count=world, shard_rows=rows) if pixels else {}
    if args.variant >= 0:
        shard["variant"] = args.variant
    tr = ptamd.PathTracer(scene, device=device, pipeline=pipeline, material_sort=int(args.sort), **shard)
    depth = scene.trace_depth

    # iterations: PIXELS -- every rank traces iterations 1..N(W+K) over its own tiles (N frames per
    # step); SAMPLES -- rank r traces the contiguous block 1 + r(W+K) .. (r+1)(W+K)
    per_step = world if pixels else 1
    it = 1 + (0 if pixels else rank * (args.warmup + args.steps))
    if args.warmup:
        tr.trace_frames(it, args.warmup * per_step)
        it += args.warmup * per_step
    tr.synchronize()
    tr.reset_stats()
    combiner = None
    if world > 1:
        combiner = (pdist.TileGather(tr, rows, world, rank, backend, device) if pixels
                    else pdist.ImageReduce(tr, rank, backend, device))

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()      # same HIP runtime as the library: covers its stream too
        tr.synchronize()

    tr.prepare_frames(args.steps * per_step)           # capture the pass graphs now, not while timed
    barrier()
    t0 = time.perf_counter()
    tr.trace_frames(it, args.steps * per_step)         # K steps: the pass graphs, back to back
    t_comb = 0.0
    if combiner is not None:
        tr.synchronize()
        tc = time.perf_counter()
        combiner.run()                                 # one framebuffer combine (RCCL over xGMI)
        t_comb = time.perf_counter() - tc
    tr.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    it += args.steps * per_step

    st = tr.stats()
    segs = st["segments_total"]
    assert st["frames_total"] == args.steps * per_step, (st["frames_total"], args.steps, per_step)
    if args.dump_image and rank == 0:
        np.save(args.dump_image, tr.image())
    prof = st_prof = spread = None
    if world == 1:
        # kernel durations: the next K frames replayed eagerly with events around every kernel
        tr.reset_stats()
        gap = float(os.environ.get("PT_BENCH_PROF_GAP", "0"))
        if gap > 0:
            time.sleep(gap)
        prof = tr.profile(it, args.steps)
        st_prof = tr.stats()
        spread = None if args.no_spread else pass_spread(tr, it + args.steps, st_prof["frames_per_pass"])
    seen_world = world
    if world > 1:
        t = torch.tensor([elapsed, float(segs), t_comb], dtype=torch.float64,
                         device="cuda" if backend == "nccl" else "cpu")
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed, segs, t_comb = float(tmax[0]), float(t[1]), float(tmax[2])
        seen_world = dist.get_world_size()
    ms_per_step = 1e3 * elapsed / args.steps
    value = segs / elapsed / 1e6

    if rank == 0:
        headline = (os.path.abspath(args.scene) == SCENE and not args.res and args.depth < 0 and not args.sort)
        name = os.path.basename(args.scene)
        workload = workload_str(name, tr.width, tr.height, depth, args.sort, args.pipeline)
        if world > 1:
            par = (f"pixel tiles x{world}: interleaved {rows}-row bands, {world} frames per step, tile gather "
                   f"to rank 0" if pixels else f"samples x{world}: whole frames per rank, framebuffer reduce")
        else:
            par = "single GPU"
        line = {
            "metric": "Mpaths/s (rays x bounces / s), 800x800 cornell depth 8" if headline
                      else f"Mpaths/s (rays x bounces / s), {workload}",
            "value": round(value, 2),
            "unit": "Mpaths/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(REF_MS_PER_FRAME / (ms_per_step / per_step), 2) if headline else None,
            "vs_baseline_basis": "reference ms/frame 42.204 (README.md:136, RTX 3060 Laptop) / our ms per frame"
                                 if headline else "no published reference number for this workload",
            "dtype": "f32",
            "data": f"scenes/{name} from the reference ({tr.width}x{tr.height}, depth {depth}, 1 spp per frame)"
                    + ("; synthetic stand-in meshes (reference OBJs absent)" if "obj" in name else
                       "; no synthetic inputs"),
            "config": {"workload": workload + (" (BASELINE configs[1])" if headline else ""),
                       "pipeline": args.pipeline,
                       "segments_per_frame": round(segs / (args.steps * per_step) / (1 if pixels else world), 1),
                       "frames_per_pass": st["frames_per_pass"], "parallelism": par},
        }
        if world > 1:
            line["distributed"] = {"world_size": seen_world, "backend": "rccl" if backend == "nccl" else backend,
                                   "shard": args.shard, "frames_per_step": per_step,
                                   "combine_ms": round(1e3 * t_comb, 3),
                                   "combine": "gather of disjoint row-band tiles" if pixels else "reduce(SUM)"}
        if prof is not None:
            line["roofline"] = roofline(prof, st_prof, args.pipeline, args.steps, depth, headline)
            line["kernels"] = kernels_digest(prof, spread)
        line["pcie_ms_per_frame"] = pcie_copy_ms(tr)
        if world == 1 and not args.no_api:
            line["api"] = api_frame_ms(tr, it + 3 * args.steps)
    tr.free()
    if rank == 0 and world == 1:
        if not args.no_configs:
            line["configs"] = [sub_config(ptamd, c) for c in SUB_CONFIGS]
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    if world > 1:
        dist.destroy_process_group()
        if rank == 0 and not args.no_inproc and (backend == "nccl" or os.environ.get("PT_BENCH_INPROC_DEVICES")):
            line["inproc"] = inproc_child(args, world)
    if rank == 0:
        print(json.dumps(line), flush=True)


def workload_str(name, w, h, depth, sort, pipeline):
    if sort and pipeline == "fused":
        s = "material sort on (block-local regrouping by material between intersection and shading)"
    elif sort:
        s = "material sort on (stable counting sort of the wavefront by material)"
    else:
        s = "sort off"
    return f"{name} {w}x{h} depth {depth}, stream compaction on, {s}"


def kernels_digest(prof, spread):
    d = {"frame_ms": round(prof["frame_ms"], 4), "passes": prof["passes"],
         "per_launch_bounce_ms": [round(x, 4) for x in prof["bounce_ms"]],
         "per_launch_bvh_ms": [round(x, 4) for x in prof["bvh_ms"]],
         "combine_ms_per_frame": round(prof["combine_ms"], 4)}
    if spread is not None:
        d["ms_per_frame_spread"] = spread
    return d


def traffic_tag(cfg):
    """The committed PMC digest (profiles/rNN_traffic_<tag>.json) of a SUB_CONFIGS entry: PMC passes
    of the same bench command (tools/r06_session.sh cfgpmc / khprof / cyrprof)."""
    _, scene_name, res, depth, sort, pipeline = cfg[:6]
    opts = cfg[8] if len(cfg) > 8 else {}
    if "bnnuy" in scene_name and res is None:
        return "c4_bunny"
    if "khaslana" in scene_name and res == (1600, 1600) and depth == 12:
        return "c5_khaslana"
    if "glass" in scene_name:
        return ("staged_c2" if pipeline == "staged" else "c2_glass") if sort else "c2_glass_sortoff"
    if "cyrene" in scene_name:
        return "m262k_cyrene_nodes" if opts else "m262k_cyrene"
    if "phainon" in scene_name:
        return "m1m_phainon_nodes" if opts else "m1m_phainon"
    return None


def sub_config(ptamd, cfg):
    """One BASELINE config on this GPU: warmup, K timed frames (pass graphs), eager profiled
    replay for its roofline.  Same timing rules as the headline."""
    tag, scene_name, res, depth, sort, pipeline, steps, warmup = cfg[:8]
    opts = cfg[8] if len(cfg) > 8 else {}
    path = os.path.join(REPO, "scenes", scene_name)
    sc = ptamd.SceneFile(path, res=res, depth=depth)
    tr = ptamd.PathTracer(sc, pipeline=ptamd.PIPELINE_STAGED if pipeline == "staged" else ptamd.PIPELINE_FUSED,
                          material_sort=int(sort), **opts)
    it = 1
    tr.trace_frames(it, warmup)
    it += warmup
    tr.synchronize()
    tr.reset_stats()
    tr.prepare_frames(steps)
    tr.synchronize()
    t0 = time.perf_counter()
    tr.trace_frames(it, steps)
    tr.synchronize()
    el = time.perf_counter() - t0
    it += steps
    st = tr.stats()
    tr.reset_stats()
    prof = tr.profile(it, steps)
    st_prof = tr.stats()
    d = sc.trace_depth
    out = {"config": tag, "workload": workload_str(scene_name, tr.width, tr.height, d, sort, pipeline),
           "pipeline": pipeline, "steps": steps, "warmup": warmup,
           "ms_per_frame": round(1e3 * el / steps, 4),
           "value": round(st["segments_total"] / el / 1e6, 2), "unit": "Mpaths/s",
           "segments_per_frame": round(st["segments_total"] / steps, 1), "frames_per_pass": st["frames_per_pass"],
           "data": "synthetic stand-in meshes (reference OBJs absent)" if "obj" in scene_name else "reference scene",
           "roofline": roofline(prof, st_prof, pipeline, steps, d, False,
                                traffic_file=traffic_tag(cfg)),
           "kernels": kernels_digest(prof, None)}
    if "obj" in scene_name:
        out["triangles"] = len(sc.triangles)
        q = sum(st["queued_total"])
        out["queued_share"] = round(q / max(1, st["segments_total"]), 4)      # paths that enter the mesh
        out["handed_share"] = round(sum(st["handed_total"]) / max(1, q), 4)   # ... of those, handed over
        out["handed_stack_mean"] = round(sum(st["handed_stack_total"]) / max(1, sum(st["handed_total"])), 2)
    if opts:
        out["options"] = opts
    if tag == "configs[4]":
        out["note"] = "BASELINE names 8 GPUs for this config; this sub-record is one GPU (bench.py --gpus 8 --scene ...)"
    tr.free()
    sc.close()
    return out


def pass_spread(tr, first_iteration, frames_per_pass, passes=16):
    """Median / p90 of ms per frame over `passes` separately timed passes (SURVEY §8d asks for
    median and p90 of frame time).  One sample = one whole multi-frame pass, graph replay and
    device sync included, divided by its frames: frames of a pass run concurrently, so a single
    frame has no time of its own.  Runs after the timed region; it is not part of `value`."""
    f = max(1, int(frames_per_pass))
    tr.prepare_frames(f)
    tr.synchronize()
    samples = []
    for p in range(passes):
        t0 = time.perf_counter()
        tr.trace_frames(first_iteration + p * f, f)
        tr.synchronize()
        samples.append(1e3 * (time.perf_counter() - t0) / f)
    samples.sort()
    pick = lambda q: samples[min(len(samples) - 1, int(round(q * (len(samples) - 1))))]  # noqa: E731
    return {"median": round(pick(0.5), 4), "p90": round(pick(0.9), 4), "passes": passes,
            "frames_per_pass": f, "note": "each pass timed alone (host wall clock incl. launch + sync)"}


def api_frame_ms(tr, first_iteration, frames=40, warm=5):
    """API-faithful frame: pathtrace(pbo, 0, iter) as main.cpp:463 calls it -- one
    frame per call (F = 1), the accumulated image copied into host memory every call
    (pathtrace.cu:783; the caller's pageable buffer, as the reference's cudaMemcpy) -- median / p90 of the
    host wall time per call, with and without that copy."""
    def run(copy, first):
        ts = []
        for k in range(warm + frames):
            t0 = time.perf_counter()
            tr.trace(first + k, copy_image=copy)
            if not copy:
                tr.synchronize()
            if k >= warm:
                ts.append(1e3 * (time.perf_counter() - t0))
        ts.sort()
        return round(ts[len(ts) // 2], 4), round(ts[int(0.9 * (len(ts) - 1))], 4)
    m_copy, p_copy = run(True, first_iteration)
    m_nc, p_nc = run(False, first_iteration + warm + frames)
    # the same calls with the next-frame speculation off (pt_set_speculation(0)): every frame
    # traced inside its own call, strictly before its copy
    tr.set_speculation(False)
    try:
        m_ns, p_ns = run(True, first_iteration + 2 * (warm + frames))
    finally:
        tr.set_speculation(True)
    return {"ms_per_frame": m_copy, "p90": p_copy, "ms_per_frame_no_copy": m_nc, "p90_no_copy": p_nc,
            "ms_per_frame_no_speculation": m_ns, "p90_no_speculation": p_ns,
            "frames": frames, "note": "pt_trace(F=1) + 7.68 MB D->H into the caller's pageable host memory per call; "
                                      "frame N+1 is traced on a second stream while frame N's image is copied "
                                      "(taken over bit-exactly by the call for N+1)"}


def _device_tensor(torch, ptr, n, device):
    """Zero-copy torch view of the library's image buffer (same HIP runtime)."""
    class _Cai:
        __cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False), "version": 2}
    return torch.as_tensor(_Cai(), device=f"cuda:{device}")


def roofline(prof, st, pipeline, steps, depth, headline=True, traffic_file=None):
    """Dominant kernel, per launch.  Fused: the bounce kernel (camera|intersect|shade|gather|
    compact; `depth` launches per pass of F frames): algorithmic bytes = 48 B per path read
    (bounce > 0) + 48 B per survivor written + 24 B image read-modify-write (or 12 B plane store)
    per terminated path, + (mesh scenes) the traversal queue's round trip per queued ray.  Staged: the compaction scatter kernel: 4 B flag per path in + 96 B per
    survivor (48 B read + 48 B written).  achieved = bytes per launch / average launch duration
    (hipExtLaunchKernel dispatch timestamps, pt_profile_frames)."""
    tot = st["live_total"]                 # per-bounce live counts summed over the timed frames
    queued = st.get("queued_total") or [0] * len(tot)
    handed = st.get("handed_total") or [0] * len(tot)
    handed_stack = st.get("handed_stack_total") or [0] * len(tot)
    launches = depth * prof["passes"]
    nbytes = 0
    for b in range(depth):
        n_in, n_out = tot[b], tot[b + 1] if b + 1 < len(tot) else 0
        if pipeline == "fused":
            gather = IMAGE_RMW_BYTES if st["frames_per_pass"] == 1 else PLANE_STORE_BYTES
            nbytes += (STATE_BYTES * n_in if b > 0 else 0) + STATE_BYTES * n_out + gather * (n_in - n_out)
            nbytes += 2 * QUEUE_ENTRY_BYTES * queued[b]      # traversal queue round trip
            nbytes += HANDOVER_BYTES * handed[b] + HANDOVER_STACK_BYTES * handed_stack[b]   # hand-over
        else:
            nbytes += 4 * n_in + 2 * STATE_BYTES * n_out
    if pipeline == "fused" and any(prof["bvh_ms"][:depth]):
        name = ("k_bounce + k_bvh_bounce + k_bvh_tail_trav + k_bvh_tail_shade (fused bounce; mesh rays "
                "traversed and shaded by the second kernel, the last rays of its waves by the third and fourth), "
                "one set of launches per bounce per pass")
    elif pipeline == "fused":
        name = "k_bounce (fused camera|intersect|shade|gather|compact, one launch per bounce per pass)"
    else:
        name = "k_compact_scatter (stable partition: flags + survivor payload move)"
    bytes_per_launch = nbytes / launches
    avg_ms = sum(prof["bounce_ms"][:depth]) / depth
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    pmc = _pmc(name) if headline else {}     # the committed PMC pass is of the headline run
    # measured HBM bytes per launch: the PMC run's bytes per frame x this run's frames per launch
    traffic = (int(pmc["hbm_bytes_per_frame"] * steps / launches) if pmc.get("hbm_bytes_per_frame")
               else pmc.get("hbm_bytes_per_launch"))
    if traffic_file:
        # a config with its own committed PMC digest (profiles/rNN_traffic_<tag>.json): both
        # kernels of a bounce, bytes per frame scaled to this run's frames per launch pair
        keys = (("k_bounce", "k_bvh_bounce", "k_bvh_tail_trav", "k_bvh_tail_shade") if pipeline == "fused"
                else ("k_compact_scatter",))
        per_frame = sum(v.get("hbm_bytes_per_frame", 0) for k, v in _pmc_digest(traffic_file).items() if k in keys)
        traffic = int(per_frame * steps / launches) if per_frame else None
    line = {"kernel": name, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "bytes_per_launch": int(bytes_per_launch), "avg_launch_ms": round(avg_ms, 5), "launches": launches,
            "duration_source": "HIP start/stop events per dispatch (hipExtLaunchKernel) over an eager replay of "
                               "K frames right after the timed region"}
    if pmc.get("SQ_INSTS_VALU") and pmc.get("GRBM_GUI_ACTIVE"):
        # what binds the fused kernel is vector-instruction issue, not HBM: a CU issues at most 2
        # wave64 VALU instructions per clock (4 SIMD-32 units, 2 cycles each; MI355X_MICROARCH.md);
        # GRBM_GUI_ACTIVE sums the 8 XCDs' clocks
        clk = pmc["GRBM_GUI_ACTIVE"] / 8.0
        rate = pmc["SQ_INSTS_VALU"] / (clk * N_CUS)
        line["valu_issue"] = {"achieved": round(rate, 3), "peak": 2.0, "unit": "wave64 VALU instr / CU / clk",
                              "frac": round(rate / 2.0, 3), "source": f"profiles/{_pmc_file()} (rocprofv3 PMC)"}
    return line


def _pmc_file():
    """The newest committed PMC digest of the headline run (profiles/rNN_traffic.json)."""
    d = os.path.join(REPO, "profiles")
    names = sorted(f for f in os.listdir(d) if f.endswith("_traffic.json") and f[1:3].isdigit()) if os.path.isdir(d) else []
    return names[-1] if names else "r01_traffic.json"


def _pmc_digest(tag):
    """The newest committed PMC digest of a config run, profiles/rNN_traffic_<tag>.json."""
    d = os.path.join(REPO, "profiles")
    names = sorted(f for f in os.listdir(d) if f.endswith(f"_traffic_{tag}.json")) if os.path.isdir(d) else []
    if not names:
        return {}
    with open(os.path.join(d, names[-1])) as f:
        return json.load(f)


def _pmc(name):
    """The kernel's per-launch PMC digest from the committed rocprofv3 pass: HBM bytes
    (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction) and counters."""
    p = os.path.join(REPO, "profiles", _pmc_file())
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        d = json.load(f)
    key = "k_bounce" if name.startswith("k_bounce") else "k_compact_scatter"
    return d.get(key, {})


def pcie_copy_ms(tr):
    """The reference copies the accumulated image to the host every frame (pathtrace.cu:783):
    time one such copy into fresh pageable memory (the `api` record copies into a reused buffer)."""
    tr.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        tr.image()
    return round((time.perf_counter() - t0) / 5 * 1e3, 3)


def cpu_baseline(budget_s):
    """The oracle (C port of the reference path: serial intersect/shade loops + cpu.cu's
    compactWithScan) on this host, BASELINE configs[0] (cornell 400x400 depth 4): 1 thread for
    `value`, and the same at this process's CPU share (OpenMP over paths) beside it."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    sc = O.load_scene(SCENE, res=(400, 400), depth=4)

    def run(threads, seconds):
        r = O.Renderer(sc, O.options(num_threads=threads))
        segs, frames, t0 = 0, 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds or frames < 2:
            frames += 1
            segs += int(np.maximum(r.trace(frames), 0).sum())
        el = time.perf_counter() - t0
        return segs / el / 1e6, frames, el

    v1, f1, e1 = run(1, budget_s)
    nt = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count() or 1))
    vn, fn, en = run(nt, budget_s / 2)
    # the headline workload itself (BASELINE configs[1], cornell 800x800 depth 8) on the same host,
    # so the GPU line has a CPU number of the same work beside it: a few frames at 1 thread
    # (~0.45 s each) and at the process's CPU share
    sc = O.load_scene(SCENE)
    h1, hf1, he1 = run(1, budget_s / 2)
    hn, hfn, hen = run(nt, budget_s / 4)
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"value": round(v1, 3), "unit": "Mpaths/s", "cores": 1, "kind": "port", "cpu_model": model,
            "sample": f"cornell.json 400x400 depth 4 (BASELINE configs[0]), {f1} frames in {e1:.1f} s, "
                      f"{e1 / f1 * 1e3:.1f} ms/frame, oracle/pt_oracle.c single thread",
            "ms_per_frame": round(e1 / f1 * 1e3, 2),
            "multithread": {"value": round(vn, 3), "unit": "Mpaths/s", "cores": nt,
                            "sample": f"same workload, {fn} frames in {en:.1f} s, OpenMP over paths"},
            "configs1": {"workload": "cornell.json 800x800 depth 8, stream compaction on (BASELINE configs[1], "
                                     "the GPU headline's workload)",
                         "value": round(h1, 3), "unit": "Mpaths/s", "cores": 1,
                         "ms_per_frame": round(he1 / hf1 * 1e3, 2),
                         "sample": f"{hf1} frames in {he1:.1f} s, oracle/pt_oracle.c single thread",
                         "multithread": {"value": round(hn, 3), "unit": "Mpaths/s", "cores": nt,
                                         "ms_per_frame": round(hen / hfn * 1e3, 2),
                                         "sample": f"{hfn} frames in {hen:.1f} s, OpenMP over paths"}}}


if __name__ == "__main__":
    main()
