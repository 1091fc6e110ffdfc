#!/usr/bin/env python3
"""Benchmark of the MI355X path-tracing inner loop (BASELINE.json metric).

Workload (BASELINE.json configs[1], the default): sample_scenes[0]
(make_scene_box), 1024^2, 256 spp, n_rays 16, depth_max 8, fp32, synthetic =
the scene itself. A *step* renders `--spp-per-step` sample passes of the
frame (one ipt_render_device call: raygen + path kernel + GridRenderPlane
accumulate kernel); the default c2 step is the full 256-spp frame, rendered
by one path-kernel launch.

Multi-GPU (torchrun, one rank per GPU): the frame's destination rows are cut
into 16-row tiles dealt round-robin to the ranks (ipt_params.tile_rows /
n_shards / shard_id); the path needs no data-path collective. The finished
frame is assembled on rank 0 at the end of the timed region by ONE gather of
each rank's owned rows (16 B per owned pixel: GridRenderPlane pixels,
counters, sums, max), scattered into place on rank 0.
  --scaling weak   (c1, c2 default): the frame stays W x H and every rank
                   renders its tiles at N x spp-per-step passes per step, so
                   the per-rank work is the 1-GPU workload ("1024^2 x N-spp");
  --scaling strong (c3, c4, c5 default): the frame and its passes are fixed
                   (C4: 4096^2, C5: 2048^2) and split over the ranks.
Either way the ranks render disjoint tiles of one frame, so the tile load
imbalance shows in `ranks` (per-rank path-kernel ms and path counts).

--config c1 is BASELINE.json configs[0], the reference's CPU-runnable case
(256^2, 16 spp, 4 bounces): the GPU renders it and the CPU baseline leg runs
the WHOLE C1 frame on the oracle (the C1 plumbing number).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

# BASELINE.json configs: scene, width, height, spp per step, steps, depth_max,
# default scaling, CPU-baseline sample (row stride, column stride) per call.
# c2's step is the whole 1024^2 x 256 spp frame (one launch of 268 M paths);
# c3/c4/c5 sample their full spp counts with calls of 33.6 M / 537 M / 268 M
# paths, so that the persistent kernel's end-of-launch tail (lanes out of
# work while the longest paths finish) stays a small share of each launch
# (c3's two 32-spp steps are its whole 64-spp frame; at 16 spp per call the
# tail cost it 6 %: 13.35 vs 14.23 Mpaths/s).
CONFIGS = {
    "c1": ("box", 256, 256, 16, 1, 4, "weak", None),                 # configs[0]: CPU plumbing case
    "c2": ("box", 1024, 1024, 256, 2, 8, "weak", (64, 1)),           # configs[1]: the metric
    "c3": ("spheres10k", 1024, 1024, 32, 2, 8, "strong", (128, 64)),  # configs[2]: 10k spheres, 2 steps = the 64-spp frame
    "c4": ("box", 4096, 4096, 32, 2, 8, "strong", (256, 4)),         # configs[3]: 4096^2 tiles (1024 spp in full)
    "c5": ("lights256", 2048, 2048, 64, 2, 8, "strong", (128, 16)),  # configs[4]: 256 emitters (512 spp in full)
}
METRIC = "Mpaths/sec at 1024^2, 8-bounce, sample_scenes[0]; achieved HBM GB/s"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS),
                    help="BASELINE.json workload: c2 (default, the metric's config), c1 the CPU plumbing "
                         "case, c3 10k spheres, c4 4096^2 multi-GPU, c5 256 emitters")
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--spp-per-step", type=int, default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--scaling", choices=("weak", "strong"), default=None)
    ap.add_argument("--n-rays", type=int, default=16)
    ap.add_argument("--depth-max", type=int, default=None)
    ap.add_argument("--seed", type=int, default=20241223)
    ap.add_argument("--tile-rows", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=30.0,
                    help="minimum duration of the CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0 = this process's CPU share, see cpu_threads())")
    ap.add_argument("--no-counters", action="store_true",
                    help="skip the (untimed) counting re-render used for the roofline")
    ap.add_argument("--sync", action="store_true",
                    help="one synchronous ipt_render_device per step instead of queuing the steps with "
                         "ipt_render_device_async (which lets each step's launch fill the previous one's tail)")
    ap.add_argument("--verify", action="store_true",
                    help="N>1: rank 0 re-renders the whole frame unsharded after the timing and "
                         "compares it bit for bit with the assembled one")
    a = ap.parse_args()
    scene, w, h, spp, steps, depth, scaling, cpu_sample = CONFIGS[a.config]
    a.scene = scene
    a.width = a.width or w
    a.height = a.height or h
    a.spp_per_step = a.spp_per_step or spp
    a.steps = a.steps or steps
    a.depth_max = depth if a.depth_max is None else a.depth_max
    a.scaling = a.scaling or scaling
    a.cpu_sample = cpu_sample
    return a


def make_desc(name):
    from ipt_amd import scenes

    if name == "box":
        return scenes.make_scene_box()
    if name == "lights256":
        return scenes.make_scene_box_lights(16)
    if name == "spheres10k":
        return scenes.make_scene_spheres(10000, seed=1)
    raise ValueError(name)


def cpu_threads(requested: int = 0) -> int:
    """Threads of the CPU baseline: this process's CPU affinity, capped at the
    job's CPU share (OMP_NUM_THREADS: 16 per GPU on the GPU box, where
    os.cpu_count() shows the whole machine)."""
    if requested > 0:
        return requested
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def physical_cores() -> int | None:
    """Physical cores of the host (distinct (package, core) pairs in sysfs)."""
    import glob

    ids = set()
    for d in glob.glob("/sys/devices/system/cpu/cpu[0-9]*/topology"):
        try:
            ids.add((open(f"{d}/physical_package_id").read().strip(), open(f"{d}/core_id").read().strip()))
        except OSError:
            pass
    return len(ids) or None


def cpu_baseline(args, desc):
    """The oracle (oracle/ipt_oracle.cpp, the recursive CPU restatement of the
    reference estimator with glibc libm) timed on this host's cores over a
    bounded sample of the same workload: strided source pixels of successive
    passes, at least args.cpu_seconds of wall time (c1: the whole frame)."""
    sys.path.insert(0, str(ROOT / "tests"))
    import ctypes as C

    import oracle_binding
    from ipt_amd import capi

    lib = oracle_binding.load()
    lib.ipt_oracle_render_rows_values.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                                  C.c_int, C.c_void_p]
    s, keep = capi.make_scene(desc)
    W, H = args.width, args.height
    threads = cpu_threads(args.cpu_threads)
    total = 0
    calls = 0
    t0 = time.perf_counter()
    if args.cpu_sample is None:  # c1: the whole C1 frame, all its passes
        p = capi.make_params(W, H, args.spp_per_step * args.steps, n_rays=args.n_rays, depth_max=args.depth_max,
                             seed=args.seed)
        vals = np.zeros(p.spp * W * H, np.float32)
        rc = lib.ipt_oracle_render_rows_values(C.addressof(s), C.addressof(p), 1, 0, 1, 0, threads, vals.ctypes.data)
        assert rc == 0
        total = p.spp * W * H
        el = time.perf_counter() - t0
        sample = (f"the whole C1 workload: {W}x{H} x {p.spp} spp = {total} paths in {el:.1f} s")
    else:
        rs, cs = args.cpu_sample
        nr, nc = (H + rs - 1) // rs, (W + cs - 1) // cs
        vals = np.zeros(nr * nc, np.float32)
        # the same sample on ONE thread for a bounded time first: the per-core
        # rate the multi-thread figure is scaled against (the job's 16-CPU
        # share is the most this box allows: a full-host run is not measured,
        # it is extrapolated from the per-core rate below)
        one_total, one_calls, t1 = 0, 0, time.perf_counter()
        while time.perf_counter() - t1 < min(8.0, args.cpu_seconds / 3):
            p = capi.make_params(W, H, 1, spp_offset=10_000 + one_calls, n_rays=args.n_rays,
                                 depth_max=args.depth_max, seed=args.seed)
            rp, cp = (37 * one_calls) % rs, (11 * one_calls) % cs
            rc = lib.ipt_oracle_render_rows_values(C.addressof(s), C.addressof(p), rs, rp, cs, cp, 1,
                                                   vals.ctypes.data)
            assert rc == 0
            one_total += len(range(rp, H, rs)) * len(range(cp, W, cs))
            one_calls += 1
        one_rate = one_total / (time.perf_counter() - t1)
        t0 = time.perf_counter()
        while True:
            # call k: rows (37k mod rs) (mod rs), columns (11k mod cs) (mod cs)
            # of pass k: co-prime strides walk every row and column phase
            p = capi.make_params(W, H, 1, spp_offset=calls, n_rays=args.n_rays, depth_max=args.depth_max,
                                 seed=args.seed)
            rp, cp = (37 * calls) % rs, (11 * calls) % cs
            rc = lib.ipt_oracle_render_rows_values(C.addressof(s), C.addressof(p), rs, rp, cs, cp, threads,
                                                   vals.ctypes.data)
            assert rc == 0
            total += len(range(rp, H, rs)) * len(range(cp, W, cs))
            calls += 1
            el = time.perf_counter() - t0
            if el >= args.cpu_seconds:
                break
        sample = (f"{calls} calls, each the source pixels at row stride {rs} and column stride {cs} of one "
                  f"pass (phases 37k mod {rs}, 11k mod {cs}) of the {W}x{H} frame: {total} paths in {el:.1f} s")
    phys = physical_cores()
    out = {
        "value": total / el / 1e6,
        "unit": "Mpaths/s",
        "cores": threads,
        "kind": "port",
        "sample": sample + (f"; {threads} threads (this process's CPU share); oracle/ipt_oracle.cpp, the "
                            f"recursive CPU restatement of main.cpp:98-184 with glibc libm (the reference's "
                            f"estimator TUs need boost and cannot be built here, DESIGN.md §2)"),
        "cpu_model": cpu_model(),
        "host_cpus": os.cpu_count(),
        "paths_per_s_per_core": total / el / threads,
        "host_physical_cores": phys,
        "threads_policy": ("the job's CPU share (OMP_NUM_THREADS, 16 per GPU on the GPU box): the pool allows no "
                           "more threads per job; a full-host figure is extrapolated, not measured"),
    }
    if args.cpu_sample is not None:
        out["single_thread_paths_per_s"] = one_rate
        out["thread_scaling"] = (total / el) / one_rate if one_rate > 0 else None
        if phys:
            out["full_host_extrapolated_Mpaths_s"] = one_rate * phys / 1e6
            out["full_host_note"] = (f"single-thread rate x {phys} physical cores (linear scaling assumed; "
                                     f"measured scaling at {threads} threads: "
                                     f"{(total / el) / one_rate / threads:.2f} of linear)")
    return out


def main():
    args = parse()
    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: WORLD_SIZE={world} but --gpus={args.gpus}", file=sys.stderr)
    dist = None
    # IPT_BENCH_SHARE_GPU=1 (rehearsal only): every rank on cuda:0, frame-end
    # collectives over gloo on host copies, so the N>1 path runs on a 1-GPU box
    share = os.environ.get("IPT_BENCH_SHARE_GPU") == "1"
    if share:
        local_rank = 0
    # IPT_BENCH_FORCE_DIST=1 (test only): the process group, frame-end gather
    # and collectives of the N>1 path also at world 1, so the RCCL branch runs
    # on a one-GPU box (tests/test_gpu_rccl_branch.py)
    if world > 1 or os.environ.get("IPT_BENCH_FORCE_DIST") == "1":
        import torch.distributed as dist

        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    from ipt_amd import capi, roofline, tiles

    desc = make_desc(args.scene)
    ctx = capi.Context(local_rank)
    ctx.upload_scene(desc)

    W, H = args.width, args.height
    npix = W * H
    weak = args.scaling == "weak"
    spp_step = args.spp_per_step * (world if weak else 1)  # passes of the frame per step
    # GridRenderPlane state [field][H][W]: pixels, counters, sums, pixel_max
    state = torch.zeros(4, H, W, dtype=torch.float32, device=dev)
    pixels, counters, sums, pmax = state[0], state[1].view(torch.int32), state[2], state[3]
    stream = torch.cuda.current_stream(dev).cuda_stream

    def params(spp, off, shard=rank, flags=0, n_shards=world):
        return capi.make_params(W, H, spp, spp_offset=off, n_rays=args.n_rays, depth_max=args.depth_max,
                                seed=args.seed, tile_rows=args.tile_rows if n_shards > 1 else 0,
                                n_shards=n_shards, shard_id=shard, flags=flags)

    def render(p, st=state):
        ctx.render_device(p, st[0].data_ptr(), st[1].data_ptr(), st[2].data_ptr(), st[3].data_ptr(), stream)

    # the steps are queued (ipt_render_device_async: a step's path kernel takes
    # the CUs the previous step's tail leaves idle; the GridRenderPlane replays
    # stay in step order on `stream`) and waited for once
    # (under rocprofv3 counter collection dispatches are serialised and a
    # gated launch would never start: synchronous steps there)
    profiled = any(k.startswith(("ROCPROF", "ROCPROFILER")) for k in os.environ)
    use_async = ctx.has_async and not args.sync and not profiled

    def render_step(p):
        if use_async:
            ctx.render_device_async(p, state[0].data_ptr(), state[1].data_ptr(), state[2].data_ptr(),
                                    state[3].data_ptr(), stream)
        else:
            render(p)

    # the tile plan of every rank (host-only, deterministic): owned rows
    owned_rows = tiles.owned_rows(W, H, args.tile_rows, world)
    max_own = max(len(o) for o in owned_rows)

    def host_coll(fn, t, **kw):
        """A collective on a small host tensor (through the device under RCCL)."""
        if share:
            fn(t, **kw)
            return t
        d = t.to(dev)
        fn(d, **kw)
        return d.cpu()

    # warmup (separate passes, then reset the image)
    for i in range(args.warmup):
        render_step(params(spp_step, 1_000_000 + i * spp_step))
    if use_async:
        ctx.wait()
    state.zero_()
    torch.cuda.synchronize(dev)

    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    path_ms = acc_ms = 0.0
    for step in range(args.steps):
        render_step(params(spp_step, step * spp_step))
        if not use_async:
            pm, am = ctx.last_kernel_ms()
            path_ms += pm
            acc_ms += am
    if use_async:
        ctx.wait()
        path_ms, acc_ms = ctx.last_kernel_ms()  # all the steps' launches (overlaps counted once)
    if dist:
        tiles.assemble(dist, state, owned_rows, rank, host=share)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    my_path_ms = path_ms
    if dist:
        tt = torch.tensor([elapsed, path_ms, acc_ms], dtype=torch.float64)
        elapsed, path_ms, acc_ms = host_coll(dist.all_reduce, tt, op=dist.ReduceOp.MAX).tolist()

    spp_total = args.steps * spp_step
    total_paths = W * H * spp_total
    value = total_paths / elapsed / 1e6

    verify = None
    if args.verify and dist and rank == 0:
        whole = torch.zeros_like(state)
        for step in range(args.steps):
            render(params(spp_step, step * spp_step, shard=0, n_shards=1), whole)
        torch.cuda.synchronize(dev)
        verify = bool(torch.equal(whole.view(torch.int32), state.view(torch.int32)))
        del whole
    mean_pixel = float(pixels.mean().item())

    # algorithmic op count of the timed work: re-render the same passes with
    # the kernel's event counters (untimed; counts are deterministic)
    roof = None
    cnt = None
    ranks = None
    if not args.no_counters:
        sv = state.clone()
        ctx.reset_counters()
        acc_alone_ms = 0.0
        for step in range(args.steps):
            render(params(spp_step, step * spp_step, flags=capi.IPT_FLAG_COUNTERS))
            acc_alone_ms += ctx.last_kernel_ms()[1]  # (a synchronous call: its accumulate ran alone)
        torch.cuda.synchronize(dev)
        cnt = ctx.counters()
        state.copy_(sv)
        del sv
        my_ops = roofline.ops_from_counters(cnt, n_spheres=len(desc.get("spheres", [])),
                                            n_lights=len(desc.get("lights", [])))
        mine = [my_path_ms, cnt["paths"], cnt["traced_rays"], my_ops]
        if dist:
            # per-rank [path ms, paths, traced rays, op-eq] as a [world, 4]
            # all-reduce of one-hot rows (no list collectives needed)
            allr = torch.zeros(world, 4, dtype=torch.float64)
            allr[rank] = torch.tensor(mine, dtype=torch.float64)
            allr = host_coll(dist.all_reduce, allr)
            ranks = [{"rank": r, "path_ms": allr[r, 0].item(), "paths": int(allr[r, 1].item()),
                      "traced_rays": int(allr[r, 2].item()), "ops": allr[r, 3].item()} for r in range(world)]
            ct = torch.tensor([cnt[k] for k in capi.COUNTER_NAMES], dtype=torch.int64)
            ct = host_coll(dist.all_reduce, ct)
            cnt = dict(zip(capi.COUNTER_NAMES, [int(x) for x in ct.tolist()]))
        ops = roofline.ops_from_counters(cnt, n_spheres=len(desc.get("spheres", [])),
                                         n_lights=len(desc.get("lights", [])))
        # per launch on one rank: ops/world per launch, the slowest rank's
        # average launch duration (raygen + path kernel, HIP events)
        launch_s = path_ms / 1e3 / args.steps
        achieved = ops / world / args.steps / launch_s
        acc_bytes = roofline.accumulate_bytes(len(owned_rows[rank]) * W, spp_step)
        acc_alone_s = acc_alone_ms / 1e3 / args.steps
        # the accumulate kernel's duration per launch: in the timed (queued)
        # steps the first step's accumulate shares the CUs with the next step's
        # path kernel; the synchronous counting re-render above times it alone
        acc_launch_s = acc_ms / 1e3 / args.steps
        cos_samples = cnt["iterations"] - cnt["light_samples"]
        paths_launch = total_paths // world // args.steps
        path_alg_bytes = roofline.path_bytes(paths_launch, cos_samples // world // args.steps,
                                             cnt["sphere_frames"] // world // args.steps)
        traffic = traffic_fabric = traffic_src = occ = dram = traffic_dram_upper = None
        for name in (f"pmc_latest_{args.config}.json",) + (("pmc_latest.json",) if args.config == "c2" else ()):
            pmc_file = ROOT / "profiles" / name
            if not pmc_file.exists():
                continue
            try:
                pm = json.load(open(pmc_file))
                c0 = pm.get("config", {})
                if (c0.get("width") == W and c0.get("height") == H and c0.get("spp_per_step") == spp_step
                        and c0.get("depth_max", args.depth_max) == args.depth_max):
                    # traffic: the measured L2 memory-side bytes (FETCH_SIZE + WRITE_SIZE,
                    # MI355X_MICROARCH.md "HBM"); it counts Infinity-Cache hits too, so it
                    # bounds the HBM bytes from above, as does the DRAM-destined request
                    # estimate beside it (traffic_dram_upper)
                    traffic_fabric = pm.get("path_kernel_hbm_bytes_per_launch")
                    dram = pm.get("path_kernel_dram")
                    traffic = traffic_fabric
                    traffic_dram_upper = pm.get("path_kernel_dram_bytes_per_launch")
                    occ = pm.get("path_kernel_occupancy")
                    cfg_tag = f"_{pm['config_name']}" if pm.get("config_name") else ""
                    traffic_src = (f"profiles/{pm['tag']}{cfg_tag}_summary.json (rocprofv3 --pmc passes of the same "
                                   f"config at N=1: FETCH_SIZE, WRITE_SIZE, TCC_EA0_RDREQ(_DRAM), "
                                   f"TCC_EA0_WRREQ(_DRAM); SQ_WAVE_CYCLES, GRBM_GUI_ACTIVE)")
                    break
            except Exception:
                traffic = occ = None
        hbm_ach = path_alg_bytes / launch_s / 1e9
        comp_bytes = roofline.compulsory_bytes(paths_launch)
        roof = {
            # BASELINE.json's metric asks for achieved HBM GB/s: the top level is
            # the path kernel's HBM roofline; the resource that actually binds
            # it is VALU issue / latency ("valu" below)
            "bound": "hbm",
            "achieved": hbm_ach,
            "peak": roofline.HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": hbm_ach / roofline.HBM_PEAK_GBPS,
            "traffic": traffic,
            "traffic_unit": "bytes/launch",
            "traffic_kind": ("fabric: L2 memory-side bytes (FETCH_SIZE + WRITE_SIZE); Infinity-Cache hits "
                             "included, so an upper bound on HBM bytes") if traffic else None,
            "traffic_fabric": traffic_fabric,
            "traffic_dram_upper": traffic_dram_upper,
            "traffic_dram_detail": dram,
            "traffic_source": traffic_src,
            "measured_GBps": (traffic / launch_s / 1e9) if traffic else None,
            "measured_fabric_GBps": (traffic_fabric / launch_s / 1e9) if traffic_fabric else None,
            "kernel": "raygen_kernel + path_kernel",
            "bytes_per_path": path_alg_bytes / paths_launch,
            "compulsory": {
                "bytes_per_path": roofline.COMPULSORY_BYTES_PER_PATH,
                "achieved": comp_bytes / launch_s / 1e9,
                "frac": comp_bytes / launch_s / 1e9 / roofline.HBM_PEAK_GBPS,
                "note": ("the reference's own traffic: the 4 B radiance + 1 B drift code per path that the "
                         "GridRenderPlane replay reads back; the top level adds the raygen records and the "
                         "CosineDdf / frame-table gathers (implementation choices that replace VALU work)"),
            },
            "launch_ms": launch_s * 1e3,
            "occupancy": occ,
            "binding": "valu",
            "valu": {
                "achieved": achieved / 1e12,
                "peak": roofline.VALU_PEAK_LANE_OPS / 1e12,
                "unit": "Tlane-op/s",
                "frac": achieved / roofline.VALU_PEAK_LANE_OPS,
                "ops_per_path": ops / cnt["paths"],
            },
            "bvh_nodes_per_trace": (cnt["bvh_nodes"] / max(cnt["traced_rays"], 1)) if desc.get("spheres") else None,
            "sphere_tests_per_trace": (cnt["sphere_tests"] / max(cnt["traced_rays"], 1)) if desc.get("spheres") else None,
            "light_tests_per_trace": cnt["light_tests"] / max(cnt["traced_rays"], 1),
            # the reference's full sphere/light scans, only where a BVH replaced them
            "reference_scan_ops_per_path": (roofline.reference_scan_ops(cnt, len(desc.get("spheres", [])))
                                            / cnt["paths"]
                                            if cnt["bvh_nodes"] or cnt["light_nodes"]
                                            or roofline.light_lattice(cnt, len(desc.get("lights", [])))
                                            else None),
            "note": ("hbm: bytes of one launch of the per-sample work (raygen_kernel + path_kernel: 5 B "
                     "radiance + drift code per path, the 32 B raygen record written and read back, 4 B "
                     "CosineDdf r gather per cosine-sampled iteration, 8 B frame-table gather per sphere "
                     "frame) / its HIP-event duration (raygen is ~0.2 %); traffic = rocprofv3 "
                     "FETCH_SIZE+WRITE_SIZE of path_kernel per launch of the same config (random 4-8 byte "
                     "gathers move 64-byte lines); occupancy = mean resident waves per SIMD from "
                     "SQ_WAVE_CYCLES (quad-cycles) x 4 / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs). The kernel "
                     "is bound by instruction issue (VALU work and the exec-mask bookkeeping of its "
                     "branches; the gather latency is hidden), DESIGN.md sections 4.3 and 6. valu: "
                     "algorithmic op-eq (SURVEY.md §8d cost table x the kernel's event counters) / launch "
                     "time against the VALU issue peak 256CU x 4 SIMD32 x 32 lanes x 2.4GHz -- the binding "
                     "resource (no MFMA shape; HBM far from peak)"),
            "hbm_accumulate": {
                "kernel": "accumulate_kernel",
                "bound": "hbm",
                "achieved": acc_bytes / acc_alone_s / 1e9 if acc_alone_s > 0 else None,
                "peak": roofline.HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": (acc_bytes / acc_alone_s / 1e9 / roofline.HBM_PEAK_GBPS
                         if acc_alone_s > 0 else None),
                "launch_ms": acc_alone_s * 1e3,
                "launch_ms_in_queued_steps": acc_launch_s * 1e3,
                "timing": ("the kernel's own first-start / last-end wall-clock stamps; launch_ms from the "
                           "synchronous counting re-render (the kernel alone, as rocprofv3's kernel trace runs "
                           "it), launch_ms_in_queued_steps from the timed steps, where the first step's "
                           "accumulate shares the CUs with the next step's path kernel"),
            },
        }

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        try:
            cpu = cpu_baseline(args, desc)
        except Exception as e:  # the GPU number stands on its own
            cpu = {"error": repr(e)}

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "Mpaths/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (sample_scenes[0] geometry/light/camera, Philox per-path RNG)",
            "config": {"workload": f"{args.config}: {args.scene} {W}x{H}, {spp_total} spp, "
                                   f"depth_max {args.depth_max}, n_rays {args.n_rays}",
                       "baseline_config": args.config,
                       "width": W, "height": H, "spp": spp_total,
                       "spp_per_step": spp_step, "depth_max": args.depth_max,
                       "n_rays": args.n_rays, "tile_rows": args.tile_rows if world > 1 else 0,
                       "calls": ("queued (ipt_render_device_async), one wait" if use_async
                                 else "synchronous ipt_render_device per step"),
                       "parallelism": f"tiles{world}",
                       "per_rank": ("the whole frame's tiles dealt round-robin; " +
                                    (f"{args.spp_per_step} x N passes per step (weak)" if weak
                                     else "the fixed frame split over the ranks (strong)"))},
            "roofline": roof,
            "cpu_baseline": cpu,
            "gpu_vs_cpu": (value / cpu["value"]) if cpu and "value" in cpu else None,
            # geometry traces per second beside the paths
            "mrays_per_s": (value * cnt["traced_rays"] / cnt["paths"]) if cnt else None,
            "events_per_path": ({k: cnt[k] / cnt["paths"] for k in cnt if k != "paths"}
                                if cnt else None),
            "mean_pixel": mean_pixel,
        }
        if dist:
            out["ranks"] = ranks
            if ranks:
                pm = [r["path_ms"] for r in ranks]
                out["rank_imbalance"] = max(pm) / (sum(pm) / len(pm))
                # the work each rank did (algorithmic op-eq from its event
                # counters), independent of timing: max / mean over ranks
                wk = [r["ops"] for r in ranks]
                out["work_imbalance"] = max(wk) / (sum(wk) / len(wk))
            out["frame_end"] = (f"one gather of the owned rows to rank 0: {tiles.payload_bytes(W, owned_rows)} B "
                                f"({16 * W * max_own} B per rank, 16 B per owned pixel)")
            if verify is not None:
                out["verify_whole_frame_bit_exact"] = verify
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
