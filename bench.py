#!/usr/bin/env python3
"""Benchmark of the MI355X-native ORB-SLAM3 matching (+ BA) hot path.

    python bench.py --gpus N --steps K --warmup W

Headline (BASELINE.json metric "Mmatches/s (256-bit Hamming) + LocalBA iters/s"), workload
configs[1]: brute-force 256-bit Hamming top-2 of 2000 x 2000 descriptors (C2).  One step = one
launch of 1024 independent 2000 x 2000 problems (frames) through the C-ABI entry
osg_hamming_top2_batch_dev (k_top2_fp4, FP4 block-scaled matrix cores; OSG_TOP2_FP4=0 selects the I8 form
k_top2_mfma) with inputs resident in HBM; the one-problem launch
(osg_hamming_top2_dev) is reported beside it as single_launch.  For N > 1 every rank matches its own
independent frames (weak scaling; no collective in the data path); value = pairs of all ranks /
max-over-ranks time.

Also reported (same run):
  * the dominant kernel's roofline (HIP events on its stream) and the C2' streaming kernel's HBM roofline
    (Q = 4 x M = 2^24);
  * the CPU restatement timed on this host (cpu_baseline);
  * the frame-batched workloads: C3, C5, DBoW2 and ComputeStereoMatches, each valued at the C++ adapter's wall
    rate (tools/adapter_wall_bench.cpp: mock ORB-SLAM3 objects -> C-ABI -> write-back, as many host threads as
    the CPU baseline) with the batched launches' device-time rate beside it, and the ORB extractor stages;
  * LocalBA iterations/s on C4 (64-window batches, --lba-threads host threads);
  * global BA on 150 KeyFrames and on the 1500-KeyFrame map.
--only STAGE[,STAGE] runs a subset of those stages (A/B runs).
stdout carries one compact JSON line (<= 8 KB, compact_line); the full record goes to --detail.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tools.adapter_arrays import (bow_arrays, frame_arrays, last_arrays, mps_arrays, pose_arrays,  # noqa: E402
                                  pose_for_mock, prefixed, slot_arrays, stereo_arrays, vocabulary_arrays)

PEAK_HBM_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
# Non-packed 32-bit VALU: 256 CU x 4 SIMD x 16 lanes per cycle x 2.4 GHz = 39.3 T lane-op/s.  Measured
# on the box (tools/micro/valu_rate.hip, profiles/r02_valu_rate.txt): v_xor_b32, v_bcnt_u32_b32,
# v_med3_u32, v_add_u32 and v_add_f32 all sustain 38.0-38.5 T lane-op/s = one wave64 instruction per
# 4 cycles per SIMD at full occupancy; the 157.3 TF FP32 "vector" figure needs packed v_pk_fma_f32
# (2 FMAs per lane-instruction), which has no integer counterpart.
PEAK_VALU_TOPS = 256 * 4 * 16 * 2.4e9 / 1e12
PEAK_VALU_GUIDE_TOPS = 2 * PEAK_VALU_TOPS   # the guide's 32 lanes / clk (MI355X_MICROARCH.md)
VALU_OPS_PER_PAIR = 19         # 8 v_xor + 8 v_bcnt(acc) + 1 v_lshl_or + v_med3 + v_min
# I8 matrix cores: v_mfma_i32_32x32x32_i8 = 32 x 32 x 32 MACs per 32 cycles per SIMD (the cycles of the BF16
# 32x32x16 form at twice the K, MI355X_MICROARCH.md "Matrix cores"): 256 CU x 4 SIMD x 1024 MAC x 2 ops x 2.4 GHz
PEAK_I8_TOPS = 256 * 4 * 1024 * 2 * 2.4e9 / 1e12
# FP4 (e2m1) block-scaled v_mfma_scale_f32_32x32x64_f8f6f4: the BF16 form's cycles at 4x K, twice the I8 rate
PEAK_FP4_TOPS = 2 * PEAK_I8_TOPS
I8_OPS_PER_PAIR = 512          # 256 MACs per (query, train row) pair
# the FP4 top-2 epilogue per key, as compiled (r06): per two keys one v_med3_f32 and one v_min3_i32, the k2
# chain merged into one v_min3_i32 per two pairs, plus 2 rebasing subtractions per tile: 22 VALU ops per
# 32-row tile per wave (30 before r06's key_push2f, csrc/hamming_mfma.hip)
MFMA_EPILOGUE_VALU_PER_PAIR = 22 / 16
MFMA_MAX_ROWS = 8192           # the I8 kernel's 13-bit row field (osg_top2_mfma_max_rows)
LINE_MAX_BYTES = 8192          # the stdout line's budget (the driver did not parse r04's 21 KB line)


def job_totals(elapsed, units, world, dist=None, device="cpu"):
    """Whole-job figures from per-rank (elapsed seconds, units processed): the slowest rank's time
    (max over ranks) and the units of all ranks (sum).  Weak scaling: every rank processes its own
    independent frames / windows; the only collectives are these two reductions and barriers."""
    if world == 1 or dist is None:
        return float(elapsed), float(units)
    import torch
    mx = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    sm = torch.tensor([float(units)], dtype=torch.float64, device=device)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    return float(mx.item()), float(sm.item())


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--ramp-s", type=float, default=0.5,
                    help="untimed launches of the headline step for this long before the warmup (GPU clock ramp)")
    ap.add_argument("--nq", type=int, default=2000)
    ap.add_argument("--nt", type=int, default=2000)
    ap.add_argument("--c2-batch", type=int, default=1024,
                    help="C2 frames per launch of the headline step (1: the single-problem launch)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-stream", action="store_true")
    ap.add_argument("--no-ba", action="store_true")
    ap.add_argument("--no-gba", action="store_true", help="skip the global BA workloads")
    ap.add_argument("--no-gba-map", action="store_true", help="skip the map-scale (1500 KF) global BA")
    ap.add_argument("--ba-reps", type=int, default=20)
    ap.add_argument("--ba-batch", type=int, default=64, help="C4 windows per GPU per lockstep batch")
    ap.add_argument("--ba-batch-reps", type=int, default=6)
    ap.add_argument("--ba-threads", type=int, default=8,
                    help="host threads per GPU for the one-frame-per-call ORB stages' wall rate, each with its own "
                         "context and HIP stream (8: ComputeKeyPointsOctTree 22.8 k frames/s against 12.2-12.6 k at "
                         "4 and 15.9 k at 16, gpurun_out/orbthr)")
    ap.add_argument("--lba-threads", type=int, default=8,
                    help="host threads per GPU driving LocalBA batches, each with its own context and HIP stream "
                         "(8 measured 9-18 %% above 4: more batches in flight cover each thread's host phases)")
    ap.add_argument("--gba-batch", type=int, default=16, help="150-KF maps per GPU per lockstep global-BA batch")
    ap.add_argument("--gba-threads", type=int, default=8, help="host threads per GPU driving global-BA batches")
    ap.add_argument("--gba-batch-reps", type=int, default=3)
    ap.add_argument("--no-frames", action="store_true", help="skip the frame-batched C3 / C5 workloads")
    ap.add_argument("--frames", type=int, default=1024, help="frames per launch (C3 / C5 batches)")
    ap.add_argument("--frame-reps", type=int, default=5)
    ap.add_argument("--no-wall", action="store_true", help="skip the C++ adapter wall-rate runs")
    ap.add_argument("--only", default="", help="comma-separated stage keys to run (A/B runs); default: all")
    ap.add_argument("--wall-frames", type=int, default=256, help="frames per batched adapter call (C++ wall bench)")
    ap.add_argument("--wall-reps", type=int, default=24, help="timed repetitions per host thread (C++ wall bench)")
    ap.add_argument("--wall-threads", type=int, default=0,
                    help="host threads of the C++ wall bench, each with its own context (Tracking threads); 0: "
                         "as many as the CPU baseline runs (the host CPUs this job may use, per rank)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="per-launch HBM traffic from the rocprofv3 PMC passes (tools/gpu/gpu_profile_r03.sh)")
    ap.add_argument("--valu-pmc", default=os.path.join(ROOT, "profiles", "r03_top2_valu_pmc.json"),
                    help="the headline kernel's VALU counters (tools/pmc_valu.py)")
    ap.add_argument("--schur-pmc", default=os.path.join(ROOT, "profiles", "r06_lba_pmc.json"),
                    help="the LBA engine's SQ / MFMA / HBM counters (tools/pmc_kernel_summary.py)")
    ap.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="file for the full per-stage record (stdout carries the compact line); '' for none")
    return ap.parse_args()


def _spawn_ranks(n):
    """`bench.py --gpus N` outside a launcher: start the N ranks (one process per GPU, torchrun on
    127.0.0.1) as a child before this process touches a GPU, and return its exit code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    t_start = time.perf_counter()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(_spawn_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}; launch one rank per GPU "
              f"(torchrun --nproc-per-node {args.gpus}) or drop the launcher", file=sys.stderr)
        sys.exit(2)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    from orb_slam3_comments_ghr_amd import Context, synth

    if rank == 0 and world == 1 and not args.no_cpu:
        _start_timing_build()  # the cpu_baseline legs' oracle, compiled for this host while the GPU runs
    ctx = Context(local_rank)
    # a dedicated (non-null) stream: the kernels and the HIP events below share it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)

    def barrier():
        if world > 1:
            dist.barrier()

    # ---- C2: 2000 x 2000 brute-force top-2 on resident inputs -------------------------------
    # Headline step: B independent 2000 x 2000 frames in one launch (osg_hamming_top2_batch_dev,
    # frame-batched throughput); the single-problem launch (osg_hamming_top2_dev, the latency form)
    # is measured beside it.  Frame 0 of the batch is the seeded C2 frame.
    nq, nt, B = args.nq, args.nt, max(1, args.c2_batch)
    q_np, t_np = synth.descriptors_c2(nq, nt, seed=synth.SEED_C2 + rank)
    frames = [(q_np, t_np)] + [synth.descriptors_c2(nq, nt, seed=synth.SEED_C2 + 7919 * (b + 1) + rank)
                               for b in range(1, B)]
    dq = torch.from_numpy(q_np).to(dev)
    dt = torch.from_numpy(t_np).to(dev)
    dout = torch.empty((nq, 3), dtype=torch.int32, device=dev)
    dqb = torch.from_numpy(np.concatenate([f[0] for f in frames])).to(dev)
    dtb = torch.from_numpy(np.concatenate([f[1] for f in frames])).to(dev)
    doutb = torch.empty((B * nq, 3), dtype=torch.int32, device=dev)

    def step_single():
        ctx.hamming_top2_dev(dq, nq, dt, nt, dout)

    def step():
        ctx.hamming_top2_batch_dev(dqb, nq, dtb, nt, B, doutb)

    # Clock ramp (untimed, before the W warmup steps): launches of the same step for --ramp-s seconds.
    # A box that has been idle runs the first ~25 launches at a lower clock: with 20 timed steps after 5
    # warmup steps the kernel read 561.7 us per launch, with 200 after 20 on the same box 482.3 us
    # (gpurun_out/r05g).  The count is reported in config.
    ramp_n, t_r = 0, time.perf_counter()
    while time.perf_counter() - t_r < args.ramp_s:
        for _ in range(8):
            step()
        torch.cuda.synchronize(dev)
        ramp_n += 8
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    # HIP events on the launch stream inside the timed region: the kernels' own time over the same K
    # steps, so the roofline's kernel_us cannot exceed ms_per_step
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    k_us_loop = ev0.elapsed_time(ev1) * 1e3 / args.steps
    pairs_per_step = B * nq * nt
    elapsed, total_pairs = job_totals(elapsed, pairs_per_step * args.steps, world, dist if world > 1 else None, dev)
    value = total_pairs / elapsed / 1e6
    # frame 0 of the batch equals the single-problem launch (both are the serial loop's result)
    step_single()
    torch.cuda.synchronize(dev)
    batch_frame0_equal = bool(torch.equal(doutb[:nq], dout))

    # ---- dominant kernel roofline: HIP events on the launch stream -------------------------
    # The kernel's average duration = (end - start) / n over n back-to-back launches between two
    # events on its stream.  A stream pre-filled with a spin kernel keeps host launch gaps out.
    # (Per-launch brackets carry a fixed ~5 us event cost on this stack even around nothing, and
    # read high against rocprofv3; the back-to-back average agrees with it.)
    def kernel_us(fn, n_ev):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(2e6 + n_ev * 2e4))
        e0.record(stream)
        for _ in range(n_ev):
            fn()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) * 1e3 / n_ev

    k_us_spin = kernel_us(step, max(20, min(args.steps, 100)))
    k1_us = kernel_us(step_single, max(50, min(args.steps, 500)))
    k_us = k_us_loop
    alg_bytes = B * ((nq + nt) * 32 + nq * 12)
    # the kernel the batched entry launches, named by the library itself
    kname = ctx.hamming_top2_batch_plan(nq, nt, B)
    mfma = kname.startswith(("k_top2_mfma", "k_top2_fp4"))
    fp4 = kname.startswith("k_top2_fp4")
    if mfma:
        ksub = kname.split("<")[0]
        achieved = pairs_per_step * I8_OPS_PER_PAIR / (k_us * 1e-6) / 1e12
        epi = pairs_per_step * MFMA_EPILOGUE_VALU_PER_PAIR / (k_us * 1e-6) / 1e12
        peak = PEAK_FP4_TOPS if fp4 else PEAK_I8_TOPS
        roofline = {
            "kernel": kname, "bound": "mfma", "achieved": round(achieved, 1), "peak": round(peak, 1),
            "unit": "TOPS (fp4 e2m1 block-scaled MFMA, 2 ops per MAC)" if fp4 else "TOPS (i8 MFMA, 2 ops per MAC)",
            "peak_source": ("v_mfma_scale_f32_32x32x64_f8f6f4 with fp4 operands: 32x32x64 MACs / 32 cycles / SIMD "
                            "(MI355X_MICROARCH.md Matrix cores: FP4 = the BF16 form's cycles at 4x K) x 1024 SIMDs x "
                            "2.4 GHz" if fp4 else
                            "v_mfma_i32_32x32x32_i8: 32x32x32 MACs / 32 cycles / SIMD (MI355X_MICROARCH.md Matrix "
                            "cores: I8 = the BF16 form's cycles at 2x K) x 1024 SIMDs x 2.4 GHz"),
            "frac": round(achieved / peak, 4),
            "frac_of_i8_peak": round(achieved / PEAK_I8_TOPS, 4),
            "algorithmic_ops_per_launch": pairs_per_step * I8_OPS_PER_PAIR,
            # the VALU side of the same kernel: the 2-op top-2 epilogue per pair against the measured 16-lane
            # ceiling and the guide's 32-lane figure
            "valu_epilogue": {"ops_per_pair": MFMA_EPILOGUE_VALU_PER_PAIR, "achieved": round(epi, 2),
                              "frac_16_lanes": round(epi / PEAK_VALU_TOPS, 4),
                              "frac_guide_32_lanes": round(epi / PEAK_VALU_GUIDE_TOPS, 4),
                              "unit": "T lane-ops/s"},
            # the popcount form's accounting, for comparison with r01-r03 (19 lane-ops per pair)
            "popcount_equivalent_frac_guide_valu": round(
                pairs_per_step * VALU_OPS_PER_PAIR / (k_us * 1e-6) / 1e12 / PEAK_VALU_GUIDE_TOPS, 4),
        }
    else:
        ql = int(os.environ.get("OSG_TOP2_BATCH_QL", "2"))
        kname = (f"k_top2_batch<{ql},{int(os.environ.get('OSG_TOP2_BATCH_SCALAR', '1'))}> "
                 f"grid={(nq + 64 * ql - 1) // (64 * ql)} x {B} x 1024")
        fp4 = False
        ksub = "k_top2_batch"
        achieved = pairs_per_step * VALU_OPS_PER_PAIR / (k_us * 1e-6) / 1e12
        vp = _load_json(args.valu_pmc)
        vk = next((v for k, v in vp.items() if "k_top2_batch" in k), None)
        roofline = {
            "kernel": kname, "bound": "valu", "achieved": round(achieved, 3),
            "peak": round(PEAK_VALU_GUIDE_TOPS, 1), "unit": "Tops/s (int32 VALU lane-ops)",
            "peak_source": "the guide's 32 lanes/clk (MI355X_MICROARCH.md) x 1024 SIMDs x 2.4 GHz",
            "frac": round(achieved / PEAK_VALU_GUIDE_TOPS, 4),
            "algorithmic_ops_per_launch": pairs_per_step * VALU_OPS_PER_PAIR,
            # the measured ceiling of this instruction mix: one wave64 instruction per 4 cycles per SIMD
            # (tools/micro/valu_rate.hip, profiles/r02_valu_rate.txt)
            "peak_measured_16_lanes": round(PEAK_VALU_TOPS, 1),
            "frac_measured_16_lanes": round(achieved / PEAK_VALU_TOPS, 4),
            "valu_issue_util_pmc": None if vk is None else round(vk["valu_issue_util_16"], 4),
            "cycles_per_valu_inst_pmc": None if vk is None else round(vk["cycles_per_valu_inst"], 3),
            "valu_pmc_source": None if vk is None else os.path.relpath(args.valu_pmc, ROOT),
        }
    tr = pmc_traffic_instance(args.traffic, kname) if ksub != "k_top2_batch" else pmc_traffic(args.traffic, ksub)
    roofline.update({
        "traffic": None if tr is None else round(tr[0]),
        "traffic_source": None if tr is None else f"{os.path.relpath(args.traffic, ROOT)}: {tr[1]}",
        # kernel time = HIP events around the K timed steps on the launch stream (inside the wall-clock
        # region, so <= ms_per_step); the back-to-back launches behind a spin kernel are reported beside it
        "kernel_us": round(k_us, 3),
        "kernel_us_backtoback_after_spin": round(k_us_spin, 3),
        "kernel_us_le_ms_per_step": bool(k_us <= elapsed / args.steps * 1e6 + 1e-6),
        "algorithmic_bytes_per_launch": alg_bytes,
        "hbm_frac_if_priced_as_hbm": round(alg_bytes / (k_us * 1e-6) / 1e9 / PEAK_HBM_GBS, 5),
    })
    plan = ctx.hamming_top2_plan(nq, nt)
    tr1 = pmc_traffic(args.traffic, plan.split(" ")[0].split("<")[0])
    single = {
        "kernel": plan, "kernel_us": round(k1_us, 3),
        "Mmatches_per_s_kernel": round(nq * nt / (k1_us * 1e-6) / 1e6, 1),
        "frac": round(nq * nt * VALU_OPS_PER_PAIR / (k1_us * 1e-6) / 1e12 / PEAK_VALU_GUIDE_TOPS, 4),
        "frac_measured_16_lanes": round(nq * nt * VALU_OPS_PER_PAIR / (k1_us * 1e-6) / 1e12 / PEAK_VALU_TOPS, 4),
        "traffic": None if tr1 is None else round(tr1[0]),
        "note": "one 2000 x 2000 problem per launch (osg_hamming_top2_dev): the latency form",
    }

    out = {
        "metric": "Mmatches/s (256-bit Hamming)",
        "value": round(value, 1),
        "unit": "Mmatches/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("fp4(e2m1)->f32" if fp4 else "i8->i32") if mfma else "u32",
        "data": "synthetic (SURVEY.md §8d C2 generator, seed 0x0B5EED01+rank; no EuRoC/ORBvoc in container)",
        "config": {"workload": f"C2: brute-force 256-bit Hamming top-2, 2000 x 2000 descriptors per frame, "
                               f"{B} independent frames per launch per GPU (headline; the one-frame launch is "
                               f"`single_launch`)",
                   "nq": nq, "nt": nt, "frames_per_step": B, "global_batch": world * B,
                   "untimed_ramp_launches": ramp_n,
                   "parallelism": f"replicas x{world} (independent frames per GPU, no data-path collective)"},
        "roofline": roofline,
        "single_launch": single,
        "batch_frame0_equals_single": batch_frame0_equal,
    }

    # ---- C2' streaming kernel: HBM roofline (Q = 4 x M = 2^24, 512 MiB > Infinity Cache) -----
    if not args.no_stream:
        M, Q = 1 << 24, 4
        g = torch.Generator(device=dev)
        g.manual_seed(synth.SEED_C2_STREAM + rank)
        st = torch.randint(0, 256, (M, 32), dtype=torch.uint8, device=dev, generator=g)
        sq = torch.randint(0, 256, (Q, 32), dtype=torch.uint8, device=dev, generator=g)
        so = torch.empty((Q, 3), dtype=torch.int32, device=dev)
        for _ in range(3):
            ctx.hamming_top2_dev(sq, Q, st, M, so)
        torch.cuda.synchronize(dev)
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(2_000_000)
        s0.record(stream)
        for _ in range(20):
            ctx.hamming_top2_dev(sq, Q, st, M, so)
        s1.record(stream)
        torch.cuda.synchronize(dev)
        s_us = s0.elapsed_time(s1) * 1e3 / 20
        sbytes = M * 32 + Q * 32 + Q * 12
        trs = pmc_traffic(args.traffic, "k_top2_stream")
        gbs = sbytes / (s_us * 1e-6) / 1e9
        out["roofline_stream"] = {
            "kernel": ctx.hamming_top2_plan(Q, M), "workload": "C2': Q=4 x M=2^24 train rows",
            "bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": None if trs is None else round(trs[0]),
            "kernel_us": round(s_us, 2),
            "algorithmic_bytes_per_launch": sbytes,
            "Mmatches_per_s": round(Q * M / (s_us * 1e-6) / 1e6, 1),
        }
        if world > 1:
            out["stream_train_sharded"] = bench_stream_sharded(ctx, dist, dev, stream, sq, st, world, rank)
        del st

    # ---- CPU baseline: the oracle (restatement of the reference serial loop) on host cores --
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cb = cpu_baseline(q_np, t_np, args.cpu_seconds)
        out["speedup_vs_cpu"] = round(value / cb["value"], 1)
        out["speedup_vs_cpu_1thread"] = round(value / cb["value_1thread"], 1)
        out["speedup_vs_cpu_node_estimate"] = round(value / cb["node_estimate"]["value"], 2)

    # ---- frame-batched C3 / C5: matching + PoseOptimization, B frames per launch ------------
    only = set(args.only.split(",")) if args.only else None

    def stage(key, fn):
        if only is not None and key not in only:
            return
        if rank == 0:  # progress on stderr: a long run shows it is alive
            print(f"[bench] {key} ({time.perf_counter() - t_start:.0f} s)", file=sys.stderr, flush=True)
        try:
            out[key] = fn(ctx, rank, world, dist, dev, args)
        except Exception as e:  # a failing secondary stage must not cost the headline line
            import traceback
            traceback.print_exc(file=sys.stderr)
            if world > 1:
                # the stages call collectives: a rank that skipped ahead would pair its next reduction
                # with a peer still inside this stage, so a multi-rank run ends here
                raise
            out[key] = {"error": f"{type(e).__name__}: {e}"[:500]}

    if not args.no_frames:
        stage("frames_c3", bench_c3)
        stage("frames_c5", bench_c5)
        stage("frames_dbow", bench_dbow)
        stage("frames_stereo", bench_stereo)
        stage("frames_orb", bench_orb)
        stage("frames_orb_detect", bench_orb_detect)
        stage("frames_orb_extract", bench_orb_extract)

    # ---- LocalBA iters/s on C4 (50 KF x 10k points), the second half of the metric ----------
    if not args.no_ba:
        stage("local_ba", bench_lba)
    if not args.no_gba:
        stage("global_ba", bench_gba)
        if not args.no_gba_map:
            stage("global_ba_map", bench_gba_map)
            stage("global_ba_loop", lambda *a: bench_gba_map(*a, loop=True))

    if rank == 0:
        # the full record goes to a file (mirrored under profiles/ by the GPU scripts); stdout carries
        # one compact line the driver can parse (the 21 KB line was not parsed)
        out["detail_file"] = os.path.relpath(args.detail, ROOT) if args.detail else None
        if args.detail:
            os.makedirs(os.path.dirname(os.path.abspath(args.detail)), exist_ok=True)
            with open(args.detail, "w") as f:
                json.dump(out, f, indent=1)
        print(compact_line(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


_LINE_HEAD = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data")
_LINE_ROOF = ("kernel", "bound", "achieved", "peak", "unit", "frac", "frac_of_i8_peak", "traffic", "kernel_us",
              "algorithmic_ops_per_launch", "algorithmic_flop_per_launch", "algorithmic_bytes_per_launch",
              "mfma_busy_frac_pmc")
_LINE_CPU = ("value", "unit", "cores", "kind", "flags", "value_1thread", "sample")
_LINE_STAGE = ("value", "unit", "speedup_vs_cpu", "speedup_vs_cpu_1thread", "kernel_frames_per_s",
               "kernel_speedup_vs_cpu", "equals_kernel_path", "ms_per_call", "s_per_gba", "peak_device_bytes", "error")


def _short(v, n):
    return v[:n - 3] + "..." if isinstance(v, str) and len(v) > n else v


def _pick(d, keys, n):
    return {k: _short(d[k], n) for k in keys if isinstance(d, dict) and k in d}


def compact_line(out, limit=LINE_MAX_BYTES):
    """The one JSON line bench.py prints: the headline keys, the dominant kernel's roofline, the CPU
    baseline, and per secondary stage its value, unit, speedup and (where it has one) its kernel's
    roofline fraction -- at most `limit` bytes.  The full record is the --detail file.  Strings are
    shortened first, then the stages' extras, until the line fits."""
    for n, full in ((160, True), (72, True), (40, False)):
        line = {k: _short(out[k], n) for k in _LINE_HEAD if k in out}
        line["config"] = {k: _short(v, n) for k, v in out.get("config", {}).items()}
        line["roofline"] = _pick(out.get("roofline", {}), _LINE_ROOF, n)
        if "cpu_baseline" in out:
            line["cpu_baseline"] = _pick(out["cpu_baseline"], _LINE_CPU, n)
        for k in ("speedup_vs_cpu", "speedup_vs_cpu_1thread", "speedup_vs_cpu_node_estimate",
                  "batch_frame0_equals_single"):
            if k in out:
                line[k] = out[k]
        if full and "single_launch" in out:
            line["single_launch"] = _pick(out["single_launch"], ("kernel", "kernel_us", "Mmatches_per_s_kernel"), n)
        if "roofline_stream" in out:
            line["roofline_stream"] = _pick(out["roofline_stream"], ("bound", "achieved", "peak", "unit", "frac",
                                                                     "traffic", "kernel_us"), n)
        if "stream_train_sharded" in out:
            line["stream_train_sharded"] = _pick(out["stream_train_sharded"], ("value", "unit", "n_gpus"), n)
        for key, st in out.items():
            if not (isinstance(st, dict) and key.startswith(("frames_", "local_ba", "global_ba"))):
                continue
            s = _pick(st, _LINE_STAGE if full else ("value", "unit", "speedup_vs_cpu", "error"), n)
            if "roofline" in st:
                s["roofline"] = _pick(st["roofline"], ("frac", "kernel_us", "traffic", "mfma_busy_frac_pmc")
                                      if full else ("frac", "kernel_us"), n)
            if full and "cpu_baseline" in st:
                s["cpu"] = _pick(st["cpu_baseline"], ("value", "cores", "kind", "flags"), n)
            line[key] = s
        if "detail_file" in out:
            line["detail_file"] = out["detail_file"]
        text = json.dumps(line, separators=(",", ":"))
        if len(text.encode()) <= limit:
            return text
    raise ValueError(f"bench line of {len(text.encode())} B exceeds {limit} B")


def bench_stream_sharded(ctx, dist, dev, stream, sq, st, world, rank, steps=20):
    """SURVEY.md §8(e) C2' train-sharded: the train set is world x 2^24 rows, rank r holding rows
    [r*M, (r+1)*M) in its HBM and the Q queries replicated; one step = the local streaming kernel, an
    all-gather of the (Q, 3) int32 triples over RCCL and the on-device merge into the serial loop's
    top-2 (shard.merge_top2_torch).  Weak scaling: pairs per step = Q x M x world."""
    import torch
    from orb_slam3_comments_ghr_amd import shard
    Q, M = sq.shape[0], st.shape[0]
    so = torch.empty((Q, 3), dtype=torch.int32, device=dev)
    parts = [torch.empty_like(so) for _ in range(world)]
    row0 = rank * M

    def step():
        ctx.hamming_top2_dev(sq, Q, st, M, so)
        so[:, 0] = torch.where(so[:, 0] >= 0, so[:, 0] + row0, so[:, 0])
        dist.all_gather(parts, so)
        return shard.merge_top2_torch(torch.stack(parts))

    for _ in range(3):
        step()
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        merged = step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    el, pairs = job_totals(el, Q * M * steps, world, dist, dev)
    # every rank holds the same merged result: check it agrees across ranks (cheap, outside timing)
    chk = merged.to(torch.int64).sum().reshape(1)
    lo, hi = chk.clone(), chk.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    return {"workload": f"C2' train-sharded: {world} x 2^24 train rows (rank-local), Q={Q} replicated; "
                        f"local kernel + RCCL all-gather of (Q,3) int32 + device merge per step",
            "value": round(pairs / el / 1e6, 1), "unit": "Mmatches/s", "ms_per_step": round(el / steps * 1e3, 4),
            "n_gpus": world, "scaling": "weak", "merged_equal_on_all_ranks": bool(lo.item() == hi.item())}


def pmc_traffic(path, kernel_substr):
    """Per-launch HBM bytes of the kernel from the committed PMC passes (FETCH_SIZE doubled per the
    gfx950 correction, + WRITE_SIZE), or None when no pass for it exists."""
    try:
        data = json.load(open(path))
    except (OSError, ValueError):
        return None
    best = None
    for key, v in data.get("kernels", {}).items():
        if kernel_substr in key.split("|")[0] and v.get("traffic_bytes") is not None:
            if best is None or v["launches_fetch_pass"] > best[1]["launches_fetch_pass"]:
                best = (key, v)
    return None if best is None else (best[1]["traffic_bytes"], best[0])


def pmc_traffic_instance(path, kname):
    """pmc_traffic of the exact template instance `kname` ("k_top2_fp4<16,1,256,3>") when a pass for it
    exists, else of any instance of its kernel."""
    try:
        data = json.load(open(path))
    except (OSError, ValueError):
        data = {}
    kname = kname.split(" ")[0]  # the plan string carries " grid=..." after the instance
    want = kname
    for key, v in data.get("kernels", {}).items():
        if want in key.split("|")[0].replace(" ", "") and v.get("traffic_bytes") is not None:
            return pmc_traffic(path, key.split("|")[0])
    return pmc_traffic(path, kname.split("<")[0])


def bench_lba(ctx, rank, world, dist, dev, args):
    """osg_local_bundle_adjustment on the C4 graph (host API: graph upload, structure build,
    optimize(10), classification, download), repeated; iterations / wall second.  Each rank runs
    its own window (replicas)."""
    import torch
    from orb_slam3_comments_ghr_amd import optimizer as op
    rng = np.random.default_rng(0x0B5EED04 + rank)
    G = op.synth_lba_graph(rng, n_kf=50, n_points=10000)
    opt = op.Optimizer(ctx)
    for _ in range(2):
        r = opt.LocalBundleAdjustment(G)
    reps = args.ba_reps
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    iters = 0
    for _ in range(reps):
        r = opt.LocalBundleAdjustment(G)
        iters += r.iterations
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    el, iters = job_totals(el, iters, world, dist if world > 1 else None, dev)
    iters = int(iters)
    single = {"value": round(iters / el, 1), "unit": "LM iterations/s", "ms_per_lba": round(el / reps * 1e3, 3),
              "iterations_per_lba": r.iterations, "trials_per_lba": r.trials,
              "note": "one window per call (the drop-in's latency)"}
    # batched: B independent C4 windows per GPU in lockstep (roofline on B = 64 graphs/GPU),
    # driven by T host threads, each with its own context (own HIP stream): one thread's structure
    # build and packing overlap the others' device steps, and their kernels share the GPU
    B = args.ba_batch
    T = max(1, args.lba_threads)
    pool = [G] + [op.synth_lba_graph(rng, n_kf=50, n_points=10000) for _ in range(7)]
    graphs = [pool[i % len(pool)] for i in range(B)]
    ctxs = [ctx] + [type(ctx)(ctx.device) for _ in range(T - 1)]
    opts = [opt] + [op.Optimizer(c) for c in ctxs[1:]]
    brep = max(1, args.ba_batch_reps)

    def timed(nthr):
        return _threaded_batches(ctxs[:nthr], opts[:nthr], graphs, brep, world, dist, dev)
    bel1, biters1 = timed(1)
    bel, biters = timed(T) if T > 1 else (bel1, biters1)
    for c in ctxs[1:]:
        c.close()
    bval = biters / bel
    # per-kernel device time of one batch (HIP events around every launch group, a separate untimed
    # pass): the dominant kernel's roofline
    op.lba_kernel_times(ctx, True)
    opt.LocalBundleAdjustmentBatch(graphs)
    kt = op.lba_kernel_times(ctx, False)
    steps = max(1, kt["schur_rows"][1])
    counts = [op.lba_structure_counts(g) for g in graphs]
    contrib = sum(c["contributions"] for c in counts)
    blocks = sum(c["blocks"] for c in counts)
    lms = sum(c["landmarks"] for c in counts)
    # k_schur_rows per launch: S_ij products (36 x 3 FMA per contribution), BD = Hpl Dinv and the
    # b_schur share per block (18 x 3 + 6 x 3 FMA); bytes: Hpl, and Hll and b_l (Dinv and Dinv b_l are
    # formed in the staging since late r04; the same bytes as reading them) once, 12 B of (rank, block)
    # per contribution, one 6x6 chunk partial per 64 contributions written
    # The compact per-block factor (the default, k_schur_rows_c): a block is its 48-B M (the Hpl rows are
    # rebuilt from it, the pose's R, t and the landmark's position: + 24 B per landmark), not its 144-B Hpl
    compact = os.environ.get("OSG_LBA_HPL", "0") != "1"
    sr_flop = 2.0 * (contrib * 108 + blocks * 72)
    sr_bytes = blocks * (48 if compact else 144) + lms * (120 if compact else 96) + contrib * 12 + (contrib / 64.0) * 288
    sr_s = kt["schur_rows"][0] / 1e3 / steps
    kernels = {k: round(v[0] / max(1, v[1]), 4) for k, v in kt.items() if v[1]}
    dom = max(kernels, key=kernels.get)
    pmc = _load_json(args.schur_pmc)
    # the MFMA form: "k_schur_rows<false>" (r03 / r04 files) or "k_schur_rows<false, false>" (late r04)
    # compact form: "k_schur_rows_c<0>" (first r06 file) or "k_schur_rows_c<1>" / "<2>" (gather-ahead depth)
    pmc_sr = next((v for k, v in pmc.items() if (k.startswith("k_schur_rows_c<") if compact else
                                                 k in ("k_schur_rows<false>", "k_schur_rows<false, false>"))), {})
    flop_iter = 72.6e6
    res = {
        "metric": "LocalBA iters/s", "value": round(bval, 1), "unit": "LM iterations/s",
        "workload": f"C4: {len(G.pose)} KF x {len(G.point)} points x {len(G.e_point)} mono edges, optimize(10); "
                    f"{B} independent windows per lockstep batch (8 distinct), {T} host threads per GPU each "
                    f"driving {brep} batches on its own context / HIP stream",
        "ms_per_round": round(bel / brep * 1e3, 3), "windows_per_batch": B, "host_threads": T,
        "windows_in_flight": B * T, "one_thread": {"value": round(biters1 / bel1, 1),
                                                   "ms_per_batch": round(bel1 / brep * 1e3, 3)},
        "n_gpus": world, "dtype": "f64",
        "scaling": "weak", "parallelism": f"replicas x{world} (independent windows per GPU)",
        "flop_per_iter_survey_formula": flop_iter,
        "roofline": {"kernel": ("k_schur_rows_c (compact per-block factor; " if compact else "k_schur_rows (") +
                               "Schur product S_ij -= sum BD_i Hpl_j^T on v_mfma_f64_4x4x4f64)",
                     "dominant_kernel": dom, "bound": "mfma", "achieved": round(sr_flop / sr_s / 1e12, 4),
                     "peak": 78.6, "unit": "TFLOP/s", "frac": round(sr_flop / sr_s / 1e12 / 78.6, 5),
                     "kernel_us": round(sr_s * 1e6, 2), "windows_per_launch": B,
                     "algorithmic_flop_per_launch": sr_flop, "algorithmic_bytes_per_launch": round(sr_bytes),
                     "hbm_GBps_if_priced_as_hbm": round(sr_bytes / sr_s / 1e9, 1),
                     "mfma_busy_frac_pmc": pmc_sr.get("mfma_busy_frac"),
                     "traffic": pmc_sr.get("hbm_bytes_per_launch"),
                     "pmc_source": os.path.relpath(args.schur_pmc, ROOT) if pmc else None},
        "kernel_ms_per_step": kernels,
        "whole_call_fp64_frac": round(bval * flop_iter / 1e12 / 78.6, 5),
        "single_window": single,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        # LM iterations per window on the CPU, averaged over the pool the workers cycle through
        it_cpu = float(np.mean([_oracle()[1].lba(_oracle()[0], g).iterations for g in pool]))
        _attach_cpu(res, _lba_worker(pool), it_cpu, "LM iterations/s", args.cpu_seconds * 0.75,
                    "C4 LBA (oracle_local_bundle_adjustment, dense LDL^T)", wall_key="")
        single["speedup_vs_cpu_1thread"] = round(single["value"] / res["cpu_baseline"]["value_1thread"], 1)
    return res


def _threaded_batches(ctxs, opts, graphs, brep, world, dist, dev):
    """Each of len(opts) host threads runs `brep` lockstep batches of `graphs`
    (osg_local_bundle_adjustment_batch) on its own context / HIP stream after one untimed batch;
    returns (max-over-ranks seconds, LM iterations of all ranks)."""
    import threading
    import torch
    nthr = len(opts)
    for o in opts:
        o.LocalBundleAdjustmentBatch(graphs)
    for c in ctxs:
        c.synchronize()
    its = [0] * nthr

    def run(t):
        for _ in range(brep):
            its[t] += sum(x.iterations for x in opts[t].LocalBundleAdjustmentBatch(graphs))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    th = [threading.Thread(target=run, args=(t,)) for t in range(nthr)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    torch.cuda.synchronize(dev)
    return job_totals(time.perf_counter() - t0, sum(its), world, dist if world > 1 else None, dev)


def _lba_worker(graphs):
    """cpu_baseline worker for BA: one graph per call, round-robin over `graphs`; outputs per thread."""
    def worker(tid):
        import ctypes as C
        from orb_slam3_comments_ghr_amd import optimizer as op
        lib, _ = _oracle()
        items = []
        for g in graphs:
            R, out = op.make_ba_result(g)
            gs = g.struct()
            items.append(((C.byref(gs), C.byref(R), None), (R, out, gs)))
        fn = lib.oracle_local_bundle_adjustment
        return lambda i, items=items: fn(*items[i % len(items)][0])
    return worker


def bench_gba(ctx, rank, world, dist, dev, args):
    """Optimizer::BundleAdjustment (global BA) on a synthetic whole map of 150
    KeyFrames x 20k points (only the init KeyFrame fixed, no Huber kernel: LoopClosing's
    GlobalBundleAdjustemnt(map, 10, &mbStopGBA, nLoopKF, false)); LM iterations per wall second of
    the whole call (structure build, upload, LM, download).
    `value`: independent maps per GPU as the CPU baseline runs them (one map per host thread there):
    B maps per lockstep batch (osg_local_bundle_adjustment_batch, the engine osg_bundle_adjustment
    runs with B = 1), T host threads with their own contexts.  `single_map`: one map per call, the
    drop-in's latency.  Replicas: the maps of each rank are its own."""
    import torch
    from orb_slam3_comments_ghr_amd import optimizer as op
    rng = np.random.default_rng(0x0B5EED30 + rank)
    G = op.synth_gba_graph(rng, n_kf=150, n_points=20000)
    opt = op.Optimizer(ctx)
    r = opt.BundleAdjustment(G)
    reps = 5
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    iters = 0
    for _ in range(reps):
        r = opt.BundleAdjustment(G)
        iters += r.iterations
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    el, iters = job_totals(el, iters, world, dist if world > 1 else None, dev)
    n_free = int(len(G.pose) - G.pose_fixed.sum())
    single = {"value": round(iters / el, 1), "unit": "LM iterations/s", "ms_per_gba": round(el / reps * 1e3, 3),
              "iterations_per_gba": r.iterations, "trials_per_gba": r.trials,
              "note": "one map per call (osg_bundle_adjustment: the drop-in's latency)"}
    B, T, brep = max(1, args.gba_batch), max(1, args.gba_threads), max(1, args.gba_batch_reps)
    pool = [G] + [op.synth_gba_graph(rng, n_kf=150, n_points=20000) for _ in range(3)]
    graphs = [pool[i % len(pool)] for i in range(B)]
    ctxs = [ctx] + [type(ctx)(ctx.device) for _ in range(T - 1)]
    opts = [opt] + [op.Optimizer(c) for c in ctxs[1:]]
    bel, biters = _threaded_batches(ctxs, opts, graphs, brep, world, dist, dev)
    for c in ctxs[1:]:
        c.close()
    res = {"metric": "GlobalBA iters/s", "value": round(biters / bel, 1), "unit": "LM iterations/s",
           "workload": f"global BA: {len(G.pose)} KF x {len(G.point)} points x {len(G.e_point)} edges, "
                       f"reduced system {6 * n_free} (dense), optimize({G.iterations}), no Huber; {B} independent "
                       f"maps per lockstep batch ({len(pool)} distinct), {T} host threads per GPU each driving "
                       f"{brep} batches on its own context / HIP stream",
           "maps_per_batch": B, "host_threads": T, "maps_per_s": round(B * T * brep * world / bel, 1),
           "single_map": single,
           "n_gpus": world, "dtype": "f64", "scaling": "weak", "parallelism": f"replicas x{world} (independent maps per GPU)"}
    if rank == 0 and world == 1 and not args.no_cpu:
        it_cpu = float(np.mean([_oracle()[1].lba(_oracle()[0], g).iterations for g in pool]))
        _attach_cpu(res, _lba_worker(pool), it_cpu, "LM iterations/s", max(3.0, args.cpu_seconds * 0.5),
                    "global BA 150 KF x 20k points (oracle, dense LDL^T), one map per thread", wall_key="")
        single["speedup_vs_cpu_1thread"] = round(single["value"] / res["cpu_baseline"]["value_1thread"], 1)
    return res


def bench_gba_map(ctx, rank, world, dist, dev, args, loop=False):
    """SURVEY.md §8(f) rank 4 at map scale: BundleAdjustment over a 1500-KeyFrame x 150 k-point map
    (optimizer.synth_map_graph: an open 0.45 km path, 600 k edges, reduced system n = 8994, banded).
    Wall time of the whole call per map.  The CPU baseline is the oracle on one thread: g2o's LM is
    single-threaded, so more cores do not speed up one map (they only run more maps).
    loop=True (global_ba_loop): the same map closed into a loop (synth_map_graph(loop=True)), the global
    BA LoopClosing starts after a loop closure (ref:src/LoopClosing.cc:2436); device memory the call
    holds (a fresh context's arena after one call, osg_ctx_device_bytes) is reported as peak_device_bytes."""
    import torch
    from orb_slam3_comments_ghr_amd import optimizer as op
    G = op.synth_map_graph(np.random.default_rng(0x0B5EED31 + rank), n_kf=1500, n_points=150000, loop=loop)
    # a context of its own, so its arena is this map's peak alone (slots grow to a call's needs and stay)
    from orb_slam3_comments_ghr_amd import Context
    mctx = Context(dev.index if dev.index is not None else 0)
    opt = op.Optimizer(mctx)
    r = opt.BundleAdjustment(G)
    torch.cuda.synchronize(dev)
    held = mctx.device_bytes()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    reps = 2
    t0 = time.perf_counter()
    iters = 0
    for _ in range(reps):
        r = opt.BundleAdjustment(G)
        iters += r.iterations
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    el, iters = job_totals(el, iters, world, dist if world > 1 else None, dev)
    n_free = int(len(G.pose) - G.pose_fixed.sum())
    res = {"metric": "GlobalBA iters/s", "value": round(iters / el, 1), "unit": "LM iterations/s",
           "s_per_gba": round(el / reps, 3), "iterations_per_gba": r.iterations, "trials_per_gba": r.trials,
           "workload": f"global BA at map scale: {len(G.pose)} KF x {len(G.point)} points x {len(G.e_point)} edges, "
                       f"reduced system {6 * n_free} ("
                       + ("a loop-closed map: the band plus its corner blocks" if loop else "banded: an open trajectory")
                       + f"), optimize({G.iterations}), no Huber",
           "peak_device_bytes": int(held),
           "peak_device_note": "device memory a fresh context holds after one call (osg_ctx_device_bytes): the "
                               "arena grows to the call's peak and stays; includes the dense n x n reduced matrix",
           "n_gpus": world, "dtype": "f64", "scaling": "weak", "parallelism": f"replicas x{world} (one map per GPU)"}
    if rank == 0 and world == 1 and not args.no_cpu:
        orc, oc = _oracle()
        from tests import cpu_mt
        t1 = time.perf_counter()
        rc = oc.lba(orc, G)
        tc = time.perf_counter() - t1
        res["cpu_baseline"] = {"value": round(rc.iterations / tc, 2), "unit": "LM iterations/s", "cores": 1,
                               "kind": "port", "flags": cpu_mt.ORACLE_FLAGS, "seconds_per_gba": round(tc, 2),
                               "sample": "one call of the oracle on the same map (envelope LDL^T; g2o's LM is "
                                         "single-threaded, so one map does not use more cores)"}
        res["speedup_vs_cpu"] = round(res["value"] / res["cpu_baseline"]["value"], 1)
        res["speedup_per_map_seconds"] = round(tc / (el / reps), 1)
    return res


_ORACLE = []


def _ref_pattern():
    """The reference's own BRIEF table (ref:src/ORBextractor.cc:212, data in tests/golden/)."""
    from tests import golden_data
    return golden_data.bit_pattern_31()


_TIMING_BUILD = {}


def _start_timing_build():
    """Compile the timing-only oracle (oracle/Makefile `timing`: -O3 -march=native, GCC's default
    contraction -- the reference's release flags) for this host's CPU in a
    background thread, so the ~2 s build overlaps the GPU stages.  -march=native means the box's own
    CPU, so the build happens here, never in the container that cross-compiles the HIP library."""
    import tempfile
    import threading
    d = tempfile.mkdtemp(prefix="osg_oracle_timing_")

    def run():
        from tests import oracle_calls
        try:
            _TIMING_BUILD["lib"] = oracle_calls.load_timing(d)
        except Exception as e:  # noqa: BLE001 - the checker build stands in, and the line says so
            _TIMING_BUILD["error"] = f"{type(e).__name__}: {e}"[:300]
    th = threading.Thread(target=run, daemon=True)
    th.start()
    _TIMING_BUILD["thread"] = th


def _oracle():
    """The CPU oracle (test infrastructure), loaded only by the cpu_baseline legs.  It times the
    reference's own arithmetic: the host libm's sin / cos / pow / atan2 (oracle_set_libm), not the
    correctly rounded evaluations the parity tests hold both sides to, compiled with the reference's
    release flags (the timing build) when that build succeeded on this host."""
    if not _ORACLE:
        from tests import cpu_mt, oracle_calls
        if "thread" not in _TIMING_BUILD:
            _start_timing_build()
        _TIMING_BUILD["thread"].join()
        if "lib" in _TIMING_BUILD:
            lib, flags = _TIMING_BUILD["lib"]
            cpu_mt.ORACLE_FLAGS = flags + " (timing build)"
        else:
            lib = oracle_calls.load()
            cpu_mt.ORACLE_FLAGS = ("-O3 -ffp-contract=off -fno-fast-math (the checker build: the timing build failed: "
                                   + _TIMING_BUILD.get("error", "?") + ")")
        lib.oracle_set_libm(1)
        _ORACLE.append((lib, oracle_calls))
    return _ORACLE[0]


def _threaded_wall(ctx, nthr, reps, call):
    """Frames per wall second with `nthr` host threads, each with its own context (own HIP stream), each
    running `reps` calls of call(ctx_t, i): the throughput of nthr independent extractor / tracking
    threads sharing one GPU."""
    import threading
    ctxs = [ctx] + [type(ctx)(ctx.device) for _ in range(nthr - 1)]
    for c in ctxs:
        call(c, 0)
    for c in ctxs:
        c.synchronize()

    def run(t):
        for i in range(reps):
            call(ctxs[t], i)
    t0 = time.perf_counter()
    th = [threading.Thread(target=run, args=(t,)) for t in range(nthr)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    el = time.perf_counter() - t0
    for c in ctxs[1:]:
        c.close()
    return nthr * reps / el


def _load_json(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def _pose_result(P):
    """An osg_pose_result with its outlier buffer (kept alive by the returned tuple)."""
    from orb_slam3_comments_ghr_amd import _abi
    r = _abi.OsgPoseResult()
    o = np.zeros(max(P.n, 1), np.uint8)
    r.outlier = o.ctypes.data
    return r, o


def _latency(gpu_call, cpu_call=None, reps=200, ctx=None):
    """Single-call latency of one drop-in call, the way Tracking issues them (one frame at a time,
    ref:src/Tracking.cc:3507): the C-ABI entry with host inputs and outputs (upload, kernels,
    download, stream sync), arguments packed beforehand as the C++ adapter packs them.  Median and
    p90 over `reps` calls; beside it the oracle's 1-thread time for the same call.  With ctx, the
    call's own kernel time (ctx.last_kernel_ms: HIP events around its launches) is recorded per call
    too: kernel_us (median) and host_us = the median call minus it."""
    ks = []

    def timeit(call, n, k=None):
        for _ in range(5):
            call()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            call()
            ts.append(time.perf_counter() - t0)
            if k is not None:
                k.append(ctx.last_kernel_ms() * 1e3)
        ts.sort()
        return ts[len(ts) // 2] * 1e6, ts[int(len(ts) * 0.9)] * 1e6
    g50, g90 = timeit(gpu_call, reps, ks if ctx is not None else None)
    out = {"gpu_us_median": round(g50, 1), "gpu_us_p90": round(g90, 1)}
    if ks:
        k50 = sorted(ks)[len(ks) // 2]
        out["kernel_us_median"] = round(k50, 1)
        out["host_us"] = round(g50 - k50, 1)
    if cpu_call is not None:
        c50, _ = timeit(cpu_call, max(10, reps // 10))
        out["cpu_1thread_us_median"] = round(c50, 1)
        out["speedup_vs_cpu_1thread"] = round(c50 / g50, 2)
    return out


def _frame_batches(ctx, rank, world, dist, dev, args, steps, cpu_worker, label, workload, n_pool, cpu_frames=1,
                   latency=None):
    """Time `steps` (a list of callables, each one batched launch over B frames that leaves its
    kernel time in ctx.last_kernel_ms()) over args.frame_reps repetitions.  value = frames / summed
    kernel time (inputs resident in HBM: the device time of the launches); the wall rate includes
    host packing and PCIe.  cpu_worker(tid) -> call(i) runs frame i of the pool (or cpu_frames frames)
    through the oracle with its arguments packed once per thread (tests/cpu_mt.py)."""
    import torch
    for f in steps:
        f()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    k_ms = 0.0
    per = [0.0] * len(steps)
    t0 = time.perf_counter()
    for _ in range(args.frame_reps):
        for i, f in enumerate(steps):
            f()
            ms = ctx.last_kernel_ms()
            per[i] += ms
            k_ms += ms
    wall = time.perf_counter() - t0
    frames = args.frames * args.frame_reps
    k_s, tot = job_totals(k_ms / 1e3, frames, world, dist if world > 1 else None, dev)
    w_s, _ = job_totals(wall, frames, world, dist if world > 1 else None, dev)
    res = {"metric": "frames/s", "value": round(tot / k_s, 1), "unit": "frames/s",
           "workload": workload, "frames_per_launch": args.frames, "distinct_frames": n_pool,
           "kernel_us_per_frame": {lab: round(v * 1e3 / frames, 3) for lab, v in zip(label, per)},
           "wall_frames_per_s_incl_host_and_pcie": round(tot / w_s, 1), "n_gpus": world,
           "scaling": "weak", "parallelism": f"replicas x{world} (independent frame batches per GPU)"}
    if latency:
        res["single_call_latency"] = latency
    if rank == 0 and world == 1 and not args.no_cpu:
        _attach_cpu(res, cpu_worker, cpu_frames, "frames/s", args.cpu_seconds * 0.4, label[0] if len(label) == 1
                    else " + ".join(label))
    return res


def _cpp_wall(res, workload, arrays, expect, args, rank, world, dist=None, dev=None):
    """The drop-in's wall rate as ORB-SLAM3 would see it: tools/adapter_wall_bench (C++) gathers mock
    Frames / KeyFrames / MapPoints through adapters/orbslam3/osg_orbslam3.h's batched entries, calls the
    C-ABI with host inputs and writes the results back into the objects, on --wall-threads host
    threads with one context each.  `arrays` is the problem pool (tools/adapter_arrays.py);
    `expect` maps each recorded per-frame result to the kernel-only path's values on the same pool,
    and `equals_kernel_path` says whether the adapter run reproduced them.  Every rank runs it on its
    own GPU (HIP_VISIBLE_DEVICES = LOCAL_RANK for the child); the whole-job rate is all ranks' frames
    over the slowest rank's wall time.  The one-frame latency runs on rank 0."""
    if args.no_wall:
        return
    import subprocess
    import tempfile
    from tools.adapter_arrays import write_arrays
    exe = os.path.join(ROOT, "tools", "adapter_wall_bench")
    env = dict(os.environ)
    if world > 1:
        # this rank's GPU in the parent's own numbering: the LOCAL_RANK-th entry of a device list the
        # launcher already set, else the ordinal itself
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
            vis = [x for x in os.environ.get(var, "").split(",") if x.strip()]
            if vis:
                env[var] = vis[lr % len(vis)]
                break
        else:
            env["HIP_VISIBLE_DEVICES"] = str(lr)
    threads = args.wall_threads
    if threads <= 0:  # the same host cores as the CPU baseline (its `cores`), split between local ranks
        from tests import cpu_mt
        threads = max(1, min(64, cpu_mt.host_threads() // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))))
    ok = os.path.exists(exe)
    if ok:
        with tempfile.TemporaryDirectory() as d:
            path = os.path.join(d, "pool.arrays")
            write_arrays(path, arrays)
            r = subprocess.run([exe, workload, path, str(args.wall_frames), str(args.wall_reps),
                                str(threads)], capture_output=True, text=True, timeout=300, env=env)
        ok = r.returncode == 0
    # every rank takes part in the reductions, whatever its own child did
    w = json.loads(r.stdout.strip().splitlines()[-1]) if ok else {"frames": 0, "wall_s": 0.0}
    bad_ranks = 1.0 - float(ok)
    w_s, frames = job_totals(w["wall_s"], w["frames"], world, dist if world > 1 else None, dev)
    if world > 1:
        _, bad_ranks = job_totals(0.0, bad_ranks, world, dist, dev)
    if not ok:
        res["wall_cpp_adapter"] = {"error": "tools/adapter_wall_bench is not built (make)" if not os.path.exists(exe)
                                   else (r.stdout + r.stderr)[-600:]}
        return
    if bad_ranks:
        res["wall_cpp_adapter"] = {"error": f"{int(bad_ranks)} rank(s) failed the adapter wall bench"}
        return
    n = min(args.wall_frames, w["distinct_problems"])
    first = w.pop("first_rep")
    bad = {}
    for k, v in expect.items():
        got, want = [int(x) for x in first[k]], [int(x) for x in v[:n]]
        if got != want:
            i = next((j for j in range(min(len(got), len(want))) if got[j] != want[j]), min(len(got), len(want)))
            bad[k] = {"first_index": i, "adapter": got[i:i + 4], "kernel_path": want[i:i + 4]}
    w["equals_kernel_path"] = not bad
    if bad:
        w["mismatch"] = bad
    w["note"] = ("tools/adapter_wall_bench.cpp: gather from mock ORB-SLAM3 objects, C-ABI call with host inputs "
                 "(pack, PCIe, kernels, download), write-back; frames / wall second over all host threads")
    res["wall_cpp_adapter_frames_per_s"] = round(frames / w_s, 1)
    res["wall_cpp_adapter"] = w
    res["equals_kernel_path"] = not bad
    if bad:
        # a wrong-result adapter run is never the stage's value: the kernel rate stays, flagged
        res["error"] = "C++ adapter results differ from the kernel path: " + json.dumps(bad)[:300]
        return
    # the drop-in's wall rate is the workload's value: what ORB-SLAM3 would see,
    # host gather, packing, PCIe and write-back included; the batched launches' device time is beside it
    res["kernel_frames_per_s"] = res["value"]
    res["value"] = res["wall_cpp_adapter_frames_per_s"]
    res["value_kind"] = ("C++ adapter wall rate (tools/adapter_wall_bench: mock ORB-SLAM3 objects -> C-ABI with host "
                         f"buffers -> write-back, {threads} host threads x {args.wall_frames} frames per call)")
    if "cpu_baseline" in res:
        cb = res["cpu_baseline"]
        res["kernel_speedup_vs_cpu"] = res["speedup_vs_cpu"]
        res["speedup_vs_cpu"] = round(res["value"] / cb["value"], 2)
        res["speedup_vs_cpu_1thread"] = round(res["value"] / cb["value_1thread"], 1)
        res["speedup_vs_cpu_node_estimate"] = round(res["value"] / cb["node_estimate"]["value"], 2)
    if rank != 0:
        return
    # the drop-in as ORB-SLAM3 calls it: one frame per call, one thread, from C++ (no Python in the loop)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "pool.arrays")
        write_arrays(path, arrays)
        r1 = subprocess.run([exe, workload, path, "1", "200", "1"], capture_output=True, text=True, timeout=300,
                            env=env)
    if r1.returncode == 0:
        w1 = json.loads(r1.stdout.strip().splitlines()[-1])
        res["single_call_latency_cpp_adapter_us"] = {k: round(v / w1["reps"] * 1e6, 1)
                                                     for k, v in w1["thread0_stage_s"].items()}


def _attach_cpu(res, worker, units, unit, seconds, label, wall_key="wall_frames_per_s_incl_host_and_pcie"):
    """res["cpu_baseline"] (N threads, one problem per thread) and the speedups: kernel-time value and,
    when recorded, the host- and PCIe-inclusive wall rate, each against the N-thread and 1-thread CPU."""
    from tests import cpu_mt
    cb = cpu_mt.baseline(worker, units, unit, seconds, label)
    res["cpu_baseline"] = cb
    res["speedup_vs_cpu"] = round(res["value"] / cb["value"], 2)
    res["speedup_vs_cpu_1thread"] = round(res["value"] / cb["value_1thread"], 1)
    res["speedup_vs_cpu_node_estimate"] = round(res["value"] / cb["node_estimate"]["value"], 2)
    if wall_key in res:
        res["wall_speedup_vs_cpu"] = round(res[wall_key] / cb["value"], 2)


def bench_c3(ctx, rank, world, dist, dev, args):
    """C3: SearchByBoW(KF, F) + PoseOptimization per frame, B frames per launch.
    The pose problem of a frame has as many edges as its BoW matches (60 % stereo, 10 % outliers)."""
    from orb_slam3_comments_ghr_amd import frames as fr, optimizer as op
    from orb_slam3_comments_ghr_amd.matcher import ORBmatcher
    n_pool = 32
    rng = np.random.default_rng(0x0B5EED03 + rank)
    pairs = [fr.synth_bow_pair(rng, n_kf=1200, n_f=1200, n_nodes=100) for _ in range(n_pool)]
    for pair in pairs:  # a MapPoint-less keypoint has no goodness flag (the mock KeyFrame holds NULL there)
        for S in pair:
            S.mp_good = (S.mp_good.astype(bool) & (S.mp_id >= 0)).astype(np.uint8)
    m = ORBmatcher(ctx, 0.7, True)
    nm, _ = m.SearchByBoWBatch([p[0] for p in pairs], [p[1] for p in pairs])
    # keypoints are float (cv::KeyPoint): the problems the adapter can gather from a Frame
    probs = [pose_for_mock(op.synth_pose_problem(rng, n_edges=int(max(nm[i], 10)))) for i in range(n_pool)]
    B = args.frames
    KB = [pairs[i % n_pool][0] for i in range(B)]
    FB = [pairs[i % n_pool][1] for i in range(B)]
    PB = [probs[i % n_pool] for i in range(B)]
    opt = op.Optimizer(ctx)

    cpu = _c3_worker(pairs, probs)
    lat = None
    if rank == 0:
        import ctypes as C
        lib, h = ctx.lib, ctx.handle
        a, b = pairs[0][0].struct(), pairs[0][1].struct()
        o = np.full(pairs[0][1].n, -1, np.int32)
        ps, (rs, keep) = probs[0].struct(), _pose_result(probs[0])
        lat = {"SearchByBoW(KF,F)": _latency(
                   lambda: lib.osg_search_by_bow_kf_f(h, C.byref(a), C.byref(b), 0.7, 1, o.ctypes.data),
                   None if args.no_cpu else lambda: _oracle()[0].oracle_search_by_bow_kf_f(
                       C.byref(a), C.byref(b), 0.7, 1, o.ctypes.data)),
               f"PoseOptimization ({probs[0].n} edges)": _latency(
                   lambda: lib.osg_pose_optimization(h, C.byref(ps), C.byref(rs)),
                   None if args.no_cpu else lambda: _oracle()[0].oracle_pose_optimization(C.byref(ps), C.byref(rs)),
                   ctx=ctx)}

    res = _frame_batches(ctx, rank, world, dist, dev, args,
                         [lambda: m.SearchByBoWBatch(KB, FB), lambda: opt.PoseOptimization(PB)], cpu,
                         ["SearchByBoW", "PoseOptimization"],
                         f"C3: SearchByBoW(KF,F) 1200x1200 (100 nodes) + PoseOptimization "
                         f"(mean {int(np.mean(nm))} edges, 60 % stereo), {B} frames per launch", n_pool,
                         latency=lat)
    arrays = {"pool.n": np.array([n_pool], np.int32)}
    for i in range(n_pool):
        arrays.update(prefixed(f"p{i}.", {**bow_arrays("B1.", pairs[i][0]), **bow_arrays("B2.", pairs[i][1]),
                                          **pose_arrays(probs[i])}))
    _cpp_wall(res, "c3", arrays, {"SearchByBoW": nm, "PoseOptimization": [r.n_inliers for r in
                                                                          opt.PoseOptimization(probs)]},
              args, rank, world, dist, dev)
    return res


def bench_c5(ctx, rank, world, dist, dev, args):
    """C5: TUM-VI-like two-camera KB8 fisheye rig (512 x 512, 1000 keypoints per
    camera): SearchByProjection(F, LastF) + SearchByProjection(F, local map) + PoseOptimization
    (40 % right-camera edges) per frame, B frames per launch."""
    from orb_slam3_comments_ghr_amd import frames as fr, optimizer as op
    from orb_slam3_comments_ghr_amd.matcher import ORBmatcher
    n_pool = 32
    rng = np.random.default_rng(0x0B5EED10 + rank)
    F = [fr.synth_frame_two_cam(rng, n_left=1000, n_right=1000, stereo_frac=0.5, width=512, height=512)
         for _ in range(n_pool)]
    L = [fr.synth_last_queries_two_cam(rng, f, n_last=2000) for f in F]
    for x in L:  # only a LastFrame slot with a MapPoint can be valid (the mock Frame holds NULL elsewhere)
        x.valid = (x.valid.astype(bool) & (x.mp_id >= 0)).astype(np.uint8)
    Q = [fr.synth_mp_queries_two_cam(rng, f, m=1500) for f in F]
    for x in Q:  # the local map's MapPoints all have observations (Tracking::UpdateLocalPoints)
        x.has_obs[:] = 1
    S = [fr.synth_slots(rng, f.n, frac_assigned=0.05) for f in F]
    # left-camera edges first, then the right camera's, as a two-camera Frame's slots are ordered
    probs = [pose_for_mock(op.synth_pose_problem(rng, n_edges=600, cam=op.kb8_camera(), body_frac=0.4))
             for _ in range(n_pool)]
    B = args.frames
    idx = [i % n_pool for i in range(B)]
    FB, LB, QB, PB = [F[i] for i in idx], [L[i] for i in idx], [Q[i] for i in idx], [probs[i] for i in idx]
    TB = [S[i][1] for i in idx]
    m = ORBmatcher(ctx, 0.9, True)
    m_local = ORBmatcher(ctx, 0.9, True)
    opt = op.Optimizer(ctx)

    cpu = _c5_worker(F, L, Q, S, probs)
    lat = None
    if rank == 0:
        import ctypes as C
        lib, h = ctx.lib, ctx.handle
        fs, ls, qs = F[0].struct(), L[0].struct(), Q[0].struct()
        sl, tk = S[0][0].copy(), np.ascontiguousarray(S[0][1], np.uint8)
        ps, (rs, keep) = probs[0].struct(), _pose_result(probs[0])
        orc = None if args.no_cpu else _oracle()[0]

        def last(fn, *pre):
            return lambda: (np.copyto(sl, S[0][0]), fn(*pre, C.byref(fs), C.byref(ls), 7.0, 0, 1, sl.ctypes.data,
                                                         tk.ctypes.data))

        def mps(fn, *pre):
            return lambda: (np.copyto(sl, S[0][0]), fn(*pre, C.byref(fs), C.byref(qs), 0.9, 3.0, 0, 20.0,
                                                         sl.ctypes.data, tk.ctypes.data))
        lat = {"SearchByProjection(F,LastF)": _latency(last(lib.osg_search_by_projection_last, h),
                                                       orc and last(orc.oracle_search_by_projection_last)),
               "SearchByProjection(F,localMPs)": _latency(mps(lib.osg_search_by_projection_mps, h),
                                                          orc and mps(orc.oracle_search_by_projection_mps)),
               f"PoseOptimization KB8 ({probs[0].n} edges)": _latency(
                   lambda: lib.osg_pose_optimization(h, C.byref(ps), C.byref(rs)),
                   orc and (lambda: orc.oracle_pose_optimization(C.byref(ps), C.byref(rs))), ctx=ctx)}

    res = _frame_batches(ctx, rank, world, dist, dev, args,
                         [lambda: m.SearchByProjectionBatch(FB, LB, 7.0, False, slot_mps=[S[i][0].copy() for i in idx],
                                                            slot_takens=TB),
                          lambda: m_local.SearchByProjectionBatch(FB, QB, 3.0, False, 20.0,
                                                                  slot_mps=[S[i][0].copy() for i in idx],
                                                                  slot_takens=TB),
                          lambda: opt.PoseOptimization(PB)], cpu,
                         ["SearchByProjection(F,LastF)", "SearchByProjection(F,localMPs)", "PoseOptimization"],
                         f"C5: two-camera KB8 512x512, 2x1000 keypoints; LastF 2000 + local map 1500 queries; "
                         f"PoseOptimization 600 edges (40 % right camera); {B} frames per launch", n_pool,
                         latency=lat)
    arrays = {"pool.n": np.array([n_pool], np.int32)}
    for i in range(n_pool):
        arrays.update(prefixed(f"p{i}.", {**frame_arrays(F[i]), **slot_arrays(*S[i]), **last_arrays(L[i]),
                                          **mps_arrays(Q[i]), **pose_arrays(probs[i])}))
    expect = {"SearchByProjection(F,LastF)": m.SearchByProjectionBatch(
                  F, L, 7.0, False, slot_mps=[x[0].copy() for x in S], slot_takens=[x[1] for x in S]),
              "SearchByProjection(F,localMPs)": m_local.SearchByProjectionBatch(
                  F, Q, 3.0, False, 20.0, slot_mps=[x[0].copy() for x in S], slot_takens=[x[1] for x in S]),
              "PoseOptimization": [r.n_inliers for r in opt.PoseOptimization(probs)]}
    _cpp_wall(res, "c5", arrays, expect, args, rank, world, dist, dev)
    return res


def bench_dbow(ctx, rank, world, dist, dev, args):
    """Frame::ComputeBoW = DBoW2 transform(features, BowVector,
    FeatureVector, levelsup = 4) against an ORBvoc-shaped vocabulary (k = 10, L = 6, seeded
    synthetic: ORBvoc.txt is not in the container), 1200 descriptors per frame, B frames per
    launch."""
    from orb_slam3_comments_ghr_amd import vocabulary as vb
    n_pool = 16
    rng = np.random.default_rng(0x0B5EEDB0 + rank)
    voc = vb.synth_vocabulary(rng, k=10, L=6, min_children=8, min_leaf_depth=6)
    gv = vb.ORBVocabulary(ctx, voc)
    pool = [vb.synth_features(rng, voc, n=1200) for _ in range(n_pool)]
    B = args.frames
    sets = [pool[i % n_pool] for i in range(B)]

    cpu = _dbow_worker(voc, pool)

    res = _frame_batches(ctx, rank, world, dist, dev, args, [lambda: gv.transform_batch(sets, 4)], cpu,
                         ["transform"],
                         f"DBoW2 transform, levelsup 4: k=10 L=6 vocabulary ({voc.n_nodes} nodes, {voc.n_words} "
                         f"words), 1200 descriptors per frame; {B} frames per launch", n_pool, cpu_frames=n_pool)
    gv.transform_batch(sets[:1], 4)
    res["single_frame_kernel_us"] = round(ctx.last_kernel_ms() * 1e3, 2)
    ref = gv.transform_batch(pool, 4)
    gv.close()
    arrays = {"pool.n": np.array([n_pool], np.int32), **vocabulary_arrays(voc)}
    for i, d in enumerate(pool):
        arrays[f"p{i}.D.desc"] = np.ascontiguousarray(d, np.uint8).reshape(-1)
    _cpp_wall(res, "dbow", arrays, {"n_words": [len(r.word) for r in ref], "n_nodes": [len(r.node_id) for r in ref]},
              args, rank, world, dist, dev)
    return res


def bench_stereo(ctx, rank, world, dist, dev, args):
    """Frame::ComputeStereoMatches on EuRoC-shaped stereo pairs (752 x 480,
    8 levels x 1.2, 1200 keypoints per side; seeded synthetic scene, no EuRoC images in the
    container), B frames per launch, both image pyramids resident in HBM."""
    from orb_slam3_comments_ghr_amd import stereo as st
    n_pool = 16
    rng = np.random.default_rng(0x0B5EED20 + rank)
    pool = [st.synth_stereo_frame(rng, n=1200) for _ in range(n_pool)]
    dpool = [f.to_device(dev) for f in pool]
    B = args.frames
    frames = [dpool[i % n_pool] for i in range(B)]

    cpu = _stereo_worker(pool)

    res = _frame_batches(ctx, rank, world, dist, dev, args, [lambda: st.ComputeStereoMatchesBatch(ctx, frames)], cpu,
                         ["ComputeStereoMatches"],
                         f"ComputeStereoMatches: EuRoC-shaped 752x480 stereo pairs, 8 levels, 1200 keypoints per "
                         f"side, pyramids in HBM; {B} frames per launch", n_pool)
    st.ComputeStereoMatchesBatch(ctx, frames[:1])
    res["single_frame_kernel_us"] = round(ctx.last_kernel_ms() * 1e3, 2)
    _, nm = st.ComputeStereoMatchesBatch(ctx, dpool)
    arrays = {"pool.n": np.array([n_pool], np.int32)}
    for i, f in enumerate(pool):
        arrays.update(prefixed(f"p{i}.", stereo_arrays(f)))
    _cpp_wall(res, "stereo", arrays, {"ComputeStereoMatches": list(nm)}, args, rank, world, dist, dev)
    return res


def bench_orb(ctx, rank, world, dist, dev, args):
    """SURVEY.md §8(f) rank 4 (ORBextractor): IC_Angle + steered BRIEF for one EuRoC frame's keypoints
    (752 x 480, 8 levels x 1.2, 1200 keypoints spread by level area; seeded synthetic images, no EuRoC
    images in the container) per call, both pyramids resident in HBM.  One frame per call: the
    angle -> host cosf/sinf -> descriptor round trip is per frame.  value = frames per wall
    second of whole calls on --ba-threads host threads with their own contexts (late r05; before, the
    kernels' rate, now kernel_frames_per_s)."""
    import torch
    from orb_slam3_comments_ghr_amd import orb
    n_pool = 4
    rng = np.random.default_rng(0x0B5EED30 + rank)
    pool = [orb.synth_orb_frame(rng, n=1200, edge=16) for _ in range(n_pool)]
    pat = _ref_pattern()
    dpool = [(orb.ImagePyramid(f[0]).to_device(dev), orb.ImagePyramid(f[1]).to_device(dev)) + tuple(f[2:])
             for f in pool]
    for f in dpool:
        orb.ORBDescribe(ctx, f[0], f[1], f[2], f[3], f[4], pat)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    reps = max(args.frame_reps, 1) * 50
    k_ms = 0.0
    t0 = time.perf_counter()
    for i in range(reps):
        f = dpool[i % n_pool]
        orb.ORBDescribe(ctx, f[0], f[1], f[2], f[3], f[4], pat)
        k_ms += ctx.last_kernel_ms()
    wall = time.perf_counter() - t0
    k_s, tot = job_totals(k_ms / 1e3, reps, world, dist if world > 1 else None, dev)
    w_s, _ = job_totals(wall, reps, world, dist if world > 1 else None, dev)
    res = {"metric": "frames/s", "value": round(tot / w_s, 1), "unit": "frames/s",
           "workload": "ORBextractor IC_Angle + computeOrbDescriptor: EuRoC-shaped 752x480, 8 levels, 1200 "
                       "keypoints per frame, pyramids in HBM; 1 frame per call (k_orb_angle + k_orb_desc)",
           "kernel_frames_per_s": round(tot / k_s, 1), "kernel_us_per_frame": round(k_ms * 1e3 / reps, 2),
           "wall_frames_per_s_incl_host_roundtrip": round(tot / w_s, 1), "n_gpus": world,
           "scaling": "weak", "parallelism": f"replicas x{world}"}
    T = max(1, args.ba_threads)
    if T > 1:
        res["value"] = res[f"wall_frames_per_s_{T}_host_threads"] = round(_threaded_wall(
            ctx, T, reps, lambda c, i: orb.ORBDescribe(c, *dpool[i % n_pool][:5], pat)), 1)
        res["value_kind"] = f"wall rate of whole calls on {T} host threads"
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = _orb_worker(pool, pat)
        _attach_cpu(res, cpu, 1, "frames/s", args.cpu_seconds * 0.4, "IC_Angle + computeOrbDescriptor",
                    wall_key="wall_frames_per_s_incl_host_roundtrip")
    return res


def bench_orb_detect(ctx, rank, world, dist, dev, args):
    """SURVEY.md §8(f) rank 4 (ORBextractor::ComputeKeyPointsOctTree): FAST per 35-px cell (iniThFAST 20,
    minThFAST 7) and DistributeOctTree down to mnFeaturesPerLevel (1000 features, 8 levels x 1.2) for one
    EuRoC-shaped 752 x 480 frame per call, the pyramid resident in HBM (seeded synthetic images with
    corners at every scale).  value = frames per wall second of the whole call (GPU FAST + per-cell
    suppression, keypoint download, host octree); the kernels' device time is beside it."""
    import torch
    from orb_slam3_comments_ghr_amd import orb
    n_pool = 4
    rng = np.random.default_rng(0x0B5EED31 + rank)
    pool = [orb.synth_fast_pyramid(rng) for _ in range(n_pool)]
    nf, sc = orb.features_per_level(1000, 8, 1.2), orb.scale_factors(8, 1.2)
    dpool = [orb.ImagePyramid(f).to_device(dev) for f in pool]
    for f in dpool:
        orb.ORBDetect(ctx, f, nf, sc)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    reps = max(args.frame_reps, 1) * 50
    k_ms, nk = 0.0, 0
    t0 = time.perf_counter()
    for i in range(reps):
        nk += len(orb.ORBDetect(ctx, dpool[i % n_pool], nf, sc)[0])
        k_ms += ctx.last_kernel_ms()
    wall = time.perf_counter() - t0
    w_s, tot = job_totals(wall, reps, world, dist if world > 1 else None, dev)
    T = max(1, args.ba_threads)
    thr = _threaded_wall(ctx, T, reps, lambda c, i: orb.ORBDetect(c, dpool[i % n_pool], nf, sc)) if T > 1 else tot / w_s
    res = {"metric": "frames/s", "value": round(thr * world, 1), "unit": "frames/s",
           "workload": "ORBextractor::ComputeKeyPointsOctTree: EuRoC-shaped 752x480, 8 levels x 1.2, 1000 features, "
                       f"FAST 20 / 7 per 35 px cell + DistributeOctTree; pyramid in HBM, 1 frame per call, {T} host "
                       "threads with their own contexts",
           "keypoints_per_frame": round(nk / reps, 1),
           "kernel_us_per_frame": round(k_ms * 1e3 / reps, 2),
           "one_thread_frames_per_s": round(tot / w_s, 1),
           "note": "wall rate of the whole call (k_fast_score + k_fast_cells + gather, keypoint download, host octree)",
           "n_gpus": world, "scaling": "weak", "parallelism": f"replicas x{world}"}
    if rank == 0 and world == 1 and not args.no_cpu:
        _attach_cpu(res, _orb_detect_worker(pool, nf, sc), 1, "frames/s", args.cpu_seconds * 0.4,
                    "ComputeKeyPointsOctTree (FAST cells + DistributeOctTree)", wall_key="")
    return res


def bench_orb_extract(ctx, rank, world, dist, dev, args):
    """SURVEY.md §8(f) rank 4, the whole ORBextractor::operator() on the GPU except the final level-0
    scaling of the keypoints (ref:src/ORBextractor.cc:1553-1690): ComputePyramid (8 levels x 1.2 with
    19-px reflect borders) and the per-level 7 x 7 GaussianBlur, ComputeKeyPointsOctTree (1000
    features), IC_Angle and steered BRIEF, for one EuRoC-shaped 752 x 480 image resident in HBM per
    call (seeded synthetic images; the reference's own bit_pattern_31_ BRIEF table).  value = frames
    per wall second of the three calls with --ba-threads host threads on their own contexts."""
    import torch
    from orb_slam3_comments_ghr_amd import orb
    n_pool = 4
    rng = np.random.default_rng(0x0B5EED41 + rank)
    imgs = [orb.synth_fast_pyramid(rng, n_levels=1)[0] for _ in range(n_pool)]
    dimgs = [torch.from_numpy(im).to(dev) for im in imgs]
    inv, sc = orb.inv_scale_factors(8, 1.2), orb.scale_factors(8, 1.2)
    nf = orb.features_per_level(1000, 8, 1.2)
    pattern = _ref_pattern()
    umax = orb.ic_umax()
    lv = np.arange(8, dtype=np.int32)
    torch.cuda.synchronize(dev)
    bufs, stage = {}, {"pyr": 0.0, "det": 0.0, "desc": 0.0}

    def extract(c, i, timed=False):
        P = orb.ComputePyramid(c, dimgs[i % n_pool], inv, out=bufs.get(id(c)), sync=False)
        bufs[id(c)] = P.buffer
        if timed:
            stage["pyr"] += c.last_kernel_ms()
        x, y, _, _, ls = orb.ORBDetect(c, P.raw, nf, sc)
        if timed:
            stage["det"] += c.last_kernel_ms()
        _, d, _ = orb.ORBDescribe(c, P.raw, P.blurred, x, y, np.repeat(lv, np.diff(ls)), pattern, umax)
        if timed:
            stage["desc"] += c.last_kernel_ms()
        return len(x)

    for i in range(n_pool):
        extract(ctx, i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    reps = max(args.frame_reps, 1) * 50
    nk = 0
    t0 = time.perf_counter()
    for i in range(reps):
        nk += extract(ctx, i, timed=True)
    wall = time.perf_counter() - t0
    w_s, tot = job_totals(wall, reps, world, dist if world > 1 else None, dev)
    T = max(1, args.ba_threads)
    thr = _threaded_wall(ctx, T, reps, extract) if T > 1 else tot / w_s
    # the batched entry: B images per osg_orb_extract_batch call, one host thread
    B = 64
    batch = torch.stack([dimgs[i % n_pool] for i in range(B)])
    for _ in range(2):
        orb.ORBExtractBatch(ctx, batch, pattern=pattern, umax=umax)  # syncs torch's stack first
    torch.cuda.synchronize(dev)
    breps = max(args.frame_reps, 1) * 4
    nkb = 0
    t0 = time.perf_counter()
    for _ in range(breps):
        nkb += int(orb.ORBExtractBatch(ctx, batch, pattern=pattern, umax=umax, sync=False).counts.sum())
    bwall = time.perf_counter() - t0
    bw_s, btot = job_totals(bwall, breps * B, world, dist if world > 1 else None, dev)
    res = {"metric": "frames/s", "value": round(btot / bw_s, 1), "unit": "frames/s",
           "workload": "ORBextractor::operator(): EuRoC-shaped 752x480 images in HBM -> ComputePyramid (8 x 1.2) + "
                       "GaussianBlur 7x7 -> FAST + DistributeOctTree (1000 features) -> IC_Angle + rBRIEF; "
                       f"{B} frames per osg_orb_extract_batch call, one host thread",
           "keypoints_per_frame": round(nkb / (breps * B), 1),
           "ms_per_batch_call": round(bwall * 1e3 / breps, 2),
           "per_frame_calls": {"frames_per_s_one_thread": round(tot / w_s, 1),
                               f"frames_per_s_{T}_host_threads": round(thr * world, 1),
                               "keypoints_per_frame": round(nk / reps, 1),
                               "kernel_us_per_frame": {k: round(v * 1e3 / reps, 2) for k, v in stage.items()},
                               "note": "three calls per frame (osg_orb_pyramid, osg_orb_detect, osg_orb_describe) "
                                       "incl. keypoint downloads and the host octree"},
           "note": "wall rate of the batched call incl. the per-image keypoint downloads, the host octrees of "
                   "all (image, level) pairs on up to 16 threads, and the descriptor download",
           "n_gpus": world, "scaling": "weak", "parallelism": f"replicas x{world}"}
    if rank == 0 and world == 1 and not args.no_cpu:
        _attach_cpu(res, _orb_extract_worker(imgs, inv, nf, sc, pattern, umax), 1, "frames/s",
                    args.cpu_seconds * 0.4, "ComputePyramid + GaussianBlur + ComputeKeyPointsOctTree + "
                    "IC_Angle + rBRIEF", wall_key="")
    return res


def _orb_extract_worker(imgs, inv, nf, sc, pattern, umax):
    """cpu_baseline worker for the whole extractor: one pool image per call through the oracle."""
    n_pool = len(imgs)

    def cpu(tid):
        from tests import oracle_calls as oc
        oracle, _ = _oracle()
        lv = np.arange(8, dtype=np.int32)

        def one(i):
            buf, lr, lc, bo, bl = oc.orb_pyramid(oracle, imgs[i % n_pool], inv)
            _, roi, blurred = oc.pyramid_levels(buf, lr, lc, bo, bl)
            x, y, _, _, ls = oc.orb_detect(oracle, roi, nf, sc, cap=8192)
            oc.orb_describe(oracle, roi, blurred, x, y, np.repeat(lv, np.diff(ls)), pattern, umax)
        return one
    return cpu


def _orb_detect_worker(pool, nf, sc):
    """cpu_baseline worker for ComputeKeyPointsOctTree: one pool pyramid per call through the oracle."""
    n_pool = len(pool)

    def cpu(tid):
        import ctypes as C
        from orb_slam3_comments_ghr_amd.stereo import ImagePyramid
        oracle, _ = _oracle()
        cap = 8192
        items = []
        for f in pool:
            P = ImagePyramid(f)
            ps = P.struct()
            outs = [np.zeros(cap, np.float32) for _ in range(4)] + [np.zeros(len(f) + 1, np.int32)]
            items.append(((C.byref(ps), 20, 7, nf.ctypes.data, sc.ctypes.data, cap) +
                          tuple(o.ctypes.data for o in outs), (P, ps, outs)))
        keep = (nf, sc, items)
        fn = oracle.oracle_orb_detect
        return lambda i, keep=keep: fn(*items[i % n_pool][0])
    return cpu


def _c3_worker(pairs, probs):
    """cpu_baseline worker for C3: SearchByBoW(KF,F) + PoseOptimization of one pool frame per call."""
    n_pool = len(pairs)

    def cpu(tid):  # the cpu_baseline leg: the oracle restatement, arguments packed per thread
        import ctypes as C
        from orb_slam3_comments_ghr_amd import _abi
        oracle, _ = _oracle()
        bow = [(p[0].struct(), p[1].struct()) for p in pairs]
        outs = [np.full(p[1].n, -1, np.int32) for p in pairs]
        pst = [p.struct() for p in probs]
        res = (_abi.OsgPoseResult * n_pool)()
        outl = [np.zeros(p.n, np.uint8) for p in probs]
        for r, o in zip(res, outl):
            r.outlier = o.ctypes.data
        args_ = [(C.byref(a), C.byref(b), o.ctypes.data, C.byref(ps), C.byref(r))
                 for (a, b), o, ps, r in zip(bow, outs, pst, res)]
        keep = (bow, outs, pst, res, outl)
        fb, fp = oracle.oracle_search_by_bow_kf_f, oracle.oracle_pose_optimization

        def call(i, keep=keep):
            a, b, o, ps, r = args_[i % n_pool]
            fb(a, b, 0.7, 1, o)
            fp(ps, r)
        return call
    return cpu


def _c5_worker(F, L, Q, S, probs):
    """cpu_baseline worker for C5: SearchByProjection(F,LastF) + (F,local map) + PoseOptimization."""
    n_pool = len(F)

    def cpu(tid):  # the cpu_baseline leg: the oracle restatement, arguments packed per thread
        import ctypes as C
        from orb_slam3_comments_ghr_amd import _abi
        oracle, _ = _oracle()
        fs = [f.struct() for f in F]
        ls = [x.struct() for x in L]
        qs = [x.struct() for x in Q]
        slot = [S[i][0].copy() for i in range(n_pool)]
        taken = [np.ascontiguousarray(S[i][1], np.uint8) for i in range(n_pool)]
        pst = [p.struct() for p in probs]
        res = (_abi.OsgPoseResult * n_pool)()
        outl = [np.zeros(p.n, np.uint8) for p in probs]
        for r, o in zip(res, outl):
            r.outlier = o.ctypes.data
        args_ = [(C.byref(fs[i]), C.byref(ls[i]), C.byref(qs[i]), slot[i], S[i][0], slot[i].ctypes.data,
                  taken[i].ctypes.data, C.byref(pst[i]), C.byref(res[i])) for i in range(n_pool)]
        keep = (fs, ls, qs, slot, taken, pst, res, outl)
        fl, fm, fp = (oracle.oracle_search_by_projection_last, oracle.oracle_search_by_projection_mps,
                      oracle.oracle_pose_optimization)

        def call(i, keep=keep):
            f, lq, mq, sl, s0, sp, tp, ps, r = args_[i % n_pool]
            np.copyto(sl, s0)  # both searches start from the frame's slot state, as in the GPU batch
            fl(f, lq, 7.0, 0, 1, sp, tp)
            np.copyto(sl, s0)
            fm(f, mq, 0.9, 3.0, 0, 20.0, sp, tp)
            fp(ps, r)
        return call
    return cpu


def _dbow_worker(voc, pool):
    """cpu_baseline worker for DBoW2 transform: the whole pool (16 frames) per call."""
    from orb_slam3_comments_ghr_amd import vocabulary as vb
    n_pool = len(pool)

    def cpu(tid):  # the cpu_baseline leg: the oracle, children index built once per 16 frames
        import ctypes as C
        from orb_slam3_comments_ghr_amd._abi import OsgBowOut
        oracle, _ = _oracle()
        sets_ = [np.ascontiguousarray(d, np.uint8).reshape(-1, 32) for d in pool]
        outs = [vb.make_bow_out(d.shape[0]) for d in sets_]
        arr = (OsgBowOut * n_pool)(*[o for o, _ in outs])
        n = np.array([d.shape[0] for d in sets_], np.int32)
        cat = np.concatenate(sets_)
        vs = voc.struct()
        a = (C.byref(vs), cat.ctypes.data, n.ctypes.data, n_pool, 4, C.addressof(arr))
        keep = (sets_, outs, arr, n, cat, vs)
        fn = oracle.oracle_dbow_transform_batch
        return lambda i, keep=keep: fn(*a)
    return cpu


def _stereo_worker(pool):
    """cpu_baseline worker for ComputeStereoMatches: one pool frame per call."""
    n_pool = len(pool)

    def cpu(tid):  # the cpu_baseline leg: the oracle restatement, arguments packed per thread
        import ctypes as C
        oracle, _ = _oracle()
        ss = [f.struct() for f in pool]
        outs = [(np.empty(f.n, np.float32), np.empty(f.n, np.float32)) for f in pool]
        args_ = [(C.byref(s_), u.ctypes.data, d.ctypes.data) for s_, (u, d) in zip(ss, outs)]
        keep = (ss, outs)
        fn = oracle.oracle_compute_stereo_matches
        return lambda i, keep=keep: fn(*args_[i % n_pool])
    return cpu


def _orb_worker(pool, pat):
    """cpu_baseline worker for IC_Angle + computeOrbDescriptor: one pool frame per call."""
    from orb_slam3_comments_ghr_amd import orb
    n_pool = len(pool)

    def cpu(tid):  # IC_Angle + computeOrbDescriptor through the oracle, arguments packed per thread
        import ctypes as C
        from orb_slam3_comments_ghr_amd._abi import OsgOrbKeypoints
        from orb_slam3_comments_ghr_amd.stereo import ImagePyramid
        oracle, _ = _oracle()
        umax = orb.ic_umax()
        patf = np.ascontiguousarray(pat, np.int32).reshape(-1)
        items = []
        for f in pool:
            rp, bp = ImagePyramid(f[0]), ImagePyramid(f[1])
            x, y = (np.ascontiguousarray(v, np.float32) for v in (f[2], f[3]))
            lv = np.ascontiguousarray(f[4], np.int32)
            K = OsgOrbKeypoints(len(x), x.ctypes.data, y.ctypes.data, lv.ctypes.data)
            ang, desc = np.zeros(len(x), np.float32), np.zeros((len(x), 32), np.uint8)
            rs, bs = rp.struct(), bp.struct()
            items.append(((C.byref(rs), C.byref(bs), C.byref(K), patf.ctypes.data, umax.ctypes.data, 1,
                           ang.ctypes.data, desc.ctypes.data), (rp, bp, x, y, lv, K, ang, desc, rs, bs)))
        keep = (umax, patf, items)
        fn = oracle.oracle_orb_describe
        return lambda i, keep=keep: fn(*items[i % n_pool][0])
    return cpu


def cpu_baseline(q_np, t_np, seconds):
    """oracle_hamming_top2 (the reference's serial DescriptorDistance + top-2 loop, restated in C, -O3),
    one whole 2000 x 2000 frame per host thread, on 1 thread and on every CPU this job may use."""
    lib, _ = _oracle()
    from tests import cpu_mt
    nq, nt = q_np.shape[0], t_np.shape[0]
    qp, tp = q_np.ctypes.data, t_np.ctypes.data

    def worker(tid):
        out = [np.empty(nq, np.int32) for _ in range(3)]
        ptrs = [o.ctypes.data for o in out]
        fn = lib.oracle_hamming_top2
        return lambda i, out=out: fn(qp, nq, tp, nt, *ptrs)

    return cpu_mt.baseline(worker, nq * nt / 1e6, "Mmatches/s", seconds, f"C2 {nq}x{nt} top-2 (oracle_hamming_top2)")


if __name__ == "__main__":
    main()
