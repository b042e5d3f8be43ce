#!/usr/bin/env python3
"""bench.py — BASELINE.json's metric: frames/s of ORB extract + match on 640x480 frames.

A step = one pass of the hot path over one batch of B synthetic 640x480 frames resident in
HBM: ORBextractor(1000, 1.2, 8, FAST, 20) on all B frames (orb_extract_batch_device), then
ORBmatcher(0.9, true).SearchForInitialization(F_t, F_t+1, window 100) on the B-1
consecutive pairs (orb_search_for_initialization_batch_device), on one stream.  --overlap 1
runs the steps as a two-stage stream pipeline instead (step t extracts batch t while batch t-1
is matched on a second stream; the serial step is then reported beside it as "serial_step"):
measured equal to the serial step on MI355X (1.80 vs 1.79 ms), so it is off by default.
N GPUs run N independent
replicas (frames shard one stream per GPU; no collectives on the data path); value is the
whole-job frames/s = N * B * K / max-over-ranks(time of K steps).

Also reported:
  roofline      dominant kernel: algorithmic bytes per launch / mean launch duration, from
                HIP events recorded around that stage on its launch stream inside the timed
                region (an untimed survey pass brackets every stage to find it and to fill the
                per-stage table; each event pair costs a ~10 us stream boundary).
  pipeline      whole-path algorithmic bytes (SURVEY.md §8d B_ext + B_match) / wall time.
  cpu_baseline  the CPU oracle (C++ restatement, oracle/) on the host cores, rank 0 only,
                on a bounded sample of the same frames.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md §Chip-level parameters)


def level_sizes(W, H, nlevels=8, scale=1.2):
    """(w_l, h_l) exactly as ComputePyramid (ORBextractor.cc:783-786)."""
    inv = [np.float32(1.0)]
    f = np.float32(np.float32(1.0) / np.float64(np.float32(scale)))
    for _ in range(1, nlevels):
        inv.append(np.float32(inv[-1] * f))
    out = []
    for s in inv:
        out.append((int(np.rint(np.float64(np.float32(W) * s))), int(np.rint(np.float64(np.float32(H) * s)))))
    return out


def stage_bytes(W, H, n_kp, n_cand, n_pairs_kp0, B):
    """Algorithmic HBM bytes per launch of each stage for a batch of B frames.

    n_kp: total keypoints of the batch; n_cand: total FAST survivors; n_pairs_kp0: sum over
    pairs of (n1_0 + n2_0) level-0 keypoints.  Definitions in DESIGN.md §Roofline.
    """
    lv = level_sizes(W, H)
    pad = [(w + 32) * (h + 32) for w, h in lv]
    px = [w * h for w, h in lv]
    return {
        "k_pyr0": B * (W * H + pad[0]),
        "k_pyr_resize": B * sum(px[l - 1] + pad[l] for l in range(1, len(lv))) / (len(lv) - 1),  # per launch
        # blur + FAST: read the level with its 3/4 px halo once, write the blurred ROI + border
        "k_level": B * sum(2 * (w + 8) * (h + 6) for w, h in lv),
        # read the level corner lists (>= survivors), write the cell candidates
        "k_cell_nms": 8 * n_cand,
        "k_select": 8 * n_cand + 4 * n_kp,
        "k_orient_desc": n_kp * (4 + 31 * 31 + 512 + 60),
    }


def pmc_traffic(kernel, W, H, B, NF):
    """HBM bytes per launch of `kernel` from the committed PMC summary of this workload
    (profiles/pmc_latest.json, written by scripts/pmc_summary.py from rocprofv3 FETCH_SIZE /
    WRITE_SIZE passes over bench.py) with the source tag and the kernel's SQ_INSTS_VALU (wave
    instructions per launch), or Nones when the summary does not cover this run."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_latest.json")) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None, None
    w = d.get("workload", {})
    if (w.get("width"), w.get("height"), w.get("batch"), w.get("nfeatures")) != (W, H, B, NF):
        return None, None, None
    k = d.get("per_launch", {}).get(kernel)
    return (k["hbm_bytes"], d.get("source"), k.get("SQ_INSTS_VALU")) if k else (None, None, None)


def cpu_baseline(frames, nfeatures, threads, W, H):
    """Oracle (test infrastructure, oracle/liborb_oracle.so) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes

    from oracle_lib import lib

    L = lib()
    fr = np.ascontiguousarray(frames)
    k = ctypes.c_int64()
    m = ctypes.c_int64()
    L.oracle_bench(nfeatures, 1.2, 8, 20, fr[:8].ctypes.data_as(ctypes.c_void_p), min(8, len(fr)), W, H, W, W * H,
                   threads, 1, ctypes.byref(k), ctypes.byref(m))  # warm-up
    dt = L.oracle_bench(nfeatures, 1.2, 8, 20, fr.ctypes.data_as(ctypes.c_void_p), len(fr), W, H, W, W * H, threads,
                        1, ctypes.byref(k), ctypes.byref(m))
    if dt <= 0:
        raise RuntimeError("oracle_bench failed")
    return len(fr) / dt, dt, int(k.value), int(m.value)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=512, help="frames per step per GPU")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--nfeatures", type=int, default=1000)
    ap.add_argument("--cpu-frames", type=int, default=3072,
                    help="CPU-baseline sample size (0 = skip); ~20 s of CPU-thread time on 16 threads")
    ap.add_argument("--overlap", type=int, default=0,
                    help="1: extract(t) on one stream while matching batch t-1 on another; 2: only the "
                         "pyramid of batch t overlaps the matching of batch t-1; 0: serial step")
    ap.add_argument("--survey-steps", type=int, default=5, help="untimed steps with every stage bracketed")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = OMP_NUM_THREADS or os.cpu_count()")
    args = ap.parse_args()
    args.survey_steps = max(1, args.survey_steps)

    import orbslam_jpminipc_amd as orb
    from orbslam_jpminipc_amd import replicas

    info = replicas.init_from_env("nccl")
    world, rank, local = info.world, info.rank, info.local_rank
    torch.cuda.set_device(local)

    W, H, B, NF = args.width, args.height, args.batch, args.nfeatures
    frames = orb.synth_stream(W, H, stream=rank, first=0, count=B)
    d_imgs = torch.from_numpy(frames).cuda()
    ext = orb.ORBextractor(NF, 1.2, 8, orb.FAST_SCORE, 20, device=local, max_batch=B)
    matcher = orb.ORBmatcher(0.9, True)
    cap = ext.max_keypoints
    d_kps = torch.empty((B, cap, 28), dtype=torch.uint8, device="cuda")
    d_desc = torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda")
    d_cnt = torch.empty((B,), dtype=torch.int32, device="cuda")
    f1 = torch.arange(0, B - 1, dtype=torch.int32, device="cuda")
    f2 = f1 + 1
    # serial mode: one stream carries the whole step, extraction then the matching that reads
    # its output.  overlap mode (default): a two-stage stream pipeline over consecutive batches —
    # step t extracts batch t on s_ext while s_match runs SearchForInitialization on batch t-1
    # (double-buffered outputs, event-ordered); every step still does B extractions and B-1
    # pair matches, so steps/s is the same work rate.
    s_ext = torch.cuda.Stream()
    s_match = torch.cuda.Stream()
    torch.cuda.current_stream().synchronize()  # inputs uploaded on the default stream
    bufs = [(d_kps, d_desc, d_cnt),
            (torch.empty_like(d_kps), torch.empty_like(d_desc), torch.empty_like(d_cnt))]
    ev_edone = [torch.cuda.Event(), torch.cuda.Event()]
    ev_mdone = [torch.cuda.Event(), torch.cuda.Event()]
    ev_m = []
    st = {"t": 0, "overlap": False}

    def match(kps, desc, cnt, stream, timed):
        if timed:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
        m12, nm = matcher.search_for_initialization_batch_device(kps, desc, cnt, f1, f2, W, H, 100, stream=stream)
        if timed:
            b.record(stream)
            ev_m.append((a, b))
        return nm

    def step(timed=False):
        if not st["overlap"]:
            with torch.cuda.stream(s_ext):
                ext.extract_batch_device(d_imgs, d_kps, d_desc, d_cnt, stream=s_ext)
                return match(d_kps, d_desc, d_cnt, s_ext, timed)
        t = st["t"]
        st["t"] += 1
        cur, prev = t % 2, (t - 1) % 2
        if st["overlap"] == 2:
            # pyramid(t) || match(t-1); detection..descriptors of t after match(t-1), so the
            # matcher's LDS-heavy work-groups never share the chip with k_level's
            with torch.cuda.stream(s_ext):
                ext.set_phases(1)
                ext.extract_batch_device(d_imgs, *bufs[cur], stream=s_ext)
            nm = None
            if t >= 1:
                with torch.cuda.stream(s_match):
                    s_match.wait_event(ev_edone[prev])
                    nm = match(*bufs[prev], s_match, timed)
                    ev_mdone[prev].record(s_match)
                s_ext.wait_event(ev_mdone[prev])  # also: match(t-2) has read bufs[cur]
            with torch.cuda.stream(s_ext):
                ext.set_phases(2)
                ext.extract_batch_device(d_imgs, *bufs[cur], stream=s_ext)
                ext.set_phases(3)
                ev_edone[cur].record(s_ext)
            return nm
        with torch.cuda.stream(s_ext):
            if t >= 2:
                s_ext.wait_event(ev_mdone[cur])  # match(t-2) has read this buffer
            ext.extract_batch_device(d_imgs, *bufs[cur], stream=s_ext)
            ev_edone[cur].record(s_ext)
        nm = None
        if t >= 1:
            with torch.cuda.stream(s_match):
                s_match.wait_event(ev_edone[prev])
                nm = match(*bufs[prev], s_match, timed)
                ev_mdone[prev].record(s_match)
        return nm

    def timed_run(overlap, time_match):
        st["overlap"], st["t"] = overlap, 0
        if overlap:
            step()  # fill the pipeline: batch 0 extracted, its match runs in the first timed step
        torch.cuda.synchronize()
        replicas.barrier(info)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            nm = step(timed=time_match)
        torch.cuda.synchronize()
        replicas.barrier(info)
        return time.perf_counter() - t0, nm

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # stage survey (untimed, serial): an event pair around every stage gives the per-stage
    # table; each pair is a stream boundary (~10 us), so the timed run below brackets only the
    # dominant stage
    ext.profile_enable(True)
    for _ in range(args.survey_steps):
        step(timed=True)
    torch.cuda.synchronize()
    survey = ext.profile_read()
    ext.profile_enable(False)
    survey["k_match_init"] = (sum(a.elapsed_time(b) for a, b in ev_m), len(ev_m))
    ev_m.clear()
    dom = max(survey, key=lambda k: survey[k][0])
    time_match = dom == "k_match_init"
    if args.overlap:  # the serial step, for reference (no events)
        serial_elapsed, _ = timed_run(False, False)
        serial_tmax = replicas.max_over_ranks(serial_elapsed, info)
    if not time_match:
        ext.profile_enable_stages([dom])
    elapsed, nm = timed_run(args.overlap, time_match)
    if time_match:
        live = (sum(a.elapsed_time(b) for a, b in ev_m), len(ev_m))
    else:
        live = ext.profile_read()[dom]
        ext.profile_enable(False)
    prof = dict(survey)
    prof[dom] = live  # the dominant stage: measured inside the timed region

    tmax = replicas.max_over_ranks(elapsed, info)

    # workload statistics of the last step (identical every step: same frames)
    cnt = d_cnt.cpu().numpy().astype(np.int64)
    kps_h = d_kps.cpu().numpy()
    oct0 = np.array([int((orb.keypoints_from_bytes(kps_h[b], cnt[b])["octave"] == 0).sum()) for b in range(B)])
    n_kp = int(cnt.sum())
    nm_h = nm.cpu().numpy()
    n_cand = int(n_kp * 3)  # refined below from the FAST survivors when available
    try:
        import ctypes

        lib = orb.hip_lib()
        tot = 0
        buf = np.zeros(4096, np.int32)
        for b in range(B):
            for l in range(8):
                n = lib.orb_debug_cell_counts(ext._h, b, l, buf.ctypes.data_as(ctypes.c_void_p), 4096)
                tot += int(buf[:n].sum())
        n_cand = tot
    except Exception:
        pass
    pairs_kp0 = int(sum(oct0[p] + oct0[p + 1] for p in range(B - 1)))
    sb = stage_bytes(W, H, n_kp, n_cand, pairs_kp0, B)
    lv = level_sizes(W, H)
    px = [w * h for w, h in lv]
    b_ext = B * (sum(px) + sum(px[1:])) + 60 * n_kp
    b_match = 32 * pairs_kp0 + 20 * int(sum(cnt[:-1]))
    sb["k_match_init"] = b_match
    stages = {}
    for name, (ms, launches) in prof.items():
        if launches == 0:
            continue
        per_launch_ms = ms / launches
        nbytes = sb.get(name, 0)
        stages[name] = {
            "ms_per_launch": per_launch_ms,
            "launches": launches,
            "bytes_per_launch": nbytes,
            "GBps": nbytes / (per_launch_ms * 1e-3) / 1e9 if per_launch_ms > 0 else None,
            "measured_in": "timed region" if name == dom else "survey pass",
        }
    # the resize stage builds levels 1-7 (k_pyr_resize per large level, the small levels in one
    # k_pyr_resize_tail launch): report per-level numbers
    if "k_pyr_resize" in stages:
        s = stages["k_pyr_resize"]
        s["launches"] *= 7
        s["ms_per_launch"] /= 7
        s["GBps"] = s["bytes_per_launch"] / (s["ms_per_launch"] * 1e-3) / 1e9
        s["note"] = "per pyramid level (levels 1-7; the small levels share one k_pyr_resize_tail launch)"
    ds = stages[dom]
    per_step_s = tmax / args.steps

    value = replicas.whole_job_rate(B * args.steps, world, tmax)
    traffic, traffic_src, valu_insts = pmc_traffic(dom, W, H, B, NF)
    # VALU issue ceiling: each SIMD issues one wave64 VALU instruction per 2 cycles
    # (MI355X_MICROARCH.md), 4 SIMDs x 256 CUs at 2.4 GHz
    valu_peak = 256 * 4 / 2 * 2.4e9
    result = {
        "metric": "frames/sec ORB extract+match, 640x480 8-level 1000 kp; HBM GB/s vs peak",
        "value": value,
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": per_step_s * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (csrc/synth.c: rectangles+discs+noise, consecutive frames shifted)",
        "config": {
            "workload": f"{W}x{H} frames, ORBextractor({NF},1.2,8,FAST,20) + SearchForInitialization(t,t+1) "
                        f"nnratio 0.9 checkOri window 100 (BASELINE.json configs[1]+[2])",
            "batch_per_gpu": B,
            "pairs_per_gpu": B - 1,
            "parallelism": f"replicas x{world} (no collectives)",
            "streams": {0: "one stream, extract then match",
                        1: "extract(t) || SearchForInitialization(t-1), double-buffered",
                        2: "pyramid(t) || SearchForInitialization(t-1), then the rest of extract(t)"}
                       [args.overlap],
        },

        "roofline": {
            "kernel": dom,
            "bound": "hbm",
            "achieved": ds["GBps"],
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": ds["GBps"] / HBM_PEAK_GBS if ds["GBps"] else None,
            "traffic": traffic,
            "traffic_unit": "bytes per launch (rocprofv3 PMC)",
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": ds["bytes_per_launch"],
            "valu_insts_per_launch": valu_insts,
            "valu_issue_frac": (valu_insts / (ds["ms_per_launch"] * 1e-3) / valu_peak) if valu_insts else None,
        },
        "pipeline": {
            "algorithmic_bytes_per_step": b_ext + b_match,
            "GBps": (b_ext + b_match) / per_step_s / 1e9,
            "frac": (b_ext + b_match) / per_step_s / 1e9 / HBM_PEAK_GBS,
        },
        "stages": stages,
        "workload_stats": {"keypoints_per_frame": n_kp / B, "fast_survivors_per_frame": n_cand / B,
                           "matches_per_pair": float(nm_h.mean())},
    }
    if args.overlap:
        result["serial_step"] = {"value": replicas.whole_job_rate(B * args.steps, world, serial_tmax),
                                 "ms_per_step": serial_tmax / args.steps * 1e3}
    if rank == 0 and world == 1 and args.cpu_frames > 0:
        threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0") or os.cpu_count())
        ncpu = args.cpu_frames
        cpu_frames = orb.synth_stream(W, H, stream=0, first=0, count=ncpu)
        fps, dt, _, _ = cpu_baseline(cpu_frames, NF, threads, W, H)
        result["cpu_baseline"] = {
            "value": fps,
            "unit": "frames/s",
            "cores": threads,
            "kind": "port",
            "sample": f"{ncpu} frames extract + {ncpu - 1} consecutive-pair SearchForInitialization, "
                      f"{dt:.2f} s wall on {threads} threads (C++ restatement oracle, -O3)",
        }
    if rank == 0:
        print(json.dumps(result))
    replicas.shutdown(info)


if __name__ == "__main__":
    main()
