#!/usr/bin/env python3
"""bench.py — BASELINE.json's metric: frames/s of ORB extract + match, with HBM GB/s vs peak.

A step = one pass of the hot path over one batch of synthetic frames resident in HBM:
ORBextractor(nfeatures, 1.2, 8, FAST, 20) on all B frames of the rank (orb_extract_batch_device),
then ORBmatcher(0.9, true).SearchForInitialization(F_t, F_t+1, window 100) on every pair of
consecutive frames of the same camera stream (orb_search_for_initialization_batch_device), both
on one stream.  value = whole-job frames/s = (frames of all ranks per step) * K / max-over-ranks
(time of K steps).

Workloads (--workload; BASELINE.json configs):
  c3  (default) configs[1]+[2]: 640x480, 1000 kp, B = 512 frames of camera stream `rank` per
      GPU (weak scaling: every rank its own stream)
  c4  configs[3]: KITTI-shaped 1241x376, 2000 kp, B = 512 frames of stream `rank` per GPU
  c5  configs[4]: 8 independent 1280x720 camera streams, 2500 kp; stream s runs on rank
      s mod N, --frames-per-stream frames of each per step (strong scaling:
      the 8 streams are the whole job)

Multi-GPU = replicas only (frames are independent, matching pairs frames of one
stream; no data-path collective).  `python bench.py --gpus N` spawns N rank processes itself
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 set before any GPU call, one per
GPU); under torch.distributed.run the ranks come from the environment.  The only collectives
are the barriers around the timed region, the max over ranks of its duration and a gather of
the per-rank durations (rank_seconds).

Also reported:
  roofline      dominant kernel: SURVEY.md §8d algorithmic bytes of its stage per launch / mean
                launch duration, from HIP events recorded around that stage on its launch stream
                inside the timed region; traffic = PMC-measured HBM bytes per launch of the same
                kernel (profiles/pmc_<workload>.json, rocprofv3 FETCH_SIZE / WRITE_SIZE passes)
  pipeline      whole-path algorithmic bytes (§8d B_ext + B_match) / step time
  latency_b1    the per-frame path the reference calls (Frame.cc:60, Tracking.cc:392-393): one
                host frame through orb_extract, one frame pair through the host
                SearchForInitialization, one device frame through orb_extract_batch_device; the
                single-thread CPU oracle beside each (rank 0, N = 1)
  host_fed      the same step fed from pinned host memory and returned to it (the operator()
                boundary: ORBextractor.h:43-45), H2D / compute / D2H overlapped on three streams;
                frames/s with the PCIe GB/s achieved each way and the link's measured ceiling
                (rank 0, N = 1; never `value`)
  bow           the BoW-bucketed matching path on the step's output: vocabulary transform
                (Frame::ComputeBoW, levelsup 4, ORBvoc-shaped tree) of every frame + batched
                SearchByBoW(KF = frame t, F = frame t+1), per-stage ms, pairs/s, rooflines (rank 0,
                N = 1; never `value`)
  cpu_baseline  the CPU oracle (C++ restatement, oracle/) on the host cores, rank 0, N = 1, on a
                bounded sample of the same frames: extract-only and extract+match frames/s on all
                threads and on the cgroup quota's thread count (value = the better of the two,
                with its thread count), single-thread ms/frame, CPU model
--overlap 1 / 2 are measured-slower stream-overlap experiments; the default (0)
is the serial step.  --dry-run runs the launcher and rank plumbing on CPU (gloo, the oracle as
the per-rank workload) for the multi-process tests.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md §Chip-level parameters)
N_CU, CLOCK_HZ = 256, 2.4e9
SALU_PEAK = N_CU * CLOCK_HZ  # SALU instructions / s: one scalar unit per CU, one issue per cycle
LDS_PEAK = N_CU * CLOCK_HZ   # LDS pipe cycles / s: one per CU per cycle
# Measured VALU issue rate of the 4-cycle instruction kinds (v_perm, v_pk_*, v_alignbyte, v_bfe,
# v_dot*, v_mul_*24, v_min/max_u32, DPP moves, 3-source VOP3) with 8 waves per SIMD, all CUs busy:
# 0.58 wave64 instructions per ns per SIMD (scripts/gen_valu_rate.py, profiles/r05_valu_rate.json;
# add / and / or / shift / f32 fma reach 1.08 alone, but a 1:1 mix with a 4-cycle kind runs 0.61)
VALU_4C_PEAK = N_CU * 4 * 0.58e9
METRIC = "frames/sec ORB extract+match, 640x480 8-level 1000 kp; HBM GB/s vs peak"

WORKLOADS = {
    "c3": dict(W=640, H=480, nf=1000, streams=0,
               label="BASELINE.json configs[1]+[2]: batched 640x480 frames, ORBextractor(1000,1.2,8,FAST,20) + "
                     "SearchForInitialization(t,t+1) nnratio 0.9 checkOri window 100"),
    "c4": dict(W=1241, H=376, nf=2000, streams=0,
               label="BASELINE.json configs[3]: KITTI-shaped 1241x376 frames, ORBextractor(2000,1.2,8,FAST,20) + "
                     "SearchForInitialization(t,t+1) nnratio 0.9 checkOri window 100"),
    "c5": dict(W=1280, H=720, nf=2500, streams=8,
               label="BASELINE.json configs[4]: 8 independent 1280x720 streams (stream s on GPU s mod N), "
                     "ORBextractor(2500,1.2,8,FAST,20) + SearchForInitialization(t,t+1) within each stream"),
}


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


def stage_bytes(W, H, n_kp, B):
    """SURVEY.md §8d algorithmic bytes per launch of each extraction stage for B frames:
    B_ext = sum_l w_l h_l (each level read once) + sum_{l>=1} w_l h_l (each derived level
    written once) + 60 N_kp (keypoint + descriptor records written), split over the stages
    that carry each term: the level-0 input read by k_pyr0, the derived levels written by the
    resize stage (per launch: per level), every level read by k_fast (detection), the records
    written by k_orient_desc.  Nothing else counts (padding, intermediates, re-reads)."""
    lv = level_sizes(W, H)
    px = [w * h for w, h in lv]
    return {
        "k_pyr0": B * px[0],
        "k_pyr_resize": B * sum(px[1:]) / (len(lv) - 1),
        "k_fast": B * sum(px),
        "k_select": 0,
        "k_orient_desc": 60 * n_kp,
    }


def pmc_traffic(kernel, workload, W, H, B, NF):
    """HBM bytes per launch of `kernel` from the committed PMC summary of this workload
    (profiles/pmc_<workload>.json, scripts/pmc_summary.py over rocprofv3 FETCH_SIZE /
    WRITE_SIZE passes of this bench), with the source tag and the kernel's SQ_INSTS_VALU, or
    Nones when no summary covers this exact run shape."""
    try:
        with open(os.path.join(ROOT, "profiles", f"pmc_{workload}.json")) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None, None
    w = d.get("workload", {})
    if (w.get("width"), w.get("height"), w.get("batch"), w.get("nfeatures")) != (W, H, B, NF):
        return None, None, None
    k = d.get("per_launch", {}).get(kernel)
    return (k["hbm_bytes"], d.get("source"), k) if k else (None, None, None)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpus():
    """What this process may run on: the affinity set (the threads the CPU baseline uses by
    default), the machine's logical CPU count, the cgroup v2 CPU quota (cpu.max, in CPUs; None
    when unlimited or absent) and OMP_NUM_THREADS as set by the environment."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    return {"affinity": affinity, "logical_cpus": os.cpu_count(), "cgroup_cpu_quota": quota,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def physical_cores():
    """Physical cores of the machine from /proc/cpuinfo (distinct (physical id, core id))."""
    cores, phys = set(), "0"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":", 1)[1].strip()
            elif line.startswith("core id"):
                cores.add((phys, line.split(":", 1)[1].strip()))
    except OSError:
        pass
    return len(cores) or None


def cpu_baseline(frames, nfeatures, threads, W, H, quota_threads=None):
    """Oracle (test infrastructure, oracle/liborb_oracle.so) on a bounded sample: extract-only
    and extract+match frames/s on `threads` threads (and on `quota_threads` threads, when the
    cgroup caps CPU time below the affinity set), single-thread ms/frame."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes

    from oracle_lib import lib

    L = lib()
    fr = np.ascontiguousarray(frames)
    k = ctypes.c_int64()
    m = ctypes.c_int64()
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731

    def run(sample, nthreads, match):
        dt = L.oracle_bench(nfeatures, 1.2, 8, 20, vp(sample), len(sample), W, H, W, W * H, nthreads, match,
                            ctypes.byref(k), ctypes.byref(m))
        if dt <= 0:
            raise RuntimeError("oracle_bench failed")
        return dt

    run(fr[:16], threads, 1)  # warm-up
    t_ext = run(fr, threads, 0)
    t_all = run(fr, threads, 1)
    n1 = min(len(fr), 48)
    t_one = run(fr[:n1], 1, 0)
    t_one_m = run(fr[:n1], 1, 1)
    extra = {}
    if quota_threads and quota_threads < threads:
        tq = run(fr, quota_threads, 1)
        extra = {"quota_threads": quota_threads, "quota_threads_extract_match_fps": len(fr) / tq}
    return {
        **extra,
        "extract_fps": len(fr) / t_ext,
        "extract_match_fps": len(fr) / t_all,
        "single_thread_ms_per_frame_extract": t_one / n1 * 1e3,
        "single_thread_ms_per_frame_extract_match": t_one_m / n1 * 1e3,
        "sample_frames": len(fr),
        "single_thread_sample_frames": n1,
        "wall_s": t_ext + t_all + t_one + t_one_m,
    }


# ---------------------------------------------------------------------------------------------
# launcher: N rank processes, spawned before anything touches a GPU
# ---------------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_replicas(n):
    """Start n copies of this script as ranks 0..n-1 (fresh processes, so the GPU is first
    touched inside each rank) and relay rank 0's output; exit code = the first failing rank's."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    # rank 0's output is drained on a thread while every rank is polled: a rank that dies early
    # would otherwise leave the others blocked in the rendezvous or the barrier
    import threading

    chunks = []
    reader = threading.Thread(target=lambda: chunks.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    failed = 0
    while any(p.poll() is None for p in procs):
        bad = next((p.returncode for p in procs if p.returncode not in (None, 0)), 0)
        if bad:
            failed = bad
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.05)
    reader.join(timeout=30)
    sys.stdout.write(b"".join(chunks).decode())
    sys.stdout.flush()
    return failed or next((p.returncode for p in procs if p.returncode), 0)


# ---------------------------------------------------------------------------------------------
# the CPU dry run (launcher / rank plumbing tests)
# ---------------------------------------------------------------------------------------------
def run_dry(args):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle

    import orbslam_jpminipc_amd as orb
    from orbslam_jpminipc_amd import replicas

    info = replicas.init_from_env()  # the default control plane (gloo)
    W, H, B = 160, 120, 2
    frames = orb.synth_stream(W, H, stream=info.rank, first=0, count=B)
    ora = Oracle(300, 1.2, 4, 1, 20)
    for _ in range(args.warmup):
        for f in frames:
            ora.extract(f)
    replicas.barrier(info)
    t0 = time.perf_counter()
    n = 0
    for _ in range(args.steps):
        for f in frames:
            n += len(ora.extract(f)[0])
    dt = time.perf_counter() - t0
    replicas.barrier(info)
    tmax = replicas.max_over_ranks(dt, info)
    ranks = replicas.gather_over_ranks(dt, info)
    if info.rank == 0:
        print(json.dumps({"metric": METRIC, "value": replicas.whole_job_rate(B * args.steps, info.world, tmax),
                          "unit": "frames/s", "n_gpus": info.world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": tmax / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
                          "vs_baseline": None, "dtype": "u8", "data": "synthetic (dry run: CPU oracle, 160x120)",
                          "config": {"workload": "dry run (launcher plumbing)", "parallelism":
                                     f"replicas x{info.world} (no collectives)"},
                          "rank_seconds": ranks, "keypoints": n}))
    replicas.shutdown(info)
    return 0


# ---------------------------------------------------------------------------------------------
# one GPU rank
# ---------------------------------------------------------------------------------------------
def latency_b1(orb, W, H, NF, device, frames, reps=100):
    """Per-call latency of the reference's per-frame path (rank 0, N = 1)."""
    import torch

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle, search_for_initialization

    f0, f1 = frames[0].copy(), frames[1].copy()
    ext = orb.ORBextractor(NF, 1.2, 8, orb.FAST_SCORE, 20, device=device, max_batch=1)
    for _ in range(10):
        ext(f0)
    t0 = time.perf_counter()
    for _ in range(reps):
        k0, d0 = ext(f0)
    t_ext = (time.perf_counter() - t0) / reps
    k1, d1 = ext(f1)
    F1 = orb.Frame(k0, d0, W, H)
    F2 = orb.Frame(k1, d1, W, H)
    prev0 = np.ascontiguousarray(np.stack([F1.mvKeys["x"], F1.mvKeys["y"]], 1).astype(np.float32))
    M = orb.ORBmatcher(0.9, True)
    m12 = []
    for _ in range(10):
        M.SearchForInitialization(F1, F2, prev0.copy(), m12, 100)
    t_sfi = 0.0
    for _ in range(reps):
        p = prev0.copy()
        t0 = time.perf_counter()
        M.SearchForInitialization(F1, F2, p, m12, 100)
        t_sfi += time.perf_counter() - t0
    t_sfi /= reps
    # device-resident frame: the kernel chain alone (launches + one stream sync)
    d = torch.from_numpy(f0.reshape(1, H, W).copy()).cuda(device)
    s = torch.cuda.Stream(device)
    outs = ext.extract_batch_device(d, stream=s)
    s.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        ext.extract_batch_device(d, *outs, stream=s)
        s.synchronize()
    t_dev = (time.perf_counter() - t0) / reps
    ora = Oracle(NF, 1.2, 8, 1, 20)
    ora.extract(f0)
    n_cpu = 20
    t0 = time.perf_counter()
    for _ in range(n_cpu):
        ora.extract(f0)
    c_ext = (time.perf_counter() - t0) / n_cpu
    t0 = time.perf_counter()
    for _ in range(n_cpu):
        search_for_initialization(F1.mvKeys, F1.mDescriptors, F2.mvKeys, F2.mDescriptors, W, H, prev0.copy(), 0.9,
                                  True, 100)
    c_sfi = (time.perf_counter() - t0) / n_cpu
    # the same entry points timed in C++ (build/latency_gpu, a child process: no Python in the
    # loop), plus SearchByBoW(KF, F) and SearchByProjection(local map) per call
    c_abi = None
    exe = os.path.join(ROOT, "build", "latency_gpu")
    if os.path.exists(exe):
        r = subprocess.run([exe, str(W), str(H), str(NF), "200"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True, timeout=120)
        if r.returncode == 0:
            c_abi = json.loads(r.stdout.strip().splitlines()[-1])
    return {
        "c_abi_us": c_abi,
        "orb_extract_host_ms": t_ext * 1e3,
        "orb_extract_device_b1_ms": t_dev * 1e3,
        "search_for_initialization_host_ms": t_sfi * 1e3,
        "cpu_oracle_single_thread_extract_ms": c_ext * 1e3,
        "cpu_oracle_single_thread_sfi_ms": c_sfi * 1e3,
        "note": f"{W}x{H}, {NF} kp, {reps} calls each through the Python binding (ctypes); host entries include "
                "the H2D/D2H copies through the handle's pinned staging and one stream synchronisation per call; "
                "the FAST(7) re-runs always run in k_rerun (more workgroups per (frame, level) at small "
                "batches), and batches below 256 frames build the pyramid with per-level launches "
                "(k_pyr0, k_pyr_resize)",
    }


def orbvoc_shaped_tree(k=10, L=6, seed=106):
    """An ORBvoc.txt-shaped vocabulary (k = 10, L = 6: 1 111 111 nodes, TF-IDF, L1) in file order,
    random node descriptors and leaf weights: the reference ships no vocabulary (Data/ is not in
    the repository) and nothing can be downloaded here."""
    rng = np.random.default_rng(seed)
    n = sum(k ** d for d in range(1, L + 1))
    parent = np.zeros(n, np.int32)
    width, pos, prev_first = 1, 0, 0
    for _ in range(1, L + 1):
        parent[pos:pos + width * k] = np.repeat(np.arange(prev_first, prev_first + width, dtype=np.int32), k)
        prev_first = pos + 1
        pos += width * k
        width *= k
    leaf = np.zeros(n, np.uint8)
    leaf[n - k ** L:] = 1
    desc = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    weight = np.where(leaf > 0, rng.uniform(0.0, 3.0, size=n), 0.0)
    return parent, leaf, desc, weight


def bow_leg(orb, d_kps, d_desc, d_cnt, f1, f2, steps, warmup, stream, workload=None, W=0, H=0, NF=0):
    """The BoW-bucketed matching path on the step's extractor output (north_star: "BoW-bucketed
    matching"): Frame::ComputeBoW for every frame (TemplatedVocabulary::transform with levelsup 4,
    Frame.cc:280-287) then SearchByBoW(KeyFrame = frame t, Frame = frame t+1) with
    TrackReferenceKeyFrame's ORBmatcher(0.7, true) (Tracking.cc:927), every KF keypoint taken as
    holding a good MapPoint (the most work per pair).  Both batched on the device, one stream;
    each stage timed with HIP events on that stream."""
    import torch

    voc = orb.ORBVocabulary.from_arrays(10, 6, 0, 0, *orbvoc_shaped_tree())
    matcher = orb.ORBmatcher(0.7, True)
    B, cap = int(d_desc.shape[0]), int(d_desc.shape[1])
    with torch.cuda.stream(stream):
        fv = voc.transform_batch_device(d_desc, d_cnt, 4, stream=stream)
        for _ in range(warmup):
            voc.transform_batch_device(d_desc, d_cnt, 4, out=fv, stream=stream)
            m, nm = matcher.search_by_bow_batch_device(False, d_kps, d_desc, d_cnt, fv, f1, f2, stream=stream)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        t_tr = t_m = 0.0
        for _ in range(steps):
            ev[0].record(stream)
            voc.transform_batch_device(d_desc, d_cnt, 4, out=fv, stream=stream)
            ev[1].record(stream)
            m, nm = matcher.search_by_bow_batch_device(False, d_kps, d_desc, d_cnt, fv, f1, f2, stream=stream)
            ev[2].record(stream)
            ev[2].synchronize()
            t_tr += ev[0].elapsed_time(ev[1])
            t_m += ev[1].elapsed_time(ev[2])
    t_tr /= steps
    t_m /= steps
    cnt = d_cnt.cpu().numpy().astype(np.int64)
    nm_h = nm.cpu().numpy()
    P = int(f1.numel())
    nfeat = int(cnt.sum())
    f1h, f2h = f1.cpu().numpy(), f2.cpu().numpy()
    # algorithmic bytes: transform = every descriptor read once + its BowVector / FeatureVector
    # entries written (word u32, weight f64, node u32, BowVector word + value, FeatureVector node /
    # offset / feature: 40 B per feature) -- the tree itself is cache-resident reuse, not counted;
    # match = both frames' descriptors read once + the output row (4 B per slot of frame b)
    b_tr = nfeat * (32 + 40)
    b_m = int(sum(32 * (cnt[a] + cnt[b]) + 4 * cap for a, b in zip(f1h, f2h)))
    tr_pmc = m_pmc = None
    if workload:
        t1 = pmc_traffic("k_voc_descend", workload, W, H, B, NF)[0]
        t2 = pmc_traffic("k_voc_bow", workload, W, H, B, NF)[0]
        tr_pmc = t1 + t2 if t1 is not None and t2 is not None else None
        m_pmc = pmc_traffic("k_bow_pairs", workload, W, H, B, NF)[0]
    return {
        "what": "Frame::ComputeBoW (transform, levelsup 4) on every frame + SearchByBoW(KF = frame t, F = frame t+1), "
                "ORBmatcher(0.7, true), batched on the device",
        "vocabulary": "ORBvoc-shaped random tree: k=10, L=6, 1111111 nodes, TF-IDF / L1 (no ORBvoc.txt in the reference)",
        "frames": B, "pairs": P, "features": nfeat,
        "transform_ms": t_tr, "match_ms": t_m, "ms_per_step": t_tr + t_m,
        "frames_per_s": B / ((t_tr + t_m) * 1e-3), "pairs_per_s": P / (t_m * 1e-3),
        "matches_per_pair": float(nm_h.mean()),
        "transform_roofline": {"bound": "hbm", "achieved": b_tr / (t_tr * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": b_tr / (t_tr * 1e-3) / 1e9 / HBM_PEAK_GBS,
                               "algorithmic_bytes": b_tr, "traffic": tr_pmc, "traffic_kernels": "k_voc_descend + k_voc_bow",
                               "traffic_unit": "bytes per step (rocprofv3 PMC, profiles/pmc_<workload>.json)"},
        "match_roofline": {"bound": "hbm", "achieved": b_m / (t_m * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": b_m / (t_m * 1e-3) / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes": b_m,
                           "traffic": m_pmc, "traffic_kernels": "k_bow_pairs",
                           "traffic_unit": "bytes per launch (rocprofv3 PMC, profiles/pmc_<workload>.json)"},
    }


def host_fed(ext, matcher, frames_h, f1, f2, W, H, steps, warmup):
    """The step fed from host memory, as a caller of ORBextractor::operator() sees it
    (ORBextractor.h:43-45: a host cv::Mat in, host keypoints / descriptors out; Frame.cc:60,
    Tracking.cc:215-217): every step's B frames start in pinned host memory and its keypoint
    records, descriptors, counts and SearchForInitialization results end in pinned host memory.
    Three streams, double-buffered device and host buffers: H2D of batch t+1 and D2H of batch
    t-1 overlap the extraction + matching of batch t (event-ordered, so a buffer is rewritten
    only after its last reader).  Returns frames/s with the achieved PCIe rate each way and the
    link's measured one-way ceiling (one large pinned copy each way, alone)."""
    import torch

    B = frames_h.shape[0]
    cap = ext.max_keypoints
    P = int(f1.numel())
    h_in = torch.from_numpy(frames_h).pin_memory()
    d_in = [torch.empty_like(h_in, device="cuda") for _ in range(2)]
    d_out = [(torch.empty((B, cap, 28), dtype=torch.uint8, device="cuda"),
              torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda"),
              torch.empty((B,), dtype=torch.int32, device="cuda")) for _ in range(2)]
    d_m = [None, None]
    h_out = [(torch.empty((B, cap, 28), dtype=torch.uint8).pin_memory(),
              torch.empty((B, cap, 32), dtype=torch.uint8).pin_memory(),
              torch.empty((B,), dtype=torch.int32).pin_memory(),
              torch.empty((P, cap), dtype=torch.int32).pin_memory(),
              torch.empty((P,), dtype=torch.int32).pin_memory()) for _ in range(2)]
    # HIP maps plain streams round-robin onto GPU_MAX_HW_QUEUES hardware queues (4 by default):
    # three plain streams here share queues with the streams created before them and the H2D
    # copies serialise with the extraction (4.18 ms per c3 step = H2D + compute, round 4).  The
    # library's dedicated-queue streams avoid that at the default queue count
    from orbslam_jpminipc_amd.streams import dedicated_stream

    dev = torch.cuda.current_device()
    s_h2d, s_comp, s_d2h = dedicated_stream(dev), dedicated_stream(dev), dedicated_stream(dev)
    ev_h2d = [torch.cuda.Event() for _ in range(2)]
    ev_comp = [torch.cuda.Event() for _ in range(2)]
    ev_d2h = [torch.cuda.Event() for _ in range(2)]
    torch.cuda.synchronize()

    def issue(t):
        i = t % 2
        with torch.cuda.stream(s_h2d):
            if t >= 2:
                s_h2d.wait_event(ev_comp[i])  # extraction t-2 has read d_in[i]
            d_in[i].copy_(h_in, non_blocking=True)
            ev_h2d[i].record(s_h2d)
        with torch.cuda.stream(s_comp):
            s_comp.wait_event(ev_h2d[i])
            if t >= 2:
                s_comp.wait_event(ev_d2h[i])  # D2H t-2 has read d_out[i]
            kps, desc, cnt = d_out[i]
            ext.extract_batch_device(d_in[i], kps, desc, cnt, stream=s_comp)
            d_m[i] = matcher.search_for_initialization_batch_device(kps, desc, cnt, f1, f2, W, H, 100,
                                                                    stream=s_comp)
            ev_comp[i].record(s_comp)
        with torch.cuda.stream(s_d2h):
            s_d2h.wait_event(ev_comp[i])
            hk, hd, hc, hm, hn = h_out[i]
            hk.copy_(d_out[i][0], non_blocking=True)
            hd.copy_(d_out[i][1], non_blocking=True)
            hc.copy_(d_out[i][2], non_blocking=True)
            hm.copy_(d_m[i][0], non_blocking=True)
            hn.copy_(d_m[i][1], non_blocking=True)
            ev_d2h[i].record(s_d2h)

    for t in range(warmup):
        issue(t)
    torch.cuda.synchronize()
    # three timed passes of `steps` steps; the best is reported with all three (the first passes
    # over fresh pinned buffers run up to ~1.7x slower on some boxes)
    passes = []
    for _ in range(3):
        t0 = time.perf_counter()
        for t in range(steps):
            issue(t)
        torch.cuda.synchronize()
        passes.append(time.perf_counter() - t0)
    dt = min(passes)
    in_bytes = h_in.numel()
    out_bytes = sum(x.numel() * x.element_size() for x in h_out[0])

    def one_way(src, dst, reps=5):
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(reps):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        return src.numel() * src.element_size() * reps / (time.perf_counter() - a) / 1e9

    h2d_peak = one_way(h_in, d_in[0])
    d2h_peak = one_way(d_in[0], h_in)

    def alone(fn, reps=5):  # one leg of the step by itself, ms per step
        fn()
        torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - a) / reps * 1e3

    def compute_leg():
        with torch.cuda.stream(s_comp):
            kps, desc, cnt = d_out[0]
            ext.extract_batch_device(d_in[0], kps, desc, cnt, stream=s_comp)
            matcher.search_for_initialization_batch_device(kps, desc, cnt, f1, f2, W, H, 100, stream=s_comp)

    def d2h_leg():
        with torch.cuda.stream(s_d2h):
            for dst, src in zip(h_out[0], (*d_out[0], *d_m[0])):
                dst.copy_(src, non_blocking=True)

    h2d_ms = alone(lambda: d_in[0].copy_(h_in, non_blocking=True))
    comp_ms = alone(compute_leg)
    d2h_ms = alone(d2h_leg)
    fps = B * steps / dt
    return {
        "value": fps,
        "unit": "frames/s",
        "ms_per_step": dt / steps * 1e3,
        "steps": steps,
        "h2d_bytes_per_step": in_bytes,
        "d2h_bytes_per_step": out_bytes,
        "h2d_GBps": in_bytes * steps / dt / 1e9,
        "d2h_GBps": out_bytes * steps / dt / 1e9,
        "h2d_link_GBps_measured": h2d_peak,
        "d2h_link_GBps_measured": d2h_peak,
        "input_bound_fps": h2d_peak * 1e9 / (in_bytes / B),
        "legs_alone_ms": {"h2d": h2d_ms, "compute": comp_ms, "d2h": d2h_ms,
                          "sum": h2d_ms + comp_ms + d2h_ms, "max": max(h2d_ms, comp_ms, d2h_ms)},
        "copy_engine_bound_ms": h2d_ms + d2h_ms,
        "passes_ms_per_step": [x / steps * 1e3 for x in passes],
        "note": f"{B} frames per step from pinned host memory; outputs (keypoint records, descriptors, counts, "
                f"vnMatches12 of {P} pairs, nmatches) to pinned host memory at full capacity ({cap} slots per frame); "
                "three dedicated-queue streams (orb_stream_create_dedicated), double-buffered; link ceilings: one pinned copy of the step's frames each way, alone",
    }


def run_rank(args):
    import torch

    import orbslam_jpminipc_amd as orb
    from orbslam_jpminipc_amd import replicas

    # The control plane (barrier, max over ranks, gather of the per-rank seconds) runs on gloo
    # by default: the path has no data-path collective, so RCCL would only add
    # its init on every rank; gloo is the backend tests/test_multiproc.py and
    # tests/test_gpu_replicas.py rehearse.  ORB_BENCH_BACKEND=nccl selects RCCL.  Rank r uses
    # device r mod count (several ranks share the one GPU of a test box).
    backend = os.environ.get("ORB_BENCH_BACKEND", "gloo")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and backend != "nccl":
        local = local % max(1, torch.cuda.device_count())  # device_count does not initialise the GPU
    torch.cuda.set_device(local)  # before the process group and before any other GPU call
    info = replicas.init_from_env(backend)
    world, rank = info.world, info.rank
    wl = WORKLOADS[args.workload]
    W = args.width or wl["W"]
    H = args.height or wl["H"]
    NF = args.nfeatures or wl["nf"]
    custom = (W, H, NF) != (wl["W"], wl["H"], wl["nf"])
    if wl["streams"]:
        if world > wl["streams"]:
            raise SystemExit(f"{args.workload}: {wl['streams']} streams cannot feed {world} ranks")
        my_streams = replicas.streams_of_rank(wl["streams"], rank, world)
        per = args.frames_per_stream
    else:
        my_streams = [rank]
        per = args.batch
    B = per * len(my_streams)
    frames = np.concatenate([orb.synth_stream(W, H, stream=s, first=0, count=per) for s in my_streams])
    d_imgs = torch.from_numpy(frames).cuda()
    ext = orb.ORBextractor(NF, 1.2, 8, orb.FAST_SCORE, 20, device=local, max_batch=B)
    matcher = orb.ORBmatcher(0.9, True)
    cap = ext.max_keypoints
    d_kps = torch.empty((B, cap, 28), dtype=torch.uint8, device="cuda")
    d_desc = torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda")
    d_cnt = torch.empty((B,), dtype=torch.int32, device="cuda")
    # pairs (t, t+1) inside each stream's run of frames
    f1 = torch.tensor([k * per + t for k in range(len(my_streams)) for t in range(per - 1)], dtype=torch.int32,
                      device="cuda")
    f2 = f1 + 1
    P = int(f1.numel())
    # serial mode (default): one stream carries the whole step, extraction then the matching that
    # reads its output.  --overlap 1 / 2 (measured slower): a two-stage stream
    # pipeline over consecutive batches, step t extracting batch t (or only its pyramid) while
    # s_match runs SearchForInitialization on batch t-1 (double-buffered, event-ordered).
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
    rank_seconds = replicas.gather_over_ranks(elapsed, info)

    # workload statistics of the last step (identical every step: same frames)
    cnt = d_cnt.cpu().numpy().astype(np.int64)
    kps_h = d_kps.cpu().numpy()
    oct0 = np.array([int((orb.keypoints_from_bytes(kps_h[b], cnt[b])["octave"] == 0).sum()) for b in range(B)])
    n_kp = int(cnt.sum())
    nm_h = nm.cpu().numpy()
    f1h, f2h = f1.cpu().numpy(), f2.cpu().numpy()
    sb = stage_bytes(W, H, n_kp, B)
    lv = level_sizes(W, H)
    px = [w * h for w, h in lv]
    b_ext = B * (sum(px) + sum(px[1:])) + 60 * n_kp
    # SURVEY §8d B_match = 32 (N1 + N2) + 20 N1 per pair
    b_match = int(sum(32 * (cnt[a] + cnt[b]) + 20 * cnt[a] for a, b in zip(f1h, f2h)))
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
    # batches >= 256 frames build the whole pyramid in one k_pyr_stream launch (profile stage 0,
    # stage 1 empty): its algorithmic bytes are the level-0 read and the derived levels written
    if "k_pyr0" in stages and "k_pyr_resize" not in stages:
        s = stages.pop("k_pyr0")
        s["bytes_per_launch"] = B * sum(px)
        s["GBps"] = s["bytes_per_launch"] / (s["ms_per_launch"] * 1e-3) / 1e9
        s["note"] = "whole pyramid (level-0 read + levels 1-7 written) in one streaming launch"
        stages = {"k_pyr_stream": s, **stages}
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
    frames_job = per * wl["streams"] if wl["streams"] else B * world  # every rank's frames of one step

    value = frames_job * args.steps / tmax
    traffic, traffic_src, pmc = pmc_traffic(dom, args.workload, W, H, B, NF)
    pmc = pmc or {}
    valu_insts = pmc.get("SQ_INSTS_VALU")
    # VALU issue ceiling: each SIMD issues one wave64 VALU instruction per 2 cycles
    # (MI355X_MICROARCH.md), 4 SIMDs x 256 CUs at 2.4 GHz
    valu_peak = N_CU * 4 / 2 * CLOCK_HZ
    # the roof that actually binds the dominant kernel: the larger of its VALU-issue fraction
    # and its PMC-measured HBM fraction (the algorithmic-bytes fraction below is the contract's
    # HBM roofline figure; it is not what limits these integer kernels)
    roofs = {}
    launch_s = ds["ms_per_launch"] * 1e-3
    if valu_insts:
        roofs["valu_issue"] = valu_insts / launch_s / valu_peak
        # the same instructions against the measured issue rate of the instruction kinds these
        # kernels are made of (4 cycles per wave64 instruction): the practical VALU ceiling
        roofs["valu_issue_4c"] = valu_insts / launch_s / VALU_4C_PEAK
    salu_insts = pmc.get("SQ_INSTS_SALU")
    if salu_insts:
        # one scalar unit per CU issuing one SALU instruction per cycle (MI355X_MICROARCH.md: 4
        # SIMDs + 1 scalar unit per CU), shared by all the CU's waves
        roofs["salu_issue"] = salu_insts / launch_s / SALU_PEAK
    lds_insts, lds_conf = pmc.get("SQ_INSTS_LDS"), pmc.get("SQ_LDS_BANK_CONFLICT")
    if lds_insts:
        # the CU's LDS pipe: at least one cycle per wave64 LDS instruction (256 B/clk/CU, a
        # dword per lane) plus every bank-conflict cycle the SQ counted (a lower bound on LDS
        # busy time: b64 / b128 accesses take 2 / 4 cycles)
        roofs["lds_issue"] = (lds_insts + (lds_conf or 0)) / launch_s / LDS_PEAK
    if traffic:
        roofs["hbm_measured_traffic"] = traffic / launch_s / 1e9 / HBM_PEAK_GBS
    binding = max(roofs, key=roofs.get) if roofs else None
    label = wl["label"] if not custom else f"custom {W}x{H}, ORBextractor({NF},1.2,8,FAST,20) + SearchForInitialization"
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": per_step_s * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if wl["streams"] else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (csrc/synth.c: rectangles+discs+noise, consecutive frames of a stream shifted)",
        "config": {
            "workload": label,
            "preset": args.workload,
            "width": W, "height": H, "nfeatures": NF,
            "batch_per_gpu": B,
            "pairs_per_gpu": P,
            "streams_of_rank0": my_streams,
            "parallelism": f"replicas x{world} (no collectives)",
            "control_backend": backend if world > 1 else None,
            "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
            "streams": {0: "one stream, extract then match",
                        1: "extract(t) || SearchForInitialization(t-1), double-buffered",
                        2: "pyramid(t) || SearchForInitialization(t-1), then the rest of extract(t)"}
                       [args.overlap],
        },
        "rank_seconds": rank_seconds,
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
            "algorithmic_bytes_basis": "SURVEY.md §8d, this stage's terms only (bench.stage_bytes)",
            "valu_insts_per_launch": valu_insts,
            "valu_issue_frac": roofs.get("valu_issue"),
            "valu_issue_4c_frac": roofs.get("valu_issue_4c"),
            "salu_issue_frac": roofs.get("salu_issue"),
            "lds_issue_frac": roofs.get("lds_issue"),
            # the other issue ports of the same PMC pass: SALU (one per CU per cycle) and the LDS
            # instructions with their bank-conflict cycles
            "salu_insts_per_launch": pmc.get("SQ_INSTS_SALU"),
            "lds_insts_per_launch": pmc.get("SQ_INSTS_LDS"),
            "lds_bank_conflict_cycles_per_launch": pmc.get("SQ_LDS_BANK_CONFLICT"),
            "binding": binding,
            "binding_frac": roofs.get(binding) if binding else None,
            "roofs": roofs,
            "bound_note": "bound/frac price the kernel against the HBM roofline with SURVEY §8d algorithmic "
                          "bytes (the contract's figure); `binding` names the roof that limits it, from the "
                          "same PMC pass: valu_issue = SQ_INSTS_VALU / (1024 SIMDs x 1 per 2 cycles), valu_issue_4c = "
                          "SQ_INSTS_VALU / (1024 SIMDs x 0.58 per ns, the measured rate of the 4-cycle "
                          "instruction kinds, profiles/r05_valu_rate.json), "
                          "salu_issue = SQ_INSTS_SALU / (256 CUs x 1 per cycle), lds_issue = (SQ_INSTS_LDS "
                          "+ SQ_LDS_BANK_CONFLICT) / (256 CUs x 1 per cycle), hbm_measured_traffic = PMC "
                          "bytes / 8 TB/s; all at 2.4 GHz over the event-timed launch",
        },
        "pipeline": {
            "algorithmic_bytes_per_step": b_ext + b_match,
            "GBps": (b_ext + b_match) / per_step_s / 1e9,
            "frac": (b_ext + b_match) / per_step_s / 1e9 / HBM_PEAK_GBS,
        },
        "stages": stages,
        "workload_stats": {"keypoints_per_frame": n_kp / B, "octave0_per_frame": float(oct0.mean()),
                           "matches_per_pair": float(nm_h.mean())},
    }
    if args.overlap:
        result["serial_step"] = {"value": frames_job * args.steps / serial_tmax,
                                 "ms_per_step": serial_tmax / args.steps * 1e3}
    if rank == 0 and world == 1 and args.host_fed:
        # (a cold first pass over fresh pinned buffers runs ~1.7x slower: warm up with whole steps)
        hf = host_fed(ext, matcher, frames, f1, f2, W, H, 10, 8)
        hf["vs_device_resident"] = hf["value"] / value
        result["host_fed"] = hf
    if rank == 0 and world == 1 and args.bow:
        result["bow"] = bow_leg(orb, d_kps, d_desc, d_cnt, f1, f2, 10, 3, s_ext, args.workload, W, H, NF)
    if rank == 0 and world == 1 and args.latency:
        result["latency_b1"] = latency_b1(orb, W, H, NF, local, frames[:2])
    if rank == 0 and world == 1 and args.cpu_frames > 0:
        hc = host_cpus()
        # every core the process may use (north_star: "all host cores, count stated")
        threads = args.cpu_threads or hc["affinity"]
        ncpu = max(args.cpu_frames, 4 * threads)  # at least 4 frames per thread
        cpu_frames = orb.synth_stream(W, H, stream=0, first=0, count=ncpu)
        quota = hc["cgroup_cpu_quota"]
        cb = cpu_baseline(cpu_frames, NF, threads, W, H, int(quota) if quota and quota >= 1 else None)
        pcores = physical_cores()
        # value = the best measured CPU rate, with the thread count it ran at (the cgroup quota
        # often makes the quota-sized run faster than one thread per affinity CPU)
        best_fps, best_threads = cb["extract_match_fps"], threads
        if cb.get("quota_threads_extract_match_fps", 0) > best_fps:
            best_fps, best_threads = cb["quota_threads_extract_match_fps"], cb["quota_threads"]
        result["cpu_baseline"] = {
            "value": best_fps,
            "unit": "frames/s",
            "cores": best_threads,
            "value_note": "the best measured CPU rate (extract + SearchForInitialization) with the threads it ran on; "
                          "the affinity-set run, the quota-sized run and the all-physical-core estimate are beside it",
            "kind": "port",
            "sample": f"{ncpu} frames of stream 0, extract + {ncpu - 1} consecutive-pair SearchForInitialization "
                      f"(C++ restatement oracle, -O3 -march=native, scalar: not OpenCV's SSE2 build)",
            "extract_fps": cb["extract_fps"],
            "affinity_threads": threads,
            "extract_match_fps": cb["extract_match_fps"],
            "single_thread_ms_per_frame_extract": cb["single_thread_ms_per_frame_extract"],
            "single_thread_ms_per_frame_extract_match": cb["single_thread_ms_per_frame_extract_match"],
            "single_thread_sample_frames": cb["single_thread_sample_frames"],
            "cpu_model": cpu_model(),
            "logical_cpus_visible": hc["logical_cpus"],
            "affinity_cpus": hc["affinity"],
            "cgroup_cpu_quota": hc["cgroup_cpu_quota"],
            "omp_num_threads_env": hc["omp_num_threads"],
            "cores_note": "threads = the process's CPU affinity set (every core it may run on)"
                          + ("" if hc["cgroup_cpu_quota"] is None else
                             f"; the cgroup caps CPU time at {hc['cgroup_cpu_quota']:g} CPUs, so the "
                             "threads share that quota"),
            "wall_s": cb["wall_s"],
        }
        if "quota_threads" in cb:
            result["cpu_baseline"]["at_quota_threads"] = {
                "threads": cb["quota_threads"], "extract_match_fps": cb["quota_threads_extract_match_fps"]}
        if pcores:
            # what the whole socket would reach if every physical core ran the single-thread rate
            # (no SMT gain, no memory contention): an estimate for the ratio, not a measurement
            result["cpu_baseline"]["machine_physical_cores"] = pcores
            result["cpu_baseline"]["estimate_all_physical_cores_fps"] = (
                pcores * 1e3 / cb["single_thread_ms_per_frame_extract_match"])
            result["cpu_baseline"]["gpu_over_estimate_all_physical_cores"] = value / (
                pcores * 1e3 / cb["single_thread_ms_per_frame_extract_match"])
        result["cpu_baseline"]["gpu_over_value"] = value / best_fps
    if rank == 0:
        print(json.dumps(result))
    replicas.shutdown(info)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks; without torch.distributed.run this script spawns "
                                                        "them itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3")
    ap.add_argument("--batch", type=int, default=512, help="frames per step per GPU (c3, c4)")
    # 512: at N = 8 every rank keeps one stream of 512 frames, the batch size at which the
    # per-frame rate has saturated (1280x720: B = 128 / 256 / 512 / 1024 -> 69 / 82 / 95 / 96k
    # frames/s on one GPU, profiles/r03_v2_c5_batch_sweep.txt)
    ap.add_argument("--frames-per-stream", type=int, default=512, help="frames of each stream per step (c5)")
    ap.add_argument("--width", type=int, default=0, help="override the preset (0 = preset)")
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--nfeatures", type=int, default=0)
    ap.add_argument("--cpu-frames", type=int, default=1536,
                    help="CPU-baseline sample size (0 = skip; at least 4 frames per thread)")
    ap.add_argument("--latency", type=int, default=1, help="1: measure latency_b1 (rank 0, N = 1)")
    ap.add_argument("--host-fed", type=int, default=1,
                    help="1: measure the host-fed step (pinned host frames in, host results out; rank 0, N = 1)")
    ap.add_argument("--bow", type=int, default=1,
                    help="1: measure the BoW leg (vocabulary transform + batched SearchByBoW; rank 0, N = 1)")
    ap.add_argument("--overlap", type=int, default=0,
                    help="0 (default): serial step; 1 / 2: stream-overlap experiments, measured slower")
    ap.add_argument("--survey-steps", type=int, default=5, help="untimed steps with every stage bracketed")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU of the affinity set")
    ap.add_argument("--dry-run", action="store_true", help="CPU only: launcher + rank plumbing with the oracle")
    args = ap.parse_args()
    args.survey_steps = max(1, args.survey_steps)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_replicas(args.gpus)
    if args.dry_run:
        return run_dry(args)
    return run_rank(args)


if __name__ == "__main__":
    sys.exit(main())
