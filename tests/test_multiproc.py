"""The N > 1 path on CPU: two gloo ranks run the replica plumbing bench.py uses (stream
sharding, barrier, max-over-ranks timing, whole-job rate) with the oracle as the per-rank
workload, and rank results are independent of the other rank (no data-path exchange)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    import time
    import pathlib

    root = pathlib.Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root))
    sys.path.insert(0, str(root / "tests"))
    import orbslam_jpminipc_amd as orb
    from orbslam_jpminipc_amd import replicas
    from oracle_lib import Oracle

    info = replicas.init_from_env()  # the default control plane (gloo), as bench.py --gpus N uses
    import torch.distributed as dist

    assert dist.get_backend() == "gloo"
    streams = replicas.streams_of_rank(4, info.rank, info.world)
    ora = Oracle(300, 1.2, 4, 1, 20)
    replicas.barrier(info)
    t0 = time.perf_counter()
    counts = []
    for s in streams:
        f = orb.synth_stream(160, 120, stream=s, first=0, count=1)[0]
        counts.append(len(ora.extract(f)[0]))
    dt = time.perf_counter() - t0 + 0.01 * (info.rank + 1)
    replicas.barrier(info)
    tmax = replicas.max_over_ranks(dt, info)
    total = replicas.sum_over_ranks(len(streams), info)
    q.put((info.rank, streams, counts, dt, tmax, total, replicas.whole_job_rate(len(streams), info.world, tmax)))
    replicas.shutdown(info)


def test_two_rank_replicas_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, s0, c0, d0, t0, n0, v0), (r1, s1, c1, d1, t1, n1, v1) = res
    assert s0 == [0, 2] and s1 == [1, 3]  # stream s -> rank s mod world
    assert t0 == t1 == max(d0, d1)  # the slowest rank's time, seen by both
    assert n0 == n1 == 4
    assert v0 == pytest.approx(2 * 2 / t0)
    # each rank's result equals a single-process run of the same stream
    import sys, pathlib
    sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent))
    import orbslam_jpminipc_amd as orb
    from oracle_lib import Oracle

    ora = Oracle(300, 1.2, 4, 1, 20)
    for s, c in zip(s0 + s1, c0 + c1):
        assert c == len(ora.extract(orb.synth_stream(160, 120, stream=s, first=0, count=1)[0])[0])


def test_bench_launcher_spawns_ranks_dry_run():
    """`python bench.py --gpus 2` with no launcher around it spawns its two ranks itself (RANK /
    WORLD_SIZE set before any device call) and prints rank 0's line: n_gpus 2, both ranks'
    timed regions, value over the slowest.  --dry-run keeps it on the CPU (gloo, oracle)."""
    import json
    import pathlib
    import subprocess
    import sys

    root = pathlib.Path(__file__).resolve().parent.parent
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--dry-run", "--steps", "2",
                        "--warmup", "1"], cwd=root, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=300)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    lines = [l for l in r.stdout.decode().splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert len(d["rank_seconds"]) == 2 and all(t > 0 for t in d["rank_seconds"])
    assert d["value"] == pytest.approx(2 * 2 * 2 / (max(d["rank_seconds"])), rel=0.05)
    assert d["config"]["parallelism"] == "replicas x2 (no collectives)"
