"""The multi-rank bench path on real hardware: `bench.py --gpus 2` spawns two rank processes
(RANK / LOCAL_RANK / WORLD_SIZE set before any GPU call), each extracts and matches its own
frames on the GPU, and the barrier / max-over-ranks / gather of the timed region run between
them.  A one-GPU box cannot give each rank its own device or run RCCL between two ranks on
one device, so the ranks share cuda:0; the control plane is the default one (gloo), the same
the driver's 8-GPU run uses.  Plumbing only: per-rank parity is the other tests' job."""
import json
import os
import pathlib
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parent.parent


def _bench(*args):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("ORB_BENCH_BACKEND", None)  # the default control plane
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--survey-steps", "1", "--cpu-frames", "0", "--latency", "0", "--host-fed", "0", *args],
                       cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_two_ranks_weak_scaling_c3():
    d = _bench("--batch", "64")
    assert d["n_gpus"] == 2 and len(d["rank_seconds"]) == 2
    assert d["config"]["control_backend"] == "gloo"
    assert d["scaling"] == "weak" and d["config"]["batch_per_gpu"] == 64
    # whole-job frames = 2 ranks x 64 frames per step, over the slowest rank's time
    assert abs(d["value"] - 2 * 64 * 3 / max(d["rank_seconds"])) < 1e-6 * d["value"]
    assert d["workload_stats"]["keypoints_per_frame"] > 900


def test_two_ranks_stream_sharding_c5():
    d = _bench("--workload", "c5", "--frames-per-stream", "8")
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["streams_of_rank0"] == [0, 2, 4, 6] and d["config"]["batch_per_gpu"] == 32
    assert abs(d["value"] - 8 * 8 * 3 / max(d["rank_seconds"])) < 1e-6 * d["value"]
