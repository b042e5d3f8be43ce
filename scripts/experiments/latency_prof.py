"""Per-call latency of the single-frame host path (ORBextractor::operator(), Frame.cc:60) at a
BASELINE workload, for rocprofv3 kernel traces of the B = 1 chain.
Usage: python scripts/latency_prof.py [--workload c3|c4|c5] [--reps 200]"""
import argparse
import json
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import orbslam_jpminipc_amd as orb  # noqa: E402

WL = {"c3": (640, 480, 1000), "c4": (1241, 376, 2000), "c5": (1280, 720, 2500)}
ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c3", choices=sorted(WL))
ap.add_argument("--reps", type=int, default=200)
a = ap.parse_args()
W, H, NF = WL[a.workload]
f = orb.synth_stream(W, H, stream=0, first=0, count=1)[0]
ext = orb.ORBextractor(NF, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=1)
for _ in range(20):
    ext(f)
ts = []
for _ in range(a.reps):
    t0 = time.perf_counter()
    ext(f)
    ts.append(time.perf_counter() - t0)
ts.sort()
print(json.dumps({"workload": a.workload, "W": W, "H": H, "nfeatures": NF, "reps": a.reps,
                  "median_ms": round(1e3 * ts[len(ts) // 2], 4), "p10_ms": round(1e3 * ts[len(ts) // 10], 4),
                  "p90_ms": round(1e3 * ts[9 * len(ts) // 10], 4)}))
