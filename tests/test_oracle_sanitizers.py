"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer: `make -C
oracle sanitize` links the oracle sources and the synthetic frame generator into
oracle/_san/sanitize_check (oracle/sanitize_check.cpp), which runs every oracle entry point the
parity tests use — the extractor at each BASELINE configuration and on the edge-case frames,
SearchForInitialization, WindowSearch, the vocabulary transform and SearchByBoW, colour
conversion, ComputeDistinctiveDescriptors, the threaded CPU baseline.  Any sanitizer report
aborts the run."""
import os
import pathlib
import subprocess

ROOT = pathlib.Path(__file__).resolve().parents[1]


def test_oracle_clean_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "sanitize"], check=True, timeout=600)
    env = dict(os.environ)
    # the harness may preload a library ahead of the ASan runtime: do not treat that as an error
    env["ASAN_OPTIONS"] = "verify_asan_link_order=0:detect_leaks=1:abort_on_error=0"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([str(ROOT / "oracle" / "_san" / "sanitize_check")], capture_output=True, text=True,
                       env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "sanitize_check: 0 failures" in r.stdout
