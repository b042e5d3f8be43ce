#!/bin/bash
# One GPU-box session made of named steps (run through gpurun from the repository root):
#   bash scripts/session.sh TAG STEP [STEP ...]
# Every step writes under gpurun_out/TAG/ and runs under its own time limit.  A test failure
# (rc 1) is recorded and the session goes on; any abnormal end (fault, abort, segfault, time
# limit: rc other than 0 / 1) ends the session there, as does a failing non-test step.
# Steps:
#   gpu                  the whole -m gpu suite
#   gpu:EXPR             the -m gpu tests selected by -k EXPR (e.g. gpu:desc-or-extract, '-' = ' ')
#   smoke                __graft_entry__.smoke()
#   diag[:REPS]          k_orient_desc determinism screen of the in-tree library (scripts/od_diag.py)
#   bench:WL[:ARGS]      bench.py --workload WL (default legs), ARGS comma-separated extra flags
#   quick:WL[:ARGS]      bench.py --workload WL without the CPU / latency / host-fed / BoW legs
#   prof:WL              rocprofv3 --kernel-trace --stats of quick:WL -> prof_WL/
#   pmc:WL               the PMC passes of scripts/pmc_pass.sh for WL + pmc_summary -> pmc_WL.json
#   ab:WL:V1,V2,..       per-kernel rocprofv3 means of the in-tree library and build/variants/V*.so
#                        (scripts/stage_times.py at WL's shape), alternating twice
#   abbench:WL:V1,..     quick:WL bench step of the in-tree library and each variant, alternating twice
#   latency              the C++ per-call latency probe (build/latency_gpu)
#   latprof              the same probe under rocprofv3 --kernel-trace --memory-copy-trace
#   py:SCRIPT:ARGS       python scripts/SCRIPT ARGS (comma-separated), e.g. py:km_timing.py:build/variants/kmt.so,--per,2
#   bin:NAME             a probe built on the CPU side, build/NAME
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
note() { echo "$*" | tee -a "$OUT/summary.txt"; }
fin() {  # fin NAME RC [fatal-on-1]
    note "$1 rc=$2"
    if [ "$2" -ne 0 ] && { [ "$2" -ne 1 ] || [ -n "$3" ]; }; then note "stopping after $1"; exit "$2"; fi
}
wl_args() {  # workload -> stage_times.py shape flags
    case "$1" in
        c3) echo "--batch 512" ;;
        c4) echo "--batch 512 --width 1241 --height 376 --nfeatures 2000" ;;
        c5) echo "--batch 512 --width 1280 --height 720 --nfeatures 2500" ;;
    esac
}
QUICK="--cpu-frames 0 --latency 0 --host-fed 0 --bow 0"
for S in "$@"; do
    IFS=: read -r kind a b <<< "$S"
    case "$kind" in
    gpu)
        if [ -n "$a" ]; then sel=(-k "${a//-/ }"); log=$OUT/gpu_${a//[^A-Za-z0-9]/_}.log; else sel=(); log=$OUT/gpu.log; fi
        timeout -k 10 1100 python -u -m pytest tests -q -m gpu "${sel[@]}" --maxfail=3 --timeout 180 \
            --timeout-method thread --durations=10 > "$log" 2>&1
        rc=$?; tail -3 "$log" | tee -a "$OUT/summary.txt"; fin "$S" $rc ;;
    smoke)
        timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1
        rc=$?; tail -1 "$OUT/smoke.log" | tee -a "$OUT/summary.txt"; fin smoke $rc fatal ;;
    diag)
        REPS=${a:-10} timeout -k 10 600 python scripts/od_diag.py 640 480 2000 "${a:-10}" > "$OUT/diag.txt" 2>&1
        rc=$?; grep -v amdgpu.ids "$OUT/diag.txt" | tail -1 | tee -a "$OUT/summary.txt"; fin diag $rc fatal ;;
    bench|quick)
        extra=${b//,/ }; [ "$kind" = quick ] && extra="$QUICK $extra"
        timeout -k 10 900 python bench.py --workload "$a" $extra > "$OUT/${kind}_$a.json" 2> "$OUT/${kind}_$a.err"
        rc=$?; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['ms_per_step'], 4))" "$OUT/${kind}_$a.json" "$S" 2>/dev/null | tee -a "$OUT/summary.txt"
        fin "$S" $rc fatal ;;
    prof)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$a" -o run --output-format csv -- \
            python bench.py --workload "$a" $QUICK --steps 20 > "$OUT/prof_$a.log" 2>&1
        rc=$?; fin "$S" $rc fatal
        f=$(find "$OUT/prof_$a" -name '*kernel_stats.csv' | head -1); cp "$f" "$OUT/kernel_stats_$a.csv"
        python3 - "$f" <<'PY' | tee -a "$OUT/summary.txt"
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
print({r["Name"].split("(")[0].replace("void ", "")[:28]: round(float(r["AverageNs"]) / 1e3, 1) for r in rows[:9]})
PY
        ;;
    pmc)
        timeout -k 10 900 bash scripts/pmc_pass.sh "$TAG/pmc_$a" --workload "$a" > "$OUT/pmc_$a.log" 2>&1
        rc=$?; fin "$S" $rc fatal
        python3 scripts/pmc_summary.py "$OUT/pmc_$a" --json "$OUT/pmc_$a.json" $(wl_args "$a") > "$OUT/pmc_$a.txt" 2>&1
        fin "pmc_summary $a" $? fatal ;;
    ab)
        for rep in 1 2; do
            for v in intree ${b//,/ }; do
                lib=""; [ "$v" = intree ] || lib=build/variants/$v.so
                d=$OUT/ab_${a}_${v}_$rep
                timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$d" -o run --output-format csv -- \
                    python scripts/stage_times.py $lib $(wl_args "$a") > "$d.log" 2>&1
                rc=$?; [ $rc -eq 0 ] || fin "ab $a $v" $rc fatal
                python3 - "$d" "$v" "$a" "$rep" <<'PY' | tee -a "$OUT/summary.txt"
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = {r["Name"].split("(")[0].replace("void ", ""): float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
print("ab", sys.argv[3], sys.argv[4], sys.argv[2], {k[:24]: round(v, 1) for k, v in rows.items() if k.startswith("k_")})
PY
            done
        done ;;
    abbench)
        for rep in 1 2; do
            for v in intree ${b//,/ }; do
                lib=""; [ "$v" = intree ] || lib=$PWD/build/variants/$v.so
                f=$OUT/abbench_${a}_${v}_$rep.json
                ORB_HIP_LIB=$lib timeout -k 10 600 python bench.py --workload "$a" $QUICK --steps 50 > "$f" 2> "${f%.json}.err"
                rc=$?; [ $rc -eq 0 ] || fin "abbench $a $v" $rc fatal
                python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('abbench', sys.argv[2], round(d['value']), round(d['ms_per_step'], 4))" "$f" "$a $rep $v" | tee -a "$OUT/summary.txt"
            done
        done ;;
    latency)
        timeout -k 10 300 ./build/latency_gpu 640 480 1000 200 > "$OUT/latency.txt" 2>&1
        rc=$?; tail -12 "$OUT/latency.txt" >> "$OUT/summary.txt"; fin latency $rc fatal ;;
    latprof)  # the latency probe under rocprofv3 (kernels + copies): per-call device timelines
        timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/latprof" -o run --output-format csv -- \
            ./build/latency_gpu 640 480 1000 50 > "$OUT/latprof.log" 2>&1
        rc=$?; fin latprof $rc fatal ;;
    py)  # py:SCRIPT:ARGS  python scripts/SCRIPT with comma-separated ARGS
        n=${a%.py}
        f=$OUT/py_${n//\//_}_${b//[^A-Za-z0-9]/_}.txt
        timeout -k 10 300 python "scripts/$a" ${b//,/ } > "$f" 2>&1
        rc=$?; grep -v amdgpu.ids "$f" | tail -4 | tee -a "$OUT/summary.txt"; fin "$S" $rc fatal ;;
    bin)  # bin:NAME  build/NAME (a probe built on the CPU side)
        timeout -k 10 300 "./build/$a" > "$OUT/bin_$a.txt" 2>&1
        rc=$?; tail -12 "$OUT/bin_$a.txt" | tee -a "$OUT/summary.txt"; fin "$S" $rc fatal ;;
    *) note "unknown step $S"; exit 2 ;;
    esac
done
note "session $TAG done"
