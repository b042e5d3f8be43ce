#!/bin/bash
# Per-stage times of the in-tree library and of every build/variants/*.so (scripts/stage_times.py).
# Usage (GPU box): bash scripts/ablation_run.sh TAG
TAG=${1:-abl}
mkdir -p gpurun_out/$TAG
for v in "" build/variants/*.so; do
  timeout -k 10 120 python scripts/stage_times.py $v >> gpurun_out/$TAG/stages.jsonl 2>> gpurun_out/$TAG/err.txt || exit $?
done
