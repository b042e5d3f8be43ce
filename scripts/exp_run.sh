# Experiment session (GPU box): GPU parity tests, then per-stage times of the in-tree library and variants.
set -o pipefail
T=${1:-exp}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ablation_run.sh $T || exit $?
