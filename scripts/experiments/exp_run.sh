# Experiment session (GPU box): GPU parity tests (in-tree library, then any build named in
# PARITY_VARIANTS), then bench survey-pass stage times of the in-tree library and variants.
set -o pipefail
T=${1:-exp}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for v in $PARITY_VARIANTS; do
  ORB_HIP_LIB=$PWD/build/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 $O/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
bash scripts/match_ablation.sh $T || exit $?
