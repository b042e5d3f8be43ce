# BASELINE configs[3] / configs[4] on one GPU (GPU box): bench line + rocprofv3 kernel stats each.
# Usage: bash scripts/configs_run.sh TAG
TAG=${1:-cfg}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for c in "kitti 1241 376 2000 1024" "hd720 1280 720 2500 512"; do
  set -- $c
  timeout -k 10 300 python bench.py --width $2 --height $3 --nfeatures $4 --cpu-frames $5 > $O/bench_$1.json 2> $O/bench_$1.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$1 -o run --output-format csv -- python bench.py --width $2 --height $3 --nfeatures $4 --cpu-frames 0 --steps 5 > $O/prof_$1.log 2>&1 || exit $?
done
