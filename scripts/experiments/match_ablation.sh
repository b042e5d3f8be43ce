# k_match_init phase ablation (GPU box): bench survey-pass stage times per library build.
T=${1:-kmabl}; O=gpurun_out/$T; mkdir -p $O
for v in "" build/variants/*.so; do
  [ -z "$v" ] || [ -f "$v" ] || continue
  ORB_HIP_LIB=${v:+$PWD/$v} timeout -k 10 120 python bench.py --cpu-frames 0 --steps 5 --warmup 2 $BENCH_ARGS > $O/b_$(basename ${v:-intree}).json 2>> $O/err.txt || exit $?
  python -c "import json,sys; d=json.load(open('$O/b_$(basename ${v:-intree}).json')); print('${v:-intree}', d['value'], {k: round(x['ms_per_launch']*1000,1) for k,x in d['stages'].items()})"
done
