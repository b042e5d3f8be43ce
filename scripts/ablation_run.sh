mkdir -p gpurun_out/abl1
for v in "" build/variants/ks_norerun.so build/variants/ks_noretain.so build/variants/ks_nolevel.so build/variants/noblur.so build/variants/nofast.so build/variants/noqueue.so build/variants/stageonly.so; do
  timeout -k 10 120 python scripts/stage_times.py $v >> gpurun_out/abl1/stages.jsonl 2>> gpurun_out/abl1/err.txt || exit $?
done
