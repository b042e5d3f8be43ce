set -o pipefail
mkdir -p gpurun_out/abl1
for v in "" build/variants/noblur.so build/variants/nofast.so build/variants/noqueue.so build/variants/stageonly.so; do
  timeout -k 10 120 python scripts/stage_times.py $v --batch 512 >> gpurun_out/abl1/times.txt 2>>gpurun_out/abl1/err.txt || exit $?
done
