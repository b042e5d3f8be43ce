#!/bin/bash
# Time the extraction stages for the in-tree library and each build/variants/NAME.so given.
# Usage (via gpurun): bash scripts/variant_times.sh TAG NAME... [-- stage_times args]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
libs=""; extra=""
while [ $# -gt 0 ]; do if [ "$1" = "--" ]; then shift; extra="$@"; break; fi; libs="$libs build/variants/$1.so"; shift; done
timeout -k 10 120 python scripts/stage_times.py --batch 512 $extra >> $OUT/times.txt 2>>$OUT/err.txt || exit $?
for v in $libs; do
  timeout -k 10 120 python scripts/stage_times.py $v --batch 512 $extra >> $OUT/times.txt 2>>$OUT/err.txt || exit $?
done
