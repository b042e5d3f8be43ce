#!/bin/bash
# round 5: k_orient_desc nondeterminism diagnosis (scripts/od_tables_variant.py variants)
set -o pipefail
mkdir -p gpurun_out/r05_diag
for v in "$@"; do
  lib=""; [ "$v" = "intree" ] || lib=$PWD/build/variants/$v.so
  echo "== $v"
  ORB_HIP_LIB=$lib timeout -k 10 240 python scripts/od_diag.py 640 480 2000 ${REPS:-6} > gpurun_out/r05_diag/$v.txt 2>&1 || { echo "diag $v rc=$?"; tail -20 gpurun_out/r05_diag/$v.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r05_diag/$v.txt | tail -2
done
