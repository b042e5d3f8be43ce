#!/bin/bash
# descriptor-difference diagnosis (scripts/od_diag.py) of the in-tree build or variants given
set -o pipefail
mkdir -p gpurun_out/r04_diag
for v in "${@:-intree}"; do
  lib=""; [ "$v" = "intree" ] || lib=$PWD/build/variants/$v.so
  echo "== $v"
  ORB_HIP_LIB=$lib timeout -k 10 200 python scripts/od_diag.py 640 480 2000 > gpurun_out/r04_diag/$v.txt 2>&1 || { echo "diag $v rc=$?"; tail -20 gpurun_out/r04_diag/$v.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r04_diag/$v.txt | tail -4
done
