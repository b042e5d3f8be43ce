#!/bin/bash
# Build k_level phase-ablation variants of liborb_hip.so into build/variants (CPU side).
set -e
cd "$(dirname "$0")/.."
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt"
S="orbslam_jpminipc_amd/csrc/orb_hip.hip orbslam_jpminipc_amd/csrc/orb_match.hip orbslam_jpminipc_amd/csrc/orb_voc.hip orbslam_jpminipc_amd/csrc/orb_mappoint.hip orbslam_jpminipc_amd/csrc/orb_pipeline.hip orbslam_jpminipc_amd/csrc/orb_persist.hip"
mkdir -p build/variants
/opt/rocm/bin/hipcc $F -DKL_SKIP_BLUR=1 -o build/variants/noblur.so $S &
/opt/rocm/bin/hipcc $F -DKL_SKIP_FAST=1 -o build/variants/nofast.so $S &
/opt/rocm/bin/hipcc $F -DKL_SKIP_QUEUE=1 -o build/variants/noqueue.so $S &
/opt/rocm/bin/hipcc $F -DKL_SKIP_BLUR=1 -DKL_SKIP_FAST=1 -o build/variants/stageonly.so $S &
wait
ls build/variants
