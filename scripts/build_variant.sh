#!/bin/bash
# Build a liborb_hip.so variant with extra -D flags into build/variants/NAME.so (CPU side).
# Usage: bash scripts/build_variant.sh NAME [-DFLAG=V ...]
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
F="$(python3 __graft_entry__.py flags)"  # the library's own flags (optional ones probed)
S="orbslam_jpminipc_amd/csrc/orb_hip.hip orbslam_jpminipc_amd/csrc/orb_match.hip orbslam_jpminipc_amd/csrc/orb_voc.hip orbslam_jpminipc_amd/csrc/orb_mappoint.hip orbslam_jpminipc_amd/csrc/orb_pipeline.hip orbslam_jpminipc_amd/csrc/orb_persist.hip orbslam_jpminipc_amd/csrc/orb_frame.hip orbslam_jpminipc_amd/csrc/orb_bow.hip"
mkdir -p build/variants
/opt/rocm/bin/hipcc $F "$@" -o build/variants/$NAME.so $S 2> build/variants/$NAME.log
echo "built build/variants/$NAME.so"
