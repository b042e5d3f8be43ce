#!/bin/bash
# Build a liborb_hip.so variant with extra -D flags into build/variants/NAME.so (CPU side).
# Usage: bash scripts/build_variant.sh NAME [-DFLAG=V ...]
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p build/variants
python3 __graft_entry__.py lib build/variants/$NAME.so orbslam_jpminipc_amd/csrc "$@" 2> build/variants/$NAME.log
echo "built build/variants/$NAME.so"
