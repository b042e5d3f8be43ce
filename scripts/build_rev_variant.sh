#!/bin/bash
# Build liborb_hip.so from the sources of git revision REV into build/variants/NAME.so (A/B timing
# of the working tree against an earlier commit on the same GPU box).
# Usage: bash scripts/build_rev_variant.sh NAME REV
set -e
cd "$(dirname "$0")/.."
NAME=$1; REV=${2:-HEAD}
T=$(mktemp -d /tmp/orbrev_XXXX)
git archive "$REV" orbslam_jpminipc_amd/csrc include | tar -x -C "$T"
F="$(python3 __graft_entry__.py flags)"  # the library's own flags (optional ones probed)
mkdir -p build/variants
C=$T/orbslam_jpminipc_amd/csrc
if [ -f $C/orb_ilp.hip ]; then  # revisions with the max-ILP unit: the library's own recipe
    python3 __graft_entry__.py lib build/variants/$NAME.so $C 2> build/variants/$NAME.log
else
    /opt/rocm/bin/hipcc $F -o build/variants/$NAME.so $C/orb_hip.hip $C/orb_match.hip $C/orb_voc.hip $C/orb_mappoint.hip $C/orb_pipeline.hip $C/orb_persist.hip $C/orb_frame.hip $C/orb_bow.hip 2> build/variants/$NAME.log
fi
rm -rf "$T"
echo "built build/variants/$NAME.so from $REV"
