#!/bin/bash
# Build k_fast phase-ablation variants of liborb_hip.so into build/variants (CPU side):
# nofast = no strength / NMS work, noqueue = pre-filter only.
set -e
cd "$(dirname "$0")/.."
bash scripts/build_variant.sh nofast -DKL_SKIP_FAST=1
bash scripts/build_variant.sh noqueue -DKL_SKIP_QUEUE=1
ls build/variants
