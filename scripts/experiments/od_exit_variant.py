#!/usr/bin/env python3
"""Scratch build (experiment harness) of the SHIPPED k_orient_desc with one change: a wave whose
slot holds no keypoint issues one rBRIEF-pattern load (inline asm, so the compiler inserts no
wait for it) and ends with that load outstanding -- the condition the pointer-table variants
(scripts/od_tables_variant.py) create as a side effect.  `scripts/r05_diag.sh NAME` screens it.
Usage: od_exit_variant.py NAME  ->  build/variants/NAME.so"""
import subprocess
import sys

rep = ("    if (!active) return;",
       "    if (!active) {\n"
       "        typedef float f32x4v __attribute__((ext_vector_type(4)));\n"
       "        f32x4v junk;\n"
       "        asm volatile(\"global_load_dwordx4 %0, %1, %2\" : \"=v\"(junk) : \"v\"(16u * (4u * (uint32_t)lane)), "
       "\"s\"((const float*)c_patternf) : \"memory\");\n"
       "        return;\n"
       "    }")
sys.exit(subprocess.call(["python3", "scripts/ablation_variant.py", sys.argv[1], *rep]))
