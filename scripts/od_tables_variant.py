#!/usr/bin/env python3
"""Scratch build (experiment harness) of the shipped k_orient_desc with ONE change: its three
constant tables (row-pass B fragments, IC disc masks, rBRIEF pattern) read through device
pointers passed as a kernel argument (hipGetSymbolAddress; global loads at 32-bit byte
offsets) instead of through the __constant__ symbols.  `scripts/r04_diag.sh NAME` on the result
reproduces the nondeterministic descriptor bits recorded in DESIGN.md §6.
Usage: od_tables_variant.py NAME  ->  build/variants/NAME.so"""
import subprocess, sys
reps = [
 ("__constant__ uint4 c_rowB[4 * 64];  // 279 patch dwords per alignment, zero-padded to 5 x 64\n",
  "__constant__ uint4 c_rowB[4 * 64];  // 279 patch dwords per alignment, zero-padded to 5 x 64\n"
  "struct ODTables { const uint4* rowB; const uint32_t* icmask; const float4* patf; };\n"
  "#define OD_LD(T, f, off) (*(const T __attribute__((address_space(1)))*)((const char __attribute__((address_space(1)))*)tb.f + (uint32_t)(off)))\n"),
 ("uint8_t* __restrict__ desc, const float* __restrict__ lvlResp) {",
  "uint8_t* __restrict__ desc, const float* __restrict__ lvlResp, ODTables tb) {"),
 ("    for (int t = 0; t < 4; ++t) Bf[t] = __builtin_bit_cast(i32x4v, c_rowB[t * 64 + lane]);",
  "    for (int t = 0; t < 4; ++t) Bf[t] = OD_LD(i32x4v, rowB, 16u * (64u * t + (uint32_t)lane));"),
 ("    for (int j = 0; j < 5; ++j) icm[j] = c_icmask[320 * ((x + 1 - xa) & 3) + lane + 64 * j];",
  "    for (int j = 0; j < 5; ++j) icm[j] = OD_LD(uint32_t, icmask, 4u * (320u * (uint32_t)((x + 1 - xa) & 3) + (uint32_t)lane + 64u * j));"),
 ("        const float4 f = ((const float4*)c_patternf)[lane * 4 + q];",
  "        typedef float f32x4v __attribute__((ext_vector_type(4)));\n        const f32x4v f = OD_LD(f32x4v, patf, 16u * (4u * (uint32_t)lane + q));"),
 ("    int2* d_lvlInfo = nullptr;     // [frame][ORB_MAX_LEVELS] (first output slot, count): k_lvl_prefix\n",
  "    int2* d_lvlInfo = nullptr;     // [frame][ORB_MAX_LEVELS] (first output slot, count): k_lvl_prefix\n    ODTables odTables{};\n"),
 ("desc, (const float*)d_lvlResp);", "desc, (const float*)d_lvlResp, odTables);"),
 ("    int st = upload_pattern(device);\n",
  "    int st = upload_pattern(device);\n    ODTables odt{};\n    HIP_TRY(hipGetSymbolAddress((void**)&odt.rowB, HIP_SYMBOL(c_rowB)));\n    HIP_TRY(hipGetSymbolAddress((void**)&odt.icmask, HIP_SYMBOL(c_icmask)));\n    HIP_TRY(hipGetSymbolAddress((void**)&odt.patf, HIP_SYMBOL(c_patternf)));\n"),
 ("    orb_extractor* h = new orb_extractor();\n", "    orb_extractor* h = new orb_extractor();\n    h->odTables = odt;\n"),
]
args = ["python3", "scripts/ablation_variant.py", sys.argv[1]]
for a, b in reps:
    args += [a, b]
sys.exit(subprocess.call(args))
