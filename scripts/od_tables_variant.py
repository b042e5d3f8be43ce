#!/usr/bin/env python3
"""Scratch build (experiment harness) of the shipped k_orient_desc with ONE change: its three
constant tables (row-pass B fragments, IC disc masks, rBRIEF pattern) read through device
pointers passed as a kernel argument (hipGetSymbolAddress; global loads at 32-bit byte
offsets) instead of through the __constant__ symbols.  `scripts/r04_diag.sh NAME` on the result
reproduces the nondeterministic descriptor bits recorded in DESIGN.md §6.
Usage: od_tables_variant.py NAME  ->  build/variants/NAME.so
Its text anchors are those of orb_hip.hip at commit 17303d2 (before round 5's IC-table change
replaced the disc masks); build that revision's sources to rerun it
(`git archive 17303d2 orbslam_jpminipc_amd/csrc include`)."""
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
 ("    int2* d_lvlInfo = nullptr;     // [frame][ORB_MAX_LEVELS] (first output slot, count): k_select's last WG\n",
  "    int2* d_lvlInfo = nullptr;     // [frame][ORB_MAX_LEVELS] (first output slot, count): k_select's last WG\n    ODTables odTables{};\n"),
 ("desc, (const float*)d_lvlResp);", "desc, (const float*)d_lvlResp, odTables);"),
 ("    int st = upload_pattern(device);\n",
  "    int st = upload_pattern(device);\n    ODTables odt{};\n    HIP_TRY(hipGetSymbolAddress((void**)&odt.rowB, HIP_SYMBOL(c_rowB)));\n    HIP_TRY(hipGetSymbolAddress((void**)&odt.icmask, HIP_SYMBOL(c_icmask)));\n    HIP_TRY(hipGetSymbolAddress((void**)&odt.patf, HIP_SYMBOL(c_patternf)));\n"),
 ("    orb_extractor* h = new orb_extractor();\n", "    orb_extractor* h = new orb_extractor();\n    h->odTables = odt;\n"),
]
if len(sys.argv) > 2 and sys.argv[2] == "nop":  # + 64 wait states between the row pass and the pattern loads
    reps.append(("    float pat[16];  // pattern points",
                 "    __builtin_amdgcn_sched_barrier(0);\n    asm volatile(\"s_nop 7\\n\\ts_nop 7\\n\\ts_nop 7\\n\\ts_nop 7\\n\\ts_nop 7\\n\\ts_nop 7\\n\\ts_nop 7\\n\\ts_nop 7\" ::: \"memory\");\n    __builtin_amdgcn_sched_barrier(0);\n    float pat[16];  // pattern points"))
LOADLINE = "        const f32x4v f = OD_LD(f32x4v, patf, 16u * (4u * (uint32_t)lane + q));"
mode = sys.argv[2] if len(sys.argv) > 2 else ""
if mode in ("sc", "asmwait"):  # the pattern loads as asm (sc: with sc0 sc1, no L1 / TCP hit), waited inside it
    reps[4] = (reps[4][0], reps[4][1].replace(LOADLINE,
        "        f32x4v f;\n        asm volatile(\"global_load_dwordx4 %0, %1, %2" + (" sc0 sc1" if mode == "sc" else "") + "\\n\\ts_waitcnt vmcnt(0)\" : \"=v\"(f) : \"v\"(16u * (4u * (uint32_t)lane + q)), \"s\"(tb.patf) : \"memory\");"))
elif mode == "dw":  # four dword loads per float4 instead of one dwordx4 (asm: not re-merged), waited in the asm
    reps[4] = (reps[4][0], reps[4][1].replace(LOADLINE,
        "        f32x4v f;\n        asm volatile(\"global_load_dword %0, %4, %5\\n\\tglobal_load_dword %1, %4, %5 offset:4\\n\\t"
        "global_load_dword %2, %4, %5 offset:8\\n\\tglobal_load_dword %3, %4, %5 offset:12\\n\\ts_waitcnt vmcnt(0)\" "
        ": \"=&v\"(f.x), \"=&v\"(f.y), \"=&v\"(f.z), \"=&v\"(f.w) : \"v\"(16u * (4u * (uint32_t)lane + q)), \"s\"(tb.patf) : \"memory\");"))
elif mode == "malloc":  # the pattern copied to a hipMalloc buffer (not the code object's segment)
    reps[7] = (reps[7][0], reps[7][1] + "    { void* pm = nullptr; HIP_TRY(hipMalloc(&pm, 4096)); HIP_TRY(hipMemcpy(pm, odt.patf, 4096, hipMemcpyDeviceToDevice)); odt.patf = (const float4*)pm; }\n")
elif mode == "drainexit":  # E1: waves without a keypoint drain their loads before they end
    reps.append(("    if (!active) return;", "    if (!active) {\n        asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n        return;\n    }"))
elif mode == "prewait":  # E2: compiler-placed pattern loads, every wave waits for them before the barrier
    reps.append(("    lds_barrier();  // s_trig is written", "    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n    lds_barrier();  // s_trig is written"))
elif mode == "probe":  # record every pattern register that differs from the table, after the second barrier
    reps.append(("struct ODTables {", "__device__ uint32_t g_odp[8 * 512];\n__device__ uint32_t g_odpn;\nstruct ODTables {"))
    reps.append(("    lds_barrier();  // s_trig is written (and the row-pass sums: LDS)\n    if (!active) return;",
        "    lds_barrier();  // s_trig is written (and the row-pass sums: LDS)\n"
        "    if (active) {\n"
        "        asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n"
        "#pragma unroll\n"
        "        for (int q = 0; q < 4; ++q) {\n"
        "            float4 gg;\n"
        "            asm volatile(\"global_load_dwordx4 %0, %1, %2 sc0 sc1\\n\\ts_waitcnt vmcnt(0)\" : \"=v\"(gg) : \"v\"(16u * (4u * (uint32_t)lane + q)), \"s\"(tb.patf) : \"memory\");\n"
        "            if (gg.x != pat[4 * q] || gg.y != pat[4 * q + 1] || gg.z != pat[4 * q + 2] || gg.w != pat[4 * q + 3]) {\n"
        "                const uint32_t i = atomicAdd(&g_odpn, 1u);\n"
        "                if (i < 512) {\n"
        "                    uint32_t* o = g_odp + 8 * i;\n"
        "                    o[0] = ((uint32_t)wave << 16) | ((uint32_t)lane << 8) | (uint32_t)q; o[1] = (uint32_t)k; o[2] = (uint32_t)b;\n"
        "                    o[3] = __float_as_uint(pat[4 * q]); o[4] = __float_as_uint(pat[4 * q + 1]);\n"
        "                    o[5] = __float_as_uint(pat[4 * q + 2]); o[6] = __float_as_uint(pat[4 * q + 3]); o[7] = blockIdx.x;\n"
        "                }\n"
        "            }\n"
        "        }\n"
        "    }\n"
        "    if (!active) return;"))
    reps.append(("int orb_debug_kf_timing(unsigned long long* out6) {",
        "extern \"C\" int orb_variant_odp(uint32_t* out, int n) {\n"
        "    uint32_t cnt = 0;\n"
        "    HIP_TRY(hipDeviceSynchronize());\n"
        "    HIP_TRY(hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(g_odpn), 4));\n"
        "    if (out && n > 0) HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_odp), 4u * 8u * (uint32_t)std::min(n, 512)));\n"
        "    const uint32_t z = 0;\n"
        "    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_odpn), &z, 4));\n"
        "    return (int)cnt;\n"
        "}\n"
        "int orb_debug_kf_timing(unsigned long long* out6) {"))
elif mode == "trig3":  # the workgroup's angle arithmetic on wave 3 instead of wave 0
    reps.append(("    if (wave == 0 && lane < OD_WAVES) {", "    if (wave == 3 && lane < OD_WAVES) {"))
elif mode == "nof64":  # (wrong output) the angle's sin / cos by a float polynomial: no f64 in the trig wave
    reps.append(("        glibc_sincosf(ang * factorPI, &sa, &ca);",
                 "        { const float xx = ang * factorPI - 3.14159265f, x2 = xx * xx; sa = -xx * (1.f - x2 * (1.f / 6.f - x2 * (1.f / 120.f))); ca = -(1.f - x2 * (0.5f - x2 * (1.f / 24.f))); }"))
elif mode == "nodiv":  # (wrong output) fastAtan2 without its division (no v_div_scale / v_rcp in the trig wave)
    reps.append(("        const float ang = fast_atan2((float)mm.x, (float)mm.y);",
                 "        const float ang = fminf(fabsf((float)mm.x * 1e-3f + (float)mm.y * 2e-3f), 359.f);"))
elif mode == "notrig":  # (wrong output) no angle arithmetic at all: a constant angle of each slot's moments
    reps.append(("        const float ang = fast_atan2((float)mm.x, (float)mm.y);",
                 "        const float ang = fminf(fabsf((float)mm.x * 1e-3f + (float)mm.y * 2e-3f), 359.f);"))
    reps.append(("        glibc_sincosf(ang * factorPI, &sa, &ca);", "        sa = ang * 1e-3f; ca = 1.f - sa;"))
assert LOADLINE in reps[4][1] or mode in ("sc", "asmwait", "dw")
args = ["python3", "scripts/ablation_variant.py", sys.argv[1]]
for a, b in reps:
    args += [a, b]
sys.exit(subprocess.call(args))
