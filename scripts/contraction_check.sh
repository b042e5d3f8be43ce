#!/bin/bash
# Evidence for the FMA contraction pattern the oracle and the HIP kernels write explicitly:
# the reference matcher/geometry expression SHAPES (ORBmatcher.cc:136-153, 540-555,
# 1536-1545, 1648-1657, 321-333; Frame.cc:150-155), re-typed as minimal functions, compiled
# as the reference build compiles them (g++ -O3 -march=native, CMakeLists.txt:13; -mavx2
# -mfma here) and disassembled.  Read: vfmadd231ss X,Y,Z = Z + X*Y; vfmadd213ss M,X,Y = X*Y+M.
set -e
T=$(mktemp -d)
cat > $T/shapes.cpp <<'CPP'
struct K { float x, y; };
float proj_u(float fx, float X, float invz, float cx) { return fx * X * invz + cx; }            // isInFrustum / SBP
float proj_u2(float fx, float X, float invz, float cx) { const float x = X * invz; return fx * x + cx; }  // Fuse / Sim3
bool epi(const K& kp1, const K& kp2, const float* F12, float s2, float* o) {                    // CheckDistEpipolarLine
    const float a = kp1.x * F12[0] + kp1.y * F12[3] + F12[6];
    const float b = kp1.x * F12[1] + kp1.y * F12[4] + F12[7];
    const float c = kp1.x * F12[2] + kp1.y * F12[5] + F12[8];
    const float num = a * kp2.x + b * kp2.y + c;
    const float den = a * a + b * b;
    if (den == 0) return false;
    const float dsqr = num * num / den;
    o[0] = a; o[1] = b; o[2] = c; o[3] = num; o[4] = den;
    return dsqr < 3.84 * s2;
}
CPP
g++ -O3 -mavx2 -mfma -c -o $T/shapes.o $T/shapes.cpp
objdump -d --no-show-raw-insn -C $T/shapes.o | grep -E "^[0-9a-f]+ <|vfm|vmul|vadd|vdiv"
rm -rf $T
