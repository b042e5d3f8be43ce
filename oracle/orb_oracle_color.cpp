// orb_oracle_color.cpp — TEST INFRASTRUCTURE ONLY (CPU parity checker; never linked by the product).
//
// Tracking::GrabImage's colour conversion (reference src/Tracking.cc:202-207:
// cvtColor(image, im, mbRGB ? CV_RGB2GRAY : CV_BGR2GRAY)) for 8-bit frames, as OpenCV 2.4's
// RGB2Gray<uchar> computes it (imgproc color.cpp, not vendored): three tables i*coeff with the
// rounding constant 1 << (yuv_shift-1) folded into the third, summed and shifted by
// yuv_shift = 14; R2Y = 4899, G2Y = 9617, B2Y = 1868; blue index 0 for BGR, 2 for RGB.
// Parity against a real OpenCV 2.4 binary is unpinned (none here); pinned by the known
// answers 76 / 150 / 29 for pure red / green / blue and gray -> gray (tests/test_color_ingest.py).
#include <cstdint>

#include "orb_oracle.h"

extern "C" int oracle_rgb_to_gray(const uint8_t* src, int w, int h, int stride, int cn, int rgb, uint8_t* dst) {
    const int yuv_shift = 14, R2Y = 4899, G2Y = 9617, B2Y = 1868;
    const int coeffs0[] = {R2Y, G2Y, B2Y};
    const int blueIdx = rgb ? 2 : 0;
    int tab[256 * 3];
    int b = 0, g = 0, r = 1 << (yuv_shift - 1);
    const int db = coeffs0[blueIdx ^ 2], dg = coeffs0[1], dr = coeffs0[blueIdx];
    for (int i = 0; i < 256; i++, b += db, g += dg, r += dr) {
        tab[i] = b;
        tab[i + 256] = g;
        tab[i + 512] = r;
    }
    for (int y = 0; y < h; ++y) {
        const uint8_t* s = src + (int64_t)y * stride;
        for (int x = 0; x < w; ++x, s += cn)
            dst[(int64_t)y * w + x] = (uint8_t)((tab[s[0]] + tab[s[1] + 256] + tab[s[2] + 512]) >> yuv_shift);
    }
    return 0;
}
