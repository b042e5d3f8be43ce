/*
 * Deterministic synthetic grayscale frames for the ORB front end.
 *
 * A stream is a static scene (background + 200 filled rectangles + 100 filled discs,
 * intensities U[0,255], sizes 8..120 px) rendered on a canvas 2*SYN_PAD larger than the
 * frame.  Frame t of the stream is a W x H crop of that canvas at an offset that random-
 * walks by an integer (dx, dy) in [-6, 6]^2 per frame, plus fresh per-pixel uniform noise
 * in [-8, 8], clamped to [0, 255].  Consecutive frames therefore overlap by construction
 * and SearchForInitialization (window 100) finds matches.  RNG: splitmix64 seeded with
 * 1234 + 1000003*stream + frame.  The reference ships no test images, so
 * these frames are the inputs for parity tests and for bench.py.
 *
 * Special frames exercise the edge cases the reference's code paths have:
 *   SYN_FLAT   all 128                 -> no corners, N = 0 (descriptor release path)
 *   SYN_LOWTEX smooth ramp + faint blobs -> cells with <=3 corners at th=20 (th=7 re-run)
 *   SYN_NOISE  uniform noise           -> saturated cells, many score ties
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SYN_PAD 128

enum { SYN_SCENE = 0, SYN_FLAT = 1, SYN_LOWTEX = 2, SYN_NOISE = 3 };

static inline uint64_t splitmix64(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline int rnd_int(uint64_t* s, int lo, int hi) { /* inclusive */
    return lo + (int)(splitmix64(s) % (uint64_t)(hi - lo + 1));
}

static uint64_t seed_of(uint64_t stream, uint64_t frame) { return 1234ull + 1000003ull * stream + frame; }

static void render_scene(uint8_t* canvas, int cw, int ch, uint64_t stream) {
    uint64_t s = seed_of(stream, 0) ^ 0x5CE7E5CE7Eull;
    int bg = rnd_int(&s, 40, 215);
    memset(canvas, bg, (size_t)cw * ch);
    for (int k = 0; k < 200; ++k) {
        int w = rnd_int(&s, 8, 120), h = rnd_int(&s, 8, 120);
        int x0 = rnd_int(&s, -w / 2, cw - w / 2), y0 = rnd_int(&s, -h / 2, ch - h / 2);
        int v = rnd_int(&s, 0, 255);
        for (int y = y0 < 0 ? 0 : y0; y < y0 + h && y < ch; ++y)
            for (int x = x0 < 0 ? 0 : x0; x < x0 + w && x < cw; ++x) canvas[(size_t)y * cw + x] = (uint8_t)v;
    }
    for (int k = 0; k < 100; ++k) {
        int d = rnd_int(&s, 8, 120), r = d / 2;
        int cx = rnd_int(&s, 0, cw - 1), cy = rnd_int(&s, 0, ch - 1);
        int v = rnd_int(&s, 0, 255);
        for (int y = cy - r; y <= cy + r; ++y) {
            if (y < 0 || y >= ch) continue;
            for (int x = cx - r; x <= cx + r; ++x) {
                if (x < 0 || x >= cw) continue;
                if ((x - cx) * (x - cx) + (y - cy) * (y - cy) <= r * r) canvas[(size_t)y * cw + x] = (uint8_t)v;
            }
        }
    }
}

static void add_noise_crop(const uint8_t* canvas, int cw, int ox, int oy, int W, int H, uint8_t* out, int stride,
                           uint64_t seed) {
    uint64_t s = seed;
    for (int y = 0; y < H; ++y) {
        const uint8_t* src = canvas + (size_t)(y + oy) * cw + ox;
        uint8_t* dst = out + (size_t)y * stride;
        int x = 0;
        while (x < W) {
            uint64_t bits = splitmix64(&s);
            for (int b = 0; b < 8 && x < W; ++b, ++x) {
                int n = (int)((bits >> (8 * b)) & 0xFF) % 17 - 8;
                int v = src[x] + n;
                dst[x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
            }
        }
    }
}

/* Offset of frame t in the canvas: a clamped random walk starting at the centre. */
static void frame_offset(uint64_t stream, uint64_t frame, int* ox, int* oy) {
    int x = SYN_PAD, y = SYN_PAD;
    for (uint64_t t = 1; t <= frame; ++t) {
        uint64_t s = seed_of(stream, t) ^ 0x0FF5E7ull;
        x += rnd_int(&s, -6, 6);
        y += rnd_int(&s, -6, 6);
        if (x < 0) x = -x;
        if (y < 0) y = -y;
        if (x > 2 * SYN_PAD) x = 4 * SYN_PAD - x;
        if (y > 2 * SYN_PAD) y = 4 * SYN_PAD - y;
    }
    *ox = x;
    *oy = y;
}

/* Frames [first, first+count) of `stream`, each W x H at `stride`, frame-major in `out`
 * (frame k at out + k*frame_pitch).  Returns 0, or -22 on bad arguments, -12 on OOM. */
int orb_synth_stream(int W, int H, uint64_t stream, uint64_t first, int count, uint8_t* out, int stride,
                     int64_t frame_pitch) {
    if (W <= 0 || H <= 0 || count < 0 || stride < W || frame_pitch < (int64_t)stride * H) return -22;
    int cw = W + 2 * SYN_PAD, ch = H + 2 * SYN_PAD;
    uint8_t* canvas = (uint8_t*)malloc((size_t)cw * ch);
    if (!canvas) return -12;
    render_scene(canvas, cw, ch, stream);
    for (int k = 0; k < count; ++k) {
        int ox, oy;
        frame_offset(stream, first + (uint64_t)k, &ox, &oy);
        add_noise_crop(canvas, cw, ox, oy, W, H, out + (size_t)k * frame_pitch, stride,
                       seed_of(stream, first + (uint64_t)k));
    }
    free(canvas);
    return 0;
}

/* One special edge-case frame (SYN_FLAT / SYN_LOWTEX / SYN_NOISE); SYN_SCENE = frame 0 of stream `seed`. */
int orb_synth_special(int kind, int W, int H, uint64_t seed, uint8_t* out, int stride) {
    if (W <= 0 || H <= 0 || stride < W) return -22;
    uint64_t s = seed_of(seed, 0) ^ 0xED6Eull;
    switch (kind) {
    case SYN_SCENE:
        return orb_synth_stream(W, H, seed, 0, 1, out, stride, (int64_t)stride * H);
    case SYN_FLAT:
        for (int y = 0; y < H; ++y) memset(out + (size_t)y * stride, 128, W);
        return 0;
    case SYN_LOWTEX: {
        /* gentle ramp, a few faint blobs (contrast 9..14 -> corners only at th=7) */
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) out[(size_t)y * stride + x] = (uint8_t)(96 + (x + y) * 32 / (W + H));
        for (int k = 0; k < 60; ++k) {
            int w = rnd_int(&s, 6, 30), h = rnd_int(&s, 6, 30);
            int x0 = rnd_int(&s, 0, W - 1), y0 = rnd_int(&s, 0, H - 1);
            int dv = rnd_int(&s, 9, 14) * (rnd_int(&s, 0, 1) ? 1 : -1);
            for (int y = y0; y < y0 + h && y < H; ++y)
                for (int x = x0; x < x0 + w && x < W; ++x) {
                    int v = out[(size_t)y * stride + x] + dv;
                    out[(size_t)y * stride + x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
                }
        }
        return 0;
    }
    case SYN_NOISE:
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) out[(size_t)y * stride + x] = (uint8_t)(splitmix64(&s) & 0xFF);
        return 0;
    default:
        return -22;
    }
}
