// CPU check of the emission's quadrant mask (dge_amd/csrc/gs_qmask.h): for random Gaussians around a
// tile, every quadrant that some pixel blends (the oracle's per-pixel skip tests, forward.cu:336-348,
// with the blend's exp: oracle/gs_oracle.c go_expf) must have its bit set.  Test infrastructure
// (tests/test_qmask.py builds and runs it).  Prints the case count, misses (must be 0) and the
// over-kept fraction (bits set where no pixel passes: cost only).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../dge_amd/csrc/gs_qmask.h"

extern "C" void go_expf(int n, const float* x, float* y);

// (comparison only) the blend's per-quadrant bound, dge_amd/csrc/gs_common.h cull_keep, on the host
static bool cull_keep_host(float gx, float gy, float a, float b, float c, float o, float bx0, float by0) {
    if (o < 1.0f / 255.0f) return false;
    if (!(a > 0.f && c > 0.f && a * c - b * b > 0.f)) return true;
    const float thr = (2.0f * 0.693147182f) * log2f(255.0f * o);
    const float X0 = gx - (bx0 + 7.0f), X1 = gx - bx0, Y0 = gy - (by0 + 7.0f), Y1 = gy - by0;
    if (X0 <= 0.f && X1 >= 0.f && Y0 <= 0.f && Y1 >= 0.f) return true;
    const float slack = 2e-3f * (1.0f + fabsf(thr));
    const float rc = 1.0f / c, ra = 1.0f / a;
    float qmin = 0.f;
    for (int e = 0; e < 2; ++e) {
        const float X = e ? X1 : X0;
        const float dy = fminf(Y1, fmaxf(Y0, (-b * X) * rc));
        const float t1 = a * X * X, t2 = 2.f * b * X * dy, t3 = c * dy * dy;
        const float q = (t1 + t2 + t3) - 1e-5f * (t1 + fabsf(t2) + t3);
        qmin = e ? fminf(qmin, q) : q;
    }
    for (int e = 0; e < 2; ++e) {
        const float Y = e ? Y1 : Y0;
        const float dx = fminf(X1, fmaxf(X0, (-b * Y) * ra));
        const float t1 = a * dx * dx, t2 = 2.f * b * dx * Y, t3 = c * Y * Y;
        qmin = fminf(qmin, (t1 + t2 + t3) - 1e-5f * (t1 + fabsf(t2) + t3));
    }
    return qmin <= thr + slack;
}

int main(int argc, char** argv) {
    const long cases = argc > 1 ? atol(argv[1]) : 200000;
    std::mt19937_64 rng(argc > 2 ? atoll(argv[2]) : 1);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    long misses = 0, set = 0, needed = 0, degenerate = 0, cull_set = 0, cull_miss = 0, aabb_set = 0;
    float pw[256], G[256];
    for (long n = 0; n < cases; ++n) {
        // tile origin: small and large image coordinates (c4: 1920 x 1080)
        const float tx0 = 16.0f * (float)(n % 3 == 0 ? 0 : n % 3 == 1 ? 37 : 119);
        const float ty0 = 16.0f * (float)(n % 5 == 0 ? 0 : n % 5 < 3 ? 21 : 67);
        // 2D covariance: random axes (log-uniform sigma 0.05 .. 200 px), angle, + the EWA 0.3
        const float s1 = expf(logf(0.05f) + U(rng) * logf(4000.0f)), s2 = expf(logf(0.05f) + U(rng) * logf(4000.0f));
        const float th = 6.2831853f * U(rng);
        const float cs = cosf(th), sn = sinf(th);
        float c00 = s1 * s1 * cs * cs + s2 * s2 * sn * sn + 0.3f;
        float c11 = s1 * s1 * sn * sn + s2 * s2 * cs * cs + 0.3f;
        float c01 = (s1 * s1 - s2 * s2) * cs * sn;
        if (n % 97 == 0) c01 = (U(rng) < 0.5f ? 1.0f : -1.0f) * sqrtf(c00 * c11) * (1.0f - 1e-6f * U(rng));
        const float det = c00 * c11 - c01 * c01;
        if (!(det > 0.0f)) { ++degenerate; continue; }
        const float a = c11 / det, b = -c01 / det, c = c00 / det;  // conic (forward.cu:223-226)
        // centre: around the tile, reach scaled with the footprint
        const float reach = 3.0f * fmaxf(s1, s2) + 8.0f;
        const float gx = tx0 + 8.0f + (2.0f * U(rng) - 1.0f) * reach, gy = ty0 + 8.0f + (2.0f * U(rng) - 1.0f) * reach;
        // opacity: log-uniform over [1e-3, 1], or at the 1/255 threshold
        float o = n % 7 == 0 ? (1.0f / 255.0f) * (1.0f + 1e-3f * (2.0f * U(rng) - 1.0f))
                             : expf(logf(1e-3f) + U(rng) * -logf(1e-3f));
        if (n % 11 == 0) o = 0.99f + 0.01f * U(rng);
        const gs::QuadCull qc = gs::quad_cull_setup(gx, gy, a, b, c, o);
        const uint32_t m = gs::quad_mask(qc, tx0, ty0);
        // the blend's test at every pixel of the four quadrants
        for (int q = 0; q < 4; ++q)
            for (int p = 0; p < 64; ++p) {
                const float px = tx0 + 8.0f * (float)(q & 1) + (float)(p & 7);
                const float py = ty0 + 8.0f * (float)(q >> 1) + (float)(p >> 3);
                const float dx = gx - px, dy = gy - py;
                pw[q * 64 + p] = -0.5f * (a * dx * dx + c * dy * dy) - b * dx * dy;
            }
        go_expf(256, pw, G);
        for (int q = 0; q < 4; ++q) {
            bool any = false;
            for (int p = 0; p < 64 && !any; ++p) {
                const float power = pw[q * 64 + p];
                const float alpha = fminf(0.99f, o * G[q * 64 + p]);
                any = !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
            }
            const bool bit = (m >> q) & 1u;
            needed += any;
            set += bit;
            const bool ck = cull_keep_host(gx, gy, a, b, c, o, tx0 + 8.0f * (float)(q & 1), ty0 + 8.0f * (float)(q >> 1));
            cull_set += ck;
            {  // (comparison only) the ellipse's bounding box against the quadrant box
                const float bx0 = tx0 + 8.0f * (float)(q & 1), by0 = ty0 + 8.0f * (float)(q >> 1);
                const bool ab = qc.all || (qc.dyE >= 0.0f && gx + qc.dxE >= bx0 && gx - qc.dxE <= bx0 + 7.0f &&
                                           gy + qc.dyE >= by0 && gy - qc.dyE <= by0 + 7.0f);
                aabb_set += ab;
            }
            cull_miss += any && !ck;
            if (any && !bit) {
                if (++misses <= 10)
                    printf("MISS case %ld q %d: g (%.6g, %.6g) conic (%.6g, %.6g, %.6g) o %.6g tile (%g, %g) mask %x\n", n,
                           q, gx, gy, a, b, c, o, tx0, ty0, m);
            }
        }
    }
    // the per-rect form (the preprocess's word) against quad_mask tile by tile
    long rect_cases = 0, rect_diff = 0;
    for (long n = 0; n < cases / 4; ++n) {
        const int w = 1 + (int)(U(rng) * gs::kBandMaxW), h = 1 + (int)(U(rng) * gs::kBandMaxH);
        const int x0 = (int)(U(rng) * 100.0f), y0 = (int)(U(rng) * 60.0f);
        const float s1 = expf(logf(0.3f) + U(rng) * logf(100.0f)), s2 = expf(logf(0.3f) + U(rng) * logf(100.0f));
        const float th = 6.2831853f * U(rng), cs = cosf(th), sn = sinf(th);
        const float c00 = s1 * s1 * cs * cs + s2 * s2 * sn * sn + 0.3f, c11 = s1 * s1 * sn * sn + s2 * s2 * cs * cs + 0.3f;
        const float c01 = (s1 * s1 - s2 * s2) * cs * sn, det = c00 * c11 - c01 * c01;
        if (!(det > 0.0f)) continue;
        const float gx = 16.0f * x0 + U(rng) * 16.0f * w, gy = 16.0f * y0 + U(rng) * 16.0f * h;
        const gs::QuadCull qc = gs::quad_cull_setup(gx, gy, c11 / det, -c01 / det, c00 / det, 0.004f + U(rng));
        const uint64_t word = gs::rect_band_ranges(qc, x0, y0, w, h);
        for (int j = 0; j < h; ++j)
            for (int i = 0; i < w; ++i) {
                const uint32_t t = gs::quad_mask(qc, 16.0f * (x0 + i), 16.0f * (y0 + j));
                rect_diff += gs::band_inst_mask(word, i, j) != t;
            }
        ++rect_cases;
    }
    printf("rect_cases %ld rect_mismatches %ld\n", rect_cases, rect_diff);
    if (rect_diff) misses += rect_diff;
    printf("cases %ld degenerate %ld quadrants_needed %ld bits_set %ld misses %ld overkept %.4f (cull_keep: %ld kept, "
           "overkept %.4f, misses %ld) (bounding box: %ld kept)\n", cases, degenerate, needed, set, misses, set ? (double)(set - needed) / (double)set : 0.0,
           cull_set, cull_set ? (double)(cull_set - needed) / (double)cull_set : 0.0, cull_miss, aabb_set);
    return misses ? 1 : 0;
}
