/*
 * pt_texture.h — the framework's deterministic definition of the reference's texture fetch,
 * shared by the HIP kernels and the CPU oracle (like pt_libm.h), so both return the SAME bits.
 *
 * The reference samples with tex2D<float4> on a cudaArray of uchar4 (pathtrace.cu:110-133,
 * 505-519): normalized coordinates, cudaAddressModeWrap, cudaFilterModeLinear,
 * cudaReadModeNormalizedFloat.  The CUDA C Programming Guide ("Texture Fetching") defines
 * that fetch as: wrap replaces x by frac(x); xB = x*W - 0.5, i = floor(xB), alpha = frac(xB)
 * held in 9-bit fixed point with 8 fractional bits (same for y / beta); result =
 * (1-a)(1-b)T[i,j] + a(1-b)T[i+1,j] + (1-a)bT[i,j+1] + abT[i+1,j+1], indices wrapping, texels
 * read as T/255.  The hardware's blend precision is unspecified, so this restatement blends
 * EXACTLY in integers with the 8-bit weights (round-to-nearest quantization) and rounds once
 * to float.  Parity with an NVIDIA GPU's texture unit is therefore unpinned (documented in
 * DESIGN.md); parity between this framework's kernels and its oracle is bit-exact.
 */
#ifndef PT_TEXTURE_H
#define PT_TEXTURE_H

#include <stdint.h>

#include "pt_libm.h"   /* PT_LIBM_FN */

/* one texture: RGBA8 texels, row 0 = first image row (stbi order), width x height */
PT_LIBM_FN void pt_tex_axis(float x, int n, int* i0, int* i1, int* w8) {
    if (!(x - x == 0.0f)) x = 0.0f;                 /* NaN / inf coordinate: treated as 0 */
    float fx = x - __builtin_floorf(x);              /* cudaAddressModeWrap */
    float xb = fx * (float)n - 0.5f;
    float fi = __builtin_floorf(xb);
    int i = (int)fi;
    int w = (int)__builtin_floorf((xb - fi) * 256.0f + 0.5f);   /* 8 fractional bits, [0, 256] */
    i = i % n;
    if (i < 0) i += n;
    int j = i + 1;
    if (j >= n) j -= n;
    *i0 = i;
    *i1 = j;
    *w8 = w;
}

/* tex2D<float4>(tex, u, v) -> out[4] (callers pass v = 1 - uv.y like the reference) */
PT_LIBM_FN void pt_tex2d(const uint32_t* texels, int width, int height, float u, float v, float out[4]) {
    int i0, i1, wa, j0, j1, wb;
    pt_tex_axis(u, width, &i0, &i1, &wa);
    pt_tex_axis(v, height, &j0, &j1, &wb);
    const uint32_t t00 = texels[(int64_t)j0 * width + i0], t10 = texels[(int64_t)j0 * width + i1];
    const uint32_t t01 = texels[(int64_t)j1 * width + i0], t11 = texels[(int64_t)j1 * width + i1];
    const int w00 = (256 - wa) * (256 - wb), w10 = wa * (256 - wb), w01 = (256 - wa) * wb, w11 = wa * wb;
    for (int c = 0; c < 4; ++c) {
        const int sh = 8 * c;                        /* little-endian RGBA8: r in the low byte */
        const int s = w00 * (int)((t00 >> sh) & 255u) + w10 * (int)((t10 >> sh) & 255u) +
                      w01 * (int)((t01 >> sh) & 255u) + w11 * (int)((t11 >> sh) & 255u);
        out[c] = (float)s / 16711680.0f;             /* / (65536 * 255): exact int, one rounding */
    }
}

#endif /* PT_TEXTURE_H */
