/*
 * wcpt_composite.h — the display step after the path: composite.comp:3-54.
 *
 * Gamma 1/2.2 then the PBR Neutral tonemap, per pixel of the float4 accumulation image. Shared by the HIP kernel
 * (pt_composite.hip) and the CPU oracle (oracle/pt_oracle.c), so both compute the identical binary32 sequence
 * (compiled with -ffp-contract=off). GLSL leaves pow's precision to the driver ("inherited from exp2 and log2");
 * here pow(x, y) = exp(y * log(x)) with the deterministic log/exp of wcpt_libm.h. The bloom input of
 * composite.comp:44-45 is never dispatched by the reference host and is not part of this step.
 */
#ifndef WCPT_COMPOSITE_H
#define WCPT_COMPOSITE_H

#include "wcpt_libm.h"

/* composite.comp:3-23 Tonemap_PBRNeutral, in place on (r, g, b) */
WCPT_HD void wcpt_tonemap_pbr_neutral(float* r, float* g, float* b)
{
    const float startCompression = 0.8f - 0.04f;
    const float desaturation = 0.15f;
    const float x = fminf(*r, fminf(*g, *b));
    const float offset = x < 0.08f ? x - 6.25f * x * x : 0.04f;
    *r -= offset;
    *g -= offset;
    *b -= offset;
    const float peak = fmaxf(*r, fmaxf(*g, *b));
    if (peak < startCompression) return;
    const float d = 1.0f - startCompression;
    const float newPeak = 1.0f - d * d / (peak + d - startCompression);
    const float scale = newPeak / peak;
    *r *= scale;
    *g *= scale;
    *b *= scale;
    const float gm = 1.0f - 1.0f / (desaturation * (peak - newPeak) + 1.0f);
    const float ig = 1.0f - gm; /* mix(color, newPeak, g) = color * (1 - g) + newPeak * g */
    *r = *r * ig + newPeak * gm;
    *g = *g * ig + newPeak * gm;
    *b = *b * ig + newPeak * gm;
}

/* pow(x, y) for the gamma step: exp(y * log(x)) (x = 0 -> 0, x < 0 -> NaN) */
WCPT_HD float wcpt_powf(float x, float y) { return wcpt_expf(y * wcpt_logf(x)); }

/* composite.comp:36-53 for one texel: the sample at the texel centre is the texel itself (same size) */
WCPT_HD void wcpt_composite_texel(const float in[4], float out[4])
{
    const float inv_gamma = 1.0f / 2.2f;
    float r = wcpt_powf(in[0], inv_gamma);
    float g = wcpt_powf(in[1], inv_gamma);
    float b = wcpt_powf(in[2], inv_gamma);
    wcpt_tonemap_pbr_neutral(&r, &g, &b);
    out[0] = r;
    out[1] = g;
    out[2] = b;
    out[3] = 1.0f;
}

/* Vulkan float -> UNORM8 conversion (round to nearest after clamping to [0, 1]; NaN -> 0) */
WCPT_HD unsigned char wcpt_unorm8(float v)
{
    if (!(v > 0.0f)) return 0;
    if (v >= 1.0f) return 255;
    return (unsigned char)(int)(v * 255.0f + 0.5f);
}

#endif
