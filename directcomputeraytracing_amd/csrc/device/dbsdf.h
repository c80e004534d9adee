// dbsdf.h -- BxDF stack on the device: Lambert, GGX (VNDF) Cook-Torrance BRDF
// and BSDF, specular BRDF/BSDF, Kulla-Conty multiscattering and the
// EvaluateBSDF / EvaluateBSDFPdf / SampleBSDF dispatch of BSDFs.inc.hlsl.
#pragma once

#include "dscene.h"

namespace dcrt {
namespace dev {

struct LCtx { V3 H; float WOdotH; };   // LightingContext.inc.hlsl
DEV void calc_h(V3 wo, V3 wi, LCtx& c)
{
    c.H = wi + wo;
    c.H = all_zero(c.H) ? mk(0.0f, 0.0f, 0.0f) : normalize(c.H);
    c.WOdotH = dot(c.H, wo);
}

// Fresnel.inc.hlsl:4-63
DEV float fresnel_dielectric(float cosThetaI, float etaO, float etaI)
{
    cosThetaI = fminf(fmaxf(cosThetaI, -1.0f), 1.0f);
    if (cosThetaI < 0.0f) { const float t = etaO; etaO = etaI; etaI = t; cosThetaI = -cosThetaI; }
    const float sinThetaI = sqrtf(1.0f - cosThetaI * cosThetaI);
    const float sinThetaT = etaO / etaI * sinThetaI;
    if (sinThetaT >= 1.0f) return 1.0f;
    const float cosThetaT = sqrtf(1.0f - sinThetaT * sinThetaT);
    const float Rparl = ((etaI * cosThetaI) - (etaO * cosThetaT)) / ((etaI * cosThetaI) + (etaO * cosThetaT));
    const float Rperp = ((etaO * cosThetaI) - (etaI * cosThetaT)) / ((etaO * cosThetaI) + (etaI * cosThetaT));
    return (Rparl * Rparl + Rperp * Rperp) * 0.5f;
}
DEV float fresnel_conductor1(float cosThetaI, float etaI, float k)   // etaO = 1
{
    cosThetaI = fminf(fmaxf(cosThetaI, -1.0f), 1.0f);
    const float eta = etaI / 1.0f;
    const float etak = k / 1.0f;
    const float c2 = cosThetaI * cosThetaI;
    const float s2 = 1.0f - c2;
    const float eta2 = eta * eta;
    const float etak2 = etak * etak;
    const float t0 = eta2 - etak2 - s2;
    const float a2plusb2 = sqrtf(fmaxf(0.0f, t0 * t0 + 4.0f * eta2 * etak2));
    const float t1 = a2plusb2 + c2;
    const float a = sqrtf(fmaxf(0.0f, 0.5f * (a2plusb2 + t0)));
    const float t2 = 2.0f * cosThetaI * a;
    const float Rs = (t1 - t2) / (t1 + t2);
    const float t3 = c2 * a2plusb2 + s2 * s2;
    const float t4 = t2 * s2;
    const float Rp = Rs * (t3 - t4) / (t3 + t4);
    return 0.5f * (Rp + Rs);
}
DEV V3 fresnel_conductor(float c, V3 eta, V3 k)
{
    return mk(fresnel_conductor1(c, eta.x, k.x), fresnel_conductor1(c, eta.y, k.y), fresnel_conductor1(c, eta.z, k.z));
}

// CookTorranceBSDF.inc.hlsl
DEV float g1(float a2, V3 m, V3 w)
{
    if (dot(w, m) * w.z <= 0.0f) return 0.0f;
    const float n = fabsf(w.z);
    const float den = sqrtf(a2 + (1.0f - a2) * n * n) + n;
    return 2.0f * n / den;
}
DEV float g2(V3 wi, V3 wo, V3 m, float alpha) { const float a2 = alpha * alpha; return g1(a2, m, wi) * g1(a2, m, wo); }
DEV float ggx_d(V3 m, float alpha)
{
    const float a2 = alpha * alpha;
    const float c = m.z;
    const float c2 = c * c;
    const float f = c2 * (a2 - 1.0f) + 1.0f;
    const float den = f * f * kPi;
    return a2 / den;
}
DEV V3 sample_vndf(V3 wo, float U1, float U2, float alpha)
{
    const V3 Vh = normalize(mk(alpha * wo.x, alpha * wo.y, wo.z));
    const float lensq = Vh.x * Vh.x + Vh.y * Vh.y;
    V3 T1;
    if (lensq > 0.0f) { const float sl = sqrtf(lensq); T1 = mk(-Vh.y / sl, Vh.x / sl, 0.0f / sl); }
    else T1 = mk(1.0f, 0.0f, 0.0f);
    const V3 T2 = cross(Vh, T1);
    const float r = sqrtf(U1);
    const float phi = 2.0f * kPi * U2;
    float sp, cp;
    det_sincos(phi, &sp, &cp);
    const float t1 = r * cp;
    float t2 = r * sp;
    const float s = 0.5f * (1.0f + Vh.z);
    t2 = (1.0f - s) * sqrtf(1.0f - t1 * t1) + s * t2;
    const V3 Nh = T1 * t1 + T2 * t2 + Vh * sqrtf(fmaxf(0.0f, 1.0f - t1 * t1 - t2 * t2));
    return normalize(mk(alpha * Nh.x, alpha * Nh.y, fmaxf(0.0f, Nh.z)));
}
DEV V3 sample_ndf(float sx, float sy, float alpha)
{
    const float theta = det_atan(alpha * sqrtf(sx / (1.0f - sx)));
    const float phi = 2.0f * kPi * sy;
    float st, ct, sp, cp;
    det_sincos(theta, &st, &ct);
    det_sincos(phi, &sp, &cp);
    return mk(cp * st, sp * st, ct);
}
DEV V3 sample_ggx(bool vndf, V3 wo, float sx, float sy, float alpha) { return vndf ? sample_vndf(wo, sx, sy, alpha) : sample_ndf(sx, sy, alpha); }
DEV float ggx_pdf(bool vndf, V3 wo, V3 m, float alpha)
{
    if (vndf) return ggx_d(m, alpha) * g1(alpha * alpha, m, wo) * fmaxf(0.0f, dot(wo, m)) / wo.z;
    return ggx_d(m, alpha) * fabsf(m.z);
}
DEV float ct_brdf(V3 wi, V3 wo, float alpha, const LCtx& c)
{
    if (wi.z <= 0.0f || wo.z <= 0.0f || c.WOdotH <= 0.0f) return 0.0f;
    if (all_zero(c.H)) return 0.0f;
    return ggx_d(c.H, alpha) * g2(wi, wo, c.H, alpha) / (4.0f * wi.z * wo.z);
}
DEV float ct_brdf_pdf(bool vndf, V3 wi, V3 wo, float alpha, const LCtx& c)
{
    if (wi.z <= 0.0f || wo.z <= 0.0f || c.WOdotH <= 0.0f) return 0.0f;
    return ggx_pdf(vndf, wo, c.H, alpha) / (4.0f * c.WOdotH);
}
template <bool NO_SCALE>
DEV float ct_bsdf(V3 wi, V3 wo, float alpha, float etaO, float etaI)
{
    const bool active = wo.z != 0.0f && wi.z != 0.0f;
    const bool refl = wi.z * wo.z > 0.0f;
    V3 m = normalize(wo * (refl ? 1.0f : etaO) + wi * (refl ? 1.0f : etaI));
    m = m.z < 0.0f ? -m : m;
    const float WIdotM = dot(wi, m), WOdotM = dot(wo, m);
    const float D = ggx_d(m, alpha);
    const float F = fresnel_dielectric(WOdotM, etaO, etaI);
    const float G = g2(wi, wo, m, alpha);
    if (refl) return active ? F * D * G / (4.0f * fabsf(wi.z) * fabsf(wo.z)) : 0.0f;
    const float sd = etaO * WOdotM + etaI * WIdotM;
    const float scale = NO_SCALE ? etaI : etaO;
    const float value = (1.0f - F) * fabsf(D * G * fabsf(WIdotM) * fabsf(WOdotM) * scale * scale / (wo.z * wi.z * sd * sd));
    return active ? value : 0.0f;
}
DEV float ct_bsdf_pdf(bool vndf, V3 wi, V3 wo, float alpha, float etaO, float etaI)
{
    bool active = wo.z != 0.0f && wi.z != 0.0f;
    const bool refl = wi.z * wo.z > 0.0f;
    V3 m = normalize(wo * (refl ? 1.0f : etaO) + wi * (refl ? 1.0f : etaI));
    m = m.z < 0.0f ? -m : m;
    const float WIdotM = dot(wi, m), WOdotM = dot(wo, m);
    active = active && (WIdotM * wi.z > 0.0f && WOdotM * wo.z > 0.0f);
    const float sd = etaO * WOdotM + etaI * WIdotM;
    const float dwh = refl ? 1.0f / (4.0f * WIdotM) : fabsf((etaI * etaI * WIdotM) / (sd * sd));
    const float pdf = ggx_pdf(vndf, wo, m, alpha);
    const float F = fresnel_dielectric(WOdotM, etaO, etaI);
    return active ? pdf * (refl ? F : 1.0f - F) * dwh : 0.0f;
}
DEV V3 ct_bsdf_sample(bool vndf, V3 wo, float sel, float sx, float sy, float alpha, float etaO, float etaI, LCtx& c)
{
    if (wo.z == 0.0f) return mk(0.0f, 0.0f, 0.0f);
    if (etaO == etaI) return -wo;
    const V3 m = sample_ggx(vndf, wo, sx, sy, alpha);
    const float WOdotM = dot(wo, m);
    c.H = m; c.WOdotH = WOdotM;
    if (WOdotM <= 0.0f) return mk(0.0f, 0.0f, 0.0f);
    const float F = fresnel_dielectric(WOdotM, etaO, etaI);
    if (sel < F) return -reflect(wo, m);
    return refract(-wo, m, etaO / etaI);
}

// KullaConty.inc.hlsl
DEV float favg_dielectric(float eta)
{
    const float eta2 = eta * eta;
    return eta >= 1.0f ? (eta - 1.0f) / (4.08567f + 1.00071f * eta)
                       : 0.997118f + 0.1014f * eta - 0.965241f * eta2 - 0.130607f * eta2 * eta;
}
DEV float favg_conductor1(float eta, float k)
{
    const float num = eta * (133.736f - 98.9833f * eta) + k * (eta * (59.5617f - 3.98288f * eta) - 182.37f)
                    + ((0.30818f * eta - 13.1093f) * eta - 62.5919f) * k * k - 8.21474f;
    const float den = k * (eta * (94.6517f - 15.8558f * eta) - 187.166f) + (-78.476f * eta - 395.268f) * eta
                    + (eta * (eta - 15.4387f) - 62.0752f) * k * k;
    return saturate(num / den);
}
DEV float ms_fresnel(float Eavg, float Favg) { return Favg * Favg * Eavg / (1.0f - Favg * (1.0f - Eavg)); }
DEV float ms_bxdf(float Ei, float Eo, float Eavg) { return Eavg < 1.0f ? (1.0f - Ei) * (1.0f - Eo) / (kPi * (1.0f - Eavg)) : 0.0f; }
DEV float ct_ms_bsdf(const DeviceScene& s, V3 wi, float alpha, float ratio, float eta, float Eo, float Eavg, float EavgInv, bool entering)
{
    const float c = fabsf(wi.z);
    if (c == 0.0f) return 0.0f;
    const bool refl = wi.z > 0.0f;
    const float Ei = lut_bsdf(s, c, alpha, eta, refl ? entering : !entering);
    const float factor = refl ? (1.0f - ratio) : ratio;
    return ms_bxdf(Ei, Eo, refl ? Eavg : EavgInv) * factor;
}
DEV float ct_ms_bsdf_pdf(V3 wi, float ratio)
{
    const float c = fabsf(wi.z);
    if (c == 0.0f) return 0.0f;
    float pdf = fabsf(wi.z) * kInvPi;
    pdf = pdf * (wi.z > 0.0f ? 1.0f - ratio : ratio);
    return pdf;
}
DEV float reciprocal_factor(float Fl, float Fe, float El, float Ee, float eta)
{
    const float inv = 1.0f / eta;
    const float f0 = (1.0f - Fl) * (1.0f - El);
    const float f1 = (1.0f - Fe) * (1.0f - Ee) * inv * inv;
    return f1 / fmaxf(0.00001f, f0 + f1);
}
DEV V3 ct_ms_brdf(const DeviceScene& s, V3 wi, V3 wo, float alpha, float Eo, float Eavg, V3 factor)
{
    if (wo.z <= 0.0f || wi.z <= 0.0f) return mk(0.0f, 0.0f, 0.0f);
    const float Ei = lut_brdf(s, wi.z, alpha);
    return factor * ms_bxdf(Ei, Eo, Eavg);
}
DEV float ct_ms_brdf_pdf(V3 wi, V3 wo) { return (wo.z <= 0.0f || wi.z <= 0.0f) ? 0.0f : wi.z * kInvPi; }

DEV float lambert(V3 wi, V3 wo) { return wi.z > 0.0f && wo.z > 0.0f ? kInvPi : 0.0f; }
DEV float lambert_pdf(V3 wi, V3 wo) { return wi.z > 0.0f && wo.z > 0.0f ? wi.z * kInvPi : 0.0f; }

// SpecularBxDF.inc.hlsl
DEV V3 specular_brdf_sample(V3 wo, float* value, float* pdf, LCtx& c)
{
    const V3 wi = mk(-wo.x, -wo.y, wo.z);
    c.H = mk(0.0f, 0.0f, 1.0f); c.WOdotH = wo.z;
    if (wo.z <= 0.0f) return wi;
    *value = 1.0f / wi.z;
    *pdf = 1.0f;
    return wi;
}
template <bool NO_SCALE>
DEV V3 specular_bsdf_sample(V3 wo, float sample, float etaO, float etaI, bool thin, float* value, float* pdf, LCtx& c)
{
    V3 wi = mk(0.0f, 0.0f, 0.0f);
    c.H = mk(0.0f, 0.0f, 1.0f); c.WOdotH = wo.z;
    if (etaO == etaI) { *value = 1.0f / wo.z; *pdf = 1.0f; return -wo; }
    if (wo.z == 0.0f) return wi;
    float F = fresnel_dielectric(wo.z, etaO, etaI);
    float T = 1.0f - F;
    if (thin && F < 1.0f) { F = F + T * T * F / (1.0f - F * F); T = 1.0f - F; }
    if (sample < F) {
        wi = mk(-wo.x, -wo.y, wo.z);
        *value = F / wi.z;
        *pdf = F;
    } else {
        wi = !thin ? refract(-wo, mk(0.0f, 0.0f, 1.0f), etaO / etaI) : -wo;
        if (wi.z == 0.0f) return wi;
        if (NO_SCALE) *value = T / (-wi.z);
        else *value = T * (!thin ? (etaO * etaO) / (etaI * etaI) : 1.0f) / (-wi.z);
        *pdf = T;
    }
    return wi;
}

// ---- BSDFs.inc.hlsl dispatch -----------------------------------------------------
DEV V3 isf_factor(const DeviceScene& s, float alpha, V3 albedo, float ior, uint32_t mode)
{
    if (mode == DCRT_INTERNAL_SCATTERING_IGNORE) return mk(1.0f, 1.0f, 1.0f);
    const float avg = lut_brdf_dielectric_avg(s, alpha, ior, true);
    const float f = 1.0f - avg;
    V3 factor = mk(f, f, f);
    if (mode == DCRT_INTERNAL_SCATTERING_MULTIPLE)
        factor = mk(factor.x / (1.0f - albedo.x * avg), factor.y / (1.0f - albedo.y * avg), factor.z / (1.0f - albedo.z * avg));
    return factor;
}
DEV V3 to_tbn(V3 w, V3 t, V3 b, V3 n) { return mk(dot(w, t), dot(w, b), dot(w, n)); }
DEV V3 from_tbn(V3 w, V3 t, V3 b, V3 n)
{
    return mk(w.x * t.x + w.y * b.x + w.z * n.x, w.x * t.y + w.y * b.y + w.z * n.y, w.x * t.z + w.y * b.z + w.z * n.z);
}
DEV V3 splat(float f) { return mk(f, f, f); }

// Shared multiscattering terms of the rough-dielectric BSDF (BSDFs.inc.hlsl:144-158).
struct DielectricMs { float E, Eavg, EinvAvg, ratio; };
DEV DielectricMs dielectric_ms(const DeviceScene& s, float cosThetaO, float alpha, float ior, bool inverted)
{
    const float EavgEnter = lut_bsdf_avg(s, alpha, ior, true);
    const float FavgEnter = favg_dielectric(1.0f / ior);
    const float EavgLeave = lut_bsdf_avg(s, alpha, ior, false);
    const float FavgLeave = favg_dielectric(ior);
    const float rf = reciprocal_factor(FavgLeave, FavgEnter, EavgLeave, EavgEnter, ior);
    DielectricMs d;
    d.E = lut_bsdf(s, cosThetaO, alpha, ior, inverted);
    const float Favg = inverted ? FavgEnter : FavgLeave;
    d.Eavg = inverted ? EavgEnter : EavgLeave;
    d.EinvAvg = inverted ? EavgLeave : EavgEnter;
    d.ratio = (inverted ? 1.0f - rf : rf) * (1.0f - Favg);
    return d;
}

// Per-hit BSDF frame shared by EvaluateBSDF, EvaluateBSDFPdf and SampleBSDF of one
// MATERIAL step (same intersection, same wo): the shading basis, wo in it, and the
// LUT terms that depend only on (cos(theta_o), alpha, ior). Each is the value the
// three functions computed on their own, so sharing them changes no bit; it saves the
// repeated basis transform and, above all, the repeated dependent LUT fetches.
struct BsdfFrame {
    V3 b, wo;            // bitangent; wo in (tangent, b, normal), z made >= 0
    bool inv;            // wo was below the shading surface
    bool any;            // !inv || two-sided
    float E, Eavg;       // lut_brdf / lut_brdf_avg (multiscattering plastic / conductor)
    float diel;          // lut_brdf_dielectric (plastic)
    V3 isf;              // isf_factor (plastic)
    DielectricMs dms;    // dielectric_ms (multiscattering rough dielectric)
};
DEV BsdfFrame bsdf_frame(const DeviceScene& s, V3 woW, const Intersection& it)
{
    BsdfFrame f;
    f.b = cross(it.normal, it.tangent);
    f.wo = to_tbn(woW, it.tangent, f.b, it.normal);
    f.inv = f.wo.z < 0.0f;
    if (f.inv) f.wo.z = -f.wo.z;
    f.any = !f.inv || it.isTwoSided;
    const float cosO = f.wo.z;
    const uint32_t type = it.materialType;
    f.E = 0.0f; f.Eavg = 0.0f; f.diel = 0.0f; f.isf = mk(1.0f, 1.0f, 1.0f);
    f.dms.E = 0.0f; f.dms.Eavg = 0.0f; f.dms.EinvAvg = 0.0f; f.dms.ratio = 0.0f;
    if (it.multiscattering && (type == DCRT_MATERIAL_TYPE_PLASTIC || type == DCRT_MATERIAL_TYPE_CONDUCTOR) && f.any) {
        f.E = lut_brdf(s, cosO, it.alpha);
        f.Eavg = lut_brdf_avg(s, it.alpha);
    }
    if (type == DCRT_MATERIAL_TYPE_PLASTIC && f.any) {
        f.diel = lut_brdf_dielectric(s, cosO, it.alpha, it.ior.x, false);
        f.isf = isf_factor(s, it.alpha, it.albedo, it.ior.x, it.internalScatteringMode);
    }
    if (type == DCRT_MATERIAL_TYPE_DIELECTRIC && it.multiscattering && !(it.alpha < kAlphaThreshold))
        f.dms = dielectric_ms(s, cosO, it.alpha, it.ior.x, f.inv);
    return f;
}

DEV V3 evaluate_bsdf(const DeviceScene& s, bool vndf, V3 wiW, const BsdfFrame& f, const Intersection& it)
{
    const V3 wo = f.wo;
    V3 wi = to_tbn(wiW, it.tangent, f.b, it.normal);
    const bool inv = f.inv;
    if (inv) wi.z = -wi.z;
    LCtx c;
    calc_h(wo, wi, c);
    const bool smooth = it.alpha < kAlphaThreshold;
    V3 value = mk(0.0f, 0.0f, 0.0f);
    const uint32_t type = it.materialType;
    if (type != DCRT_MATERIAL_TYPE_DIELECTRIC && type != DCRT_MATERIAL_TYPE_THIN_DIELECTRIC) {
        bool hasL = false, hasCT = false, hasMS = false, dielF = false;
        float ratioL = 0.0f;
        const float E = f.E, Eavg = f.Eavg;
        V3 Fms = mk(0.0f, 0.0f, 0.0f), isf = mk(1.0f, 1.0f, 1.0f);
        const bool any = f.any;
        if (type == DCRT_MATERIAL_TYPE_DIFFUSE && any) {
            hasL = true; ratioL = 1.0f;
        } else if (type == DCRT_MATERIAL_TYPE_PLASTIC && any) {
            hasL = true; hasCT = !smooth; hasMS = it.multiscattering && !smooth; dielF = true;
            ratioL = 1.0f - f.diel;
            if (hasMS) {
                const float fm = ms_fresnel(Eavg, favg_dielectric(it.ior.x));
                Fms = splat(fm);
                ratioL = fmaxf(ratioL - Fms.x * (1.0f - E), 0.0f);
            }
            isf = f.isf;
        } else if (type == DCRT_MATERIAL_TYPE_CONDUCTOR && any && !smooth) {
            hasCT = true; hasMS = it.multiscattering;
            if (hasMS) {
                const V3 k = it.albedo;
                Fms = mk(ms_fresnel(Eavg, favg_conductor1(it.ior.x, k.x)), ms_fresnel(Eavg, favg_conductor1(it.ior.y, k.y)),
                         ms_fresnel(Eavg, favg_conductor1(it.ior.z, k.z)));
            }
        }
        if (hasL) value = value + it.albedo * (lambert(wi, wo) * ratioL) * isf;
        if (hasCT) {
            const float bv = ct_brdf(wi, wo, it.alpha, c);
            const V3 F = dielF ? splat(fresnel_dielectric(c.WOdotH, 1.0f, it.ior.x)) : fresnel_conductor(c.WOdotH, it.ior, it.albedo);
            value = value + F * bv;
        }
        if (hasMS) value = value + ct_ms_brdf(s, wi, wo, it.alpha, E, Eavg, Fms);
    } else if (type != DCRT_MATERIAL_TYPE_THIN_DIELECTRIC && !smooth) {
        const float etaO = inv ? it.ior.x : 1.0f, etaI = inv ? 1.0f : it.ior.x;
        value = value + splat(ct_bsdf<false>(wi, wo, it.alpha, etaO, etaI));
        if (it.multiscattering) {
            const DielectricMs& d = f.dms;
            value = value + splat(ct_ms_bsdf(s, wi, it.alpha, d.ratio, it.ior.x, d.E, d.Eavg, d.EinvAvg, inv));
        }
    }
    return value;
}

DEV float evaluate_bsdf_pdf(const DeviceScene& s, bool vndf, V3 wiW, const BsdfFrame& f, const Intersection& it)
{
    const V3 wo = f.wo;
    V3 wi = to_tbn(wiW, it.tangent, f.b, it.normal);
    const bool inv = f.inv;
    if (inv) wi.z = -wi.z;
    LCtx c;
    calc_h(wo, wi, c);
    const bool smooth = it.alpha < kAlphaThreshold;
    float pdf = 0.0f;
    const uint32_t type = it.materialType;
    if (type != DCRT_MATERIAL_TYPE_DIELECTRIC && type != DCRT_MATERIAL_TYPE_THIN_DIELECTRIC) {
        bool hasL = false, hasCT = false, hasMS = false;
        float wl = 0.0f, wct = 0.0f, wms = 0.0f;
        const bool any = f.any;
        if (type == DCRT_MATERIAL_TYPE_DIFFUSE && any) {
            hasL = true; wl = 1.0f;
        } else if (type == DCRT_MATERIAL_TYPE_PLASTIC && any) {
            hasL = true; hasCT = !smooth; hasMS = it.multiscattering && !smooth;
            wct = f.diel;
            wl = 1.0f - wct;
            if (hasMS) {
                const float E = f.E;
                const float Eavg = f.Eavg;
                const float Fms = ms_fresnel(Eavg, favg_dielectric(it.ior.x));
                wms = Fms * (1.0f - E);
                wl = fmaxf(wl - wms, 0.0f);
            }
        } else if (type == DCRT_MATERIAL_TYPE_CONDUCTOR && any && !smooth) {
            hasCT = true; hasMS = it.multiscattering;
            wct = 1.0f;
            if (hasMS) { wct = 0.5f; wms = 0.5f; }
        }
        if (hasL) pdf = pdf + lambert_pdf(wi, wo) * wl;
        if (hasCT) pdf = pdf + ct_brdf_pdf(vndf, wi, wo, it.alpha, c) * wct;
        if (hasMS) pdf = pdf + ct_ms_brdf_pdf(wi, wo) * wms;
    } else if (type != DCRT_MATERIAL_TYPE_THIN_DIELECTRIC && !smooth) {
        float wb = 1.0f, wms = 0.0f, ratio = 0.0f;
        const float etaO = inv ? it.ior.x : 1.0f, etaI = inv ? 1.0f : it.ior.x;
        if (it.multiscattering) {
            const DielectricMs& d = f.dms;
            ratio = d.ratio;
            wb = d.E; wms = 1.0f - d.E;
        }
        pdf = pdf + ct_bsdf_pdf(vndf, wi, wo, it.alpha, etaO, etaI) * wb;
        if (it.multiscattering) pdf = pdf + ct_ms_bsdf_pdf(wi, ratio) * wms;
    }
    return pdf;
}

DEV void sample_bsdf(const DeviceScene& s, bool vndf, const BsdfFrame& f, float sx, float sy, float sel, const Intersection& it,
                     V3* wiOut, V3* valueOut, float* pdfOut, bool* isDelta)
{
    V3 wi = mk(0.0f, 0.0f, 0.0f), value = mk(0.0f, 0.0f, 0.0f);
    float pdf = 0.0f;
    *isDelta = false;
    const V3 b = f.b;
    const V3 wo = f.wo;
    const bool inv = f.inv;
    LCtx c;
    c.H = mk(0.0f, 0.0f, 0.0f); c.WOdotH = 0.0f;
    const bool smooth = it.alpha < kAlphaThreshold;
    const uint32_t type = it.materialType;
    if (type != DCRT_MATERIAL_TYPE_DIELECTRIC && type != DCRT_MATERIAL_TYPE_THIN_DIELECTRIC) {
        bool hasL = false, hasCT = false, hasMS = false, dielF = false;
        float wl = 0.0f, wct = 0.0f, wms = 0.0f;
        const float E = f.E, Eavg = f.Eavg;
        V3 Fms = mk(0.0f, 0.0f, 0.0f), isf = mk(1.0f, 1.0f, 1.0f);
        const bool any = f.any;
        if (type == DCRT_MATERIAL_TYPE_DIFFUSE && any) {
            hasL = true; wl = 1.0f;
        } else if (type == DCRT_MATERIAL_TYPE_PLASTIC && any) {
            hasL = true; hasCT = true; hasMS = it.multiscattering && !smooth; dielF = true;
            wct = f.diel;
            wl = 1.0f - wct;
            if (hasMS) {
                const float fm = ms_fresnel(Eavg, favg_dielectric(it.ior.x));
                Fms = splat(fm);
                wms = Fms.x * (1.0f - E);
                wl = fmaxf(wl - wms, 0.0f);
            }
            isf = f.isf;
        } else if (type == DCRT_MATERIAL_TYPE_CONDUCTOR && any) {
            hasCT = true; hasMS = it.multiscattering && !smooth;
            wct = 1.0f;
            if (hasMS) {
                const V3 k = it.albedo;
                Fms = mk(ms_fresnel(Eavg, favg_conductor1(it.ior.x, k.x)), ms_fresnel(Eavg, favg_conductor1(it.ior.y, k.y)),
                         ms_fresnel(Eavg, favg_conductor1(it.ior.z, k.z)));
                wct = 0.5f; wms = 0.5f;
            }
        }
        if (sel < wl) {
            wi = cosine_hemisphere(sx, sy);
            calc_h(wo, wi, c);
        } else if (sel < wl + wct) {
            if (!smooth) {
                const V3 m = sample_ggx(vndf, wo, sx, sy, it.alpha);
                wi = -reflect(wo, m);
                c.H = m; c.WOdotH = dot(m, wo);
            } else {
                float vr = value.x;
                wi = specular_brdf_sample(wo, &vr, &pdf, c);
                const V3 F = dielF ? splat(fresnel_dielectric(c.WOdotH, 1.0f, it.ior.x)) : fresnel_conductor(c.WOdotH, it.ior, it.albedo);
                value = F * vr;
                pdf = pdf * wct;
                *isDelta = true;
                hasL = false; hasCT = false; hasMS = false;
            }
        } else {
            wi = cosine_hemisphere(sx, sy);
            calc_h(wo, wi, c);
        }
        if (hasL) {
            value = value + it.albedo * (lambert(wi, wo) * wl) * isf;
            pdf = pdf + lambert_pdf(wi, wo) * wl;
        }
        if (hasCT && !smooth) {
            const float mv = ct_brdf(wi, wo, it.alpha, c);
            const V3 F = dielF ? splat(fresnel_dielectric(c.WOdotH, 1.0f, it.ior.x)) : fresnel_conductor(c.WOdotH, it.ior, it.albedo);
            value = value + F * mv;
            pdf = pdf + ct_brdf_pdf(vndf, wi, wo, it.alpha, c) * wct;
        }
        if (hasMS) {
            value = value + ct_ms_brdf(s, wi, wo, it.alpha, E, Eavg, Fms);
            pdf = pdf + ct_ms_brdf_pdf(wi, wo) * wms;
        }
    } else if (type == DCRT_MATERIAL_TYPE_THIN_DIELECTRIC || smooth) {
        const bool thin = type == DCRT_MATERIAL_TYPE_THIN_DIELECTRIC;
        const bool entering = thin ? false : inv;
        const float etaO = entering ? it.ior.x : 1.0f, etaI = entering ? 1.0f : it.ior.x;
        float vr = value.x;
        wi = specular_bsdf_sample<false>(wo, sel, etaO, etaI, thin, &vr, &pdf, c);
        value = splat(vr);
        *isDelta = true;
    } else {
        float wb = 1.0f, wms = 0.0f;
        const DielectricMs& d = f.dms;
        const float etaO = inv ? it.ior.x : 1.0f, etaI = inv ? 1.0f : it.ior.x;
        if (it.multiscattering) {
            wb = d.E; wms = 1.0f - d.E;
        }
        if (sel < wb) {
            wi = ct_bsdf_sample(vndf, wo, sel, sx, sy, it.alpha, etaO, etaI, c);
        } else if (wo.z != 0.0f) {
            wi = cosine_hemisphere(sx, sy);
            if (!(sel >= d.ratio)) wi.z = -wi.z;
        }
        value = value + splat(ct_bsdf<false>(wi, wo, it.alpha, etaO, etaI));
        pdf = pdf + ct_bsdf_pdf(vndf, wi, wo, it.alpha, etaO, etaI) * wb;
        if (it.multiscattering) {
            value = value + splat(ct_ms_bsdf(s, wi, it.alpha, d.ratio, it.ior.x, d.E, d.Eavg, d.EinvAvg, inv));
            pdf = pdf + ct_ms_bsdf_pdf(wi, d.ratio) * wms;
        }
    }
    if (inv) wi.z = -wi.z;
    *wiOut = from_tbn(wi, it.tangent, b, it.normal);
    *valueOut = value;
    *pdfOut = pdf;
}

}  // namespace dev
}  // namespace dcrt
