/*
 * dcrt_oracle_scene.c -- TEST INFRASTRUCTURE ONLY (see dcrt_oracle.h).
 *
 * The floating-point half of the oracle's own CScene flattening (the bookkeeping half is
 * oracle/__init__.py: flatten_scene): the frame constants Render() uploads
 * (WavefrontPathTracer.cpp:372-428) -- the camera matrix (Camera.cpp:87-96), the film
 * distance and aperture (Scene.cpp:837-847), the blade vertex -- and the directional
 * lights' direction (SPunctualLight::CalculateDirection, Scene.cpp:946-955).
 *
 * Restated here from the reference sources and from DirectXMath's published algorithms,
 * separately from the product's host code (csrc/host/scene.cpp, xmath.cpp):
 *  - XMVectorSinCos (SSE2 path): XMVectorModAngles (quotient rounded by XMVectorRound's
 *    2^23 add/subtract carrying the sign, no SSE4.1), reflection into [-pi/2, pi/2], the
 *    11-degree sine / 10-degree cosine polynomials evaluated as separate multiplies and
 *    adds (x64 SSE2: XM_FMADD_PS is mul + add);
 *  - XMMatrixRotationRollPitchYawFromVector in the product form of the scalar
 *    (_XM_NO_INTRINSICS_) code path, on XMVectorSinCos's sines and cosines (the SSE
 *    product order of its three-factor entries is not available here: parity unpinned);
 *  - XMVector3Transform: z*r2 + r3, then y*r1 + that, then x*r0 + that.
 * The CRT's tanf / cosf / sinf are the host libm's (MSVC's are parity unpinned).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "dcrt_oracle.h"

/* DirectXMath constants (DirectXMathMisc / g_XMSinCoefficients0/1, g_XMCosCoefficients0/1) */
#define XM_PI_F       3.141592654f
#define XM_2PI_F      6.283185307f
#define XM_1DIV2PI_F  0.159154943f
#define XM_PIDIV2_F   1.570796327f

/* XMVectorRound without SSE4.1: |v| <= 2^23 rounds to nearest-even by (v + m) - m, with m
 * = 2^23 carrying v's sign bit; larger magnitudes are already integers and pass through */
static float xm_round(float v)
{
    const float magic = signbit(v) ? -8388608.0f : 8388608.0f;
    if (!(fabsf(v) <= 8388608.0f)) return v;
    volatile float t = v + magic;
    return t - magic;
}

static void xm_vector_sincos(float angle, float* s, float* c)
{
    /* XMVectorModAngles: angle - round(angle / 2pi) * 2pi */
    const float q = xm_round(angle * XM_1DIV2PI_F);
    const float x0 = angle - q * XM_2PI_F;
    /* sign-selected reflection: |x| <= pi/2 keeps x, else (+-pi) - x with cos negated */
    const float pi_signed = signbit(x0) ? -XM_PI_F : XM_PI_F;
    const int keep = fabsf(x0) <= XM_PIDIV2_F;
    const float x = keep ? x0 : pi_signed - x0;
    const float sgn = keep ? 1.0f : -1.0f;
    const float x2 = x * x;
    float r = -2.3889859e-08f * x2 + 2.7525562e-06f;
    r = r * x2 + -0.00019840874f;
    r = r * x2 + 0.0083333310f;
    r = r * x2 + -0.16666667f;
    r = r * x2 + 1.0f;
    *s = r * x;
    float k = -2.6051615e-07f * x2 + 2.4760495e-05f;
    k = k * x2 + -0.0013888378f;
    k = k * x2 + 0.041666638f;
    k = k * x2 + -0.5f;
    k = k * x2 + 1.0f;
    *c = k * sgn;
}

/* XMMatrixRotationRollPitchYawFromVector((pitch, yaw, roll)): row-major 4x4 */
static void rotation_roll_pitch_yaw(const float euler[3], float m[16])
{
    float sp, cp, sy, cy, sr, cr;
    xm_vector_sincos(euler[0], &sp, &cp);
    xm_vector_sincos(euler[1], &sy, &cy);
    xm_vector_sincos(euler[2], &sr, &cr);
    memset(m, 0, 16 * sizeof(float));
    m[0] = cr * cy + sr * sp * sy;
    m[1] = sr * cp;
    m[2] = sr * sp * cy - cr * sy;
    m[4] = cr * sp * sy - sr * cy;
    m[5] = cr * cp;
    m[6] = sr * sy + cr * sp * cy;
    m[8] = cp * sy;
    m[9] = -sp;
    m[10] = cp * cy;
    m[15] = 1.0f;
}

/* SPunctualLight::CalculateDirection (Scene.cpp:946-955): XMVector3Transform of
 * g_XMIdentityR0 = (1, 0, 0) by the roll-pitch-yaw matrix */
void oracle_punctual_direction(const float euler[3], float out[3])
{
    float m[16];
    rotation_roll_pitch_yaw(euler, m);
    const float v[3] = { 1.0f, 0.0f, 0.0f };
    for (int c = 0; c < 3; ++c) {
        float t = v[2] * m[8 + c] + m[12 + c];
        t = v[1] * m[4 + c] + t;
        out[c] = v[0] * m[c] + t;
    }
}

/* SNewPathConstants / SMaterialConstants (WavefrontPathTracer.cpp:396-425) from the scene
 * state; light_count / environment light index from the light lists (Scene.h GetLightCount,
 * WavefrontPathTracer.cpp:425: the environment light follows the mesh lights) */
void oracle_frame_params(const dcrt_scene_settings* s, uint32_t frame_seed, dcrt_frame_params* p)
{
    memset(p, 0, sizeof(*p));
    /* Camera::GetTransformMatrix (Camera.cpp:87-96): rotation, translation in row 3 */
    rotation_roll_pitch_yaw(s->camera_euler_angles, p->camera_transform);
    p->camera_transform[12] = s->camera_position[0];
    p->camera_transform[13] = s->camera_position[1];
    p->camera_transform[14] = s->camera_position[2];
    p->resolution[0] = s->resolution[0];
    p->resolution[1] = s->resolution[1];
    p->film_size[0] = s->film_size[0];
    p->film_size[1] = s->film_size[1];
    /* CalculateApertureDiameter (Scene.cpp:844-847) * 0.5 */
    const int pinhole = s->camera_type == 0;
    const float diameter = pinhole ? 0.0f : s->focal_length / s->relative_aperture;
    p->aperture_radius = diameter * 0.5f;
    p->focal_distance = s->focal_distance;
    /* CalculateFilmDistance (Scene.cpp:837-842): pinhole from the fov, thin lens from the
     * Gaussian lens equation */
    if (pinhole) {
        const float t = tanf(0.5f * s->fov_x);
        p->film_distance = 0.5f * s->film_size[0] / (t < 0.0001f ? 0.0001f : t);
    } else {
        p->film_distance = (s->focal_length * s->focal_distance) / (s->focal_length + s->focal_distance);
    }
    p->blade_count = s->aperture_blade_count;
    const float half_blade = XM_PI_F / (float)s->aperture_blade_count;
    p->blade_vertex_pos[0] = cosf(half_blade) * p->aperture_radius;
    p->blade_vertex_pos[1] = sinf(half_blade) * p->aperture_radius;
    p->aperture_base_angle = s->aperture_rotation;
    p->frame_seed = frame_seed;
    p->max_bounce_count = s->max_bounce_count;
    p->light_count = s->mesh_light_count + s->punctual_light_count + (s->has_environment_light ? 1u : 0u);
    p->environment_light_index = s->has_environment_light ? s->mesh_light_count : DCRT_LIGHT_INDEX_INVALID;
    p->features = s->features;
}
