/*
 * dcrt_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of YaoTiancheng/DirectComputeRayTracing's wavefront path
 * (Shaders/ *.hlsl) used as the parity checker for the MI355X HIP kernels and as
 * the scalar CPU baseline (MegakernelPathTracing.hlsl:65-208 transcription).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it. The product (directcomputeraytracing_amd/) never links or calls it.
 *
 * Parity status: pinned against the reference's own public constants (SplitMix64,
 * xoshiro128** 1.0) and against independent native-uint64 / textbook restatements;
 * the reference has no tests or golden vectors, so image-level
 * parity vs. the D3D12 renderer itself is "parity unpinned" (no D3D12/DXC exists here).
 */
#ifndef DCRT_ORACLE_H_
#define DCRT_ORACLE_H_

#include "../include/dcrt.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_MODE_WAVEFRONT  0   /* WavefrontPathTracing.hlsl state machine (per path)  */
#define ORACLE_MODE_MEGAKERNEL 1   /* MegakernelPathTracing.hlsl:110-208                  */

typedef struct oracle_counters {
    uint64_t extension_rays;
    uint64_t shadow_rays;
    uint64_t node_visits;       /* iterationCounter semantics, BVHAccel.inc.hlsl:121 */
    uint64_t triangle_tests;
    uint64_t blas_entries;
    uint64_t shadow_node_visits;
    uint64_t shadow_triangle_tests;
    uint64_t shadow_blas_entries;
} oracle_counters;

/* Render pixels [x0,x0+w) x [y0,y0+h) of image `frame->frame_seed`; writes the
 * sample textures (position W*H*2, value W*H*4, alpha lane = 0) at full-film
 * addressing, and optionally the terminal RNG state (W*H*4). */
int oracle_render(const dcrt_flat_scene* scene, const dcrt_bxdf_luts* luts, const dcrt_frame_params* frame,
                  int mode, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
                  float* sample_position, float* sample_value, uint32_t* rng_state,
                  oracle_counters* counters, int num_threads);

/* SampleConvolution.hlsl:67-106 over the whole film. */
void oracle_sample_convolution(const dcrt_filter_params* filter, uint32_t width, uint32_t height,
                               const float* sample_position, const float* sample_value, float* film_rgba,
                               uint32_t row_begin, uint32_t row_end);

/* BVHIntersectNoInterp / BVHIntersect over a ray batch (BVHAccel.inc.hlsl:85-369). */
void oracle_trace_rays(const dcrt_flat_scene* scene, const dcrt_ray* rays, uint32_t count, dcrt_ray_hit* hits,
                       uint32_t features, oracle_counters* counters);
void oracle_occluded(const dcrt_flat_scene* scene, const dcrt_ray* rays, uint32_t count, uint32_t* occluded,
                     uint32_t features, oracle_counters* counters);

/* BxDFTexturesBuilding.hlsl restated. which: 0 = BRDF, 1 = BRDF dielectric, 2 = BSDF.
 * Integrates texels [texel_begin, texel_end) of that table's R32 accumulation
 * image (full MC, all batches) into out_float; `finalize` converts whole tables. */
void oracle_lut_integrate(int which, uint32_t texel_begin, uint32_t texel_end, float* out_float);
void oracle_lut_finalize(const float* brdf_f32, const float* brdf_dielectric_f32, const float* bsdf_f32,
                         dcrt_bxdf_luts* out_luts);
int oracle_build_luts(dcrt_bxdf_luts* out_luts, int num_threads);

/* RNG / sampling primitives for known-answer tests (Samples.inc.hlsl, Xoshiro.inc.hlsl). */
void oracle_rng_init(uint32_t px, uint32_t py, uint32_t frame_seed, uint32_t state[4]);
uint32_t oracle_rng_next(uint32_t state[4]);
void oracle_splitmix64_pair(uint32_t lo, uint32_t hi, uint32_t out[6]);
uint32_t oracle_morton(uint32_t x, uint32_t y);
void oracle_xoshiro_jump(uint32_t state[4]);
void oracle_offset_ray_origin(const float p[3], const float n[3], const float d[3], float out[3]);
void oracle_generate_camera_ray(const dcrt_frame_params* frame, uint32_t px, uint32_t py, float origin[3],
                                float direction[3], uint32_t rng_out[4]);
/* function: 0 sin, 1 cos, 2 exp, 3 atan, 4 log */
void oracle_math_eval(int function, const float* x, uint32_t count, float* y);

/* One material's BSDF (BSDFs.inc.hlsl EvaluateBSDF / EvaluateBSDFPdf / SampleBSDF) in the frame
   normal = geometric normal = (0,0,1), tangent = (1,0,0), for the BxDF physics pins
   (tests/test_bsdf_pins.py). material: type, albedo[3], alpha, ior, two-sided, multiscattering,
   internal scattering mode. eval: f (3 per pair) and pdf for `count` (wi, wo) pairs; sample: for
   `count` wo and (sx, sy, sel) triples, wi, f, pdf and the delta flag. */
typedef struct oracle_bsdf_material {
    uint32_t type;
    float albedo[3];
    float alpha, ior;
    int two_sided, multiscattering;
    uint32_t internal_scattering;
} oracle_bsdf_material;
void oracle_bsdf_eval(const dcrt_bxdf_luts* luts, const oracle_bsdf_material* m, const float* wi, const float* wo,
                      uint32_t count, float* f_out, float* pdf_out);
void oracle_bsdf_sample(const dcrt_bxdf_luts* luts, const oracle_bsdf_material* m, const float* wo, const float* u,
                        uint32_t count, float* wi_out, float* f_out, float* pdf_out, int* delta_out);

/* Post-processing (PostProcessings.hlsl, SumLuminance.hlsl): tone-mapped sRGB8 RGBA. */
float oracle_sum_log_luminance(const float* film_rgba, uint32_t width, uint32_t height);
void oracle_resolve_image(const float* film_rgba, uint32_t width, uint32_t height, int enabled, int auto_exposure, float ev100,
                          float luminance_white, const float* srgb_thresholds, uint8_t* out_rgba8);

/* ---- BVH build (dcrt_oracle_bvh.c, BVHAccel.cpp:76-447) ---------------------- */
/* BVHAccel::BVHNode before packing: center/extents box, child or first primitive,
 * primitive count (TLAS leaves: count until the scene patches in the instance). */
typedef struct oracle_bvh_node {
    float center[3], extents[3];
    uint32_t child_or_prim;
    uint32_t count_or_instance;
    uint32_t is_leaf;
    uint32_t split_axis;
} oracle_bvh_node;
/* BuildBLAS over one mesh: nodes (capacity 2 * tri_count - 1), BVH-ordered index
 * triples, tri_order[new] = load-order triangle; maxDepth / maxStackSize. */
int oracle_bvh_build_blas(const dcrt_vertex* vertices, const uint32_t* indices, uint32_t tri_count, oracle_bvh_node* nodes,
                          uint32_t* node_count, uint32_t* reordered_indices, uint32_t* tri_order, uint32_t* max_depth,
                          uint32_t* max_stack);
/* BuildTLAS over instance boxes (BLAS root center+extents, 6 floats) and XMFLOAT4X3
 * transforms (12 floats, 4 rows of 3). */
int oracle_bvh_build_tlas(const float* blas_root_boxes, const float* transforms, uint32_t instance_count,
                          oracle_bvh_node* nodes, uint32_t* node_count, uint32_t* instance_order, uint32_t* max_depth,
                          uint32_t* max_stack, uint32_t* instance_depths);
void oracle_bvh_pack(const oracle_bvh_node* nodes, uint32_t count, int is_blas, dcrt_bvh_node* out, uint32_t node_offset,
                     uint32_t prim_offset);

/* dcrt_oracle_scene.c: the float half of CScene's flattening (frame constants,
 * WavefrontPathTracer.cpp:372-428; directional light direction, Scene.cpp:946-955). */
void oracle_frame_params(const dcrt_scene_settings* settings, uint32_t frame_seed, dcrt_frame_params* out);
void oracle_punctual_direction(const float euler[3], float out[3]);

#ifdef __cplusplus
}
#endif

#endif
