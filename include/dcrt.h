/*
 * dcrt.h -- C ABI of the MI355X-native wavefront path tracer.
 *
 * This is the drop-in boundary for the hot path of
 * YaoTiancheng/DirectComputeRayTracing: the `CWavefrontPathTracer` plug-in
 * (Source/PathTracer.h:6-26, Source/WavefrontPathTracer.cpp:70-1162) and the
 * scene buffers `CScene` flattens for it (Source/Scene.cpp:273-608).
 *
 * Conventions (every entry point):
 *   - plain C types, pointers and sizes; no C++ or torch types cross the ABI;
 *   - return int status: 0 = ok, negative = error (see DCRT_E_*); nothing throws;
 *   - one tracer handle per HIP device; calls on a handle are serialised by the caller;
 *   - all GPU work of a tracer is ordered on the stream passed to dcrt_tracer_create
 *     (NULL = the tracer's own non-blocking stream).
 *
 * Wire format: the structs below reproduce the reference's GPU layouts byte for
 * byte (Appendix B of SURVEY.md): Vertex 44 B, BVHNode 32 B, Material 52 B,
 * SLight 28 B, float4x3 48 B (HLSL column-major), so a maintainer can hand the
 * reference's CScene arrays straight through.
 */
#ifndef DCRT_H_
#define DCRT_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCRT_API __attribute__((visibility("default")))

/* ---- status codes ---------------------------------------------------- */
#define DCRT_OK              0
#define DCRT_E_INVALID_ARG  -1
#define DCRT_E_HIP          -2   /* a HIP runtime call failed               */
#define DCRT_E_NO_SCENE     -3   /* render before dcrt_tracer_upload_scene   */
#define DCRT_E_IO           -4   /* file could not be read / parsed         */
#define DCRT_E_LIMIT        -5   /* a reference limit was exceeded          */
#define DCRT_E_NO_DEVICE    -6   /* no HIP device visible                   */

/* ---- constants shared with the reference shaders ----------------------- */
/* Shaders/LightSharedDef.inc.hlsl:6-12 */
#define DCRT_LIGHT_INDEX_INVALID        0xFFFFFFFFu
#define DCRT_LIGHT_FLAGS_POINT_LIGHT        0x1u
#define DCRT_LIGHT_FLAGS_MESH_LIGHT         0x2u
#define DCRT_LIGHT_FLAGS_DIRECTIONAL_LIGHT  0x4u
#define DCRT_LIGHT_FLAGS_ENVIRONMENT_LIGHT  0x8u
/* Shaders/Material.inc.hlsl:6-19 */
#define DCRT_MATERIAL_FLAG_ROUGHNESS_TEXTURE 0x20u
#define DCRT_MATERIAL_FLAG_IS_TWOSIDED       0x40u
#define DCRT_MATERIAL_FLAG_MULTISCATTERING   0x80u
#define DCRT_MATERIAL_FLAG_INTERNAL_SCATTERING_SHIFT 8
#define DCRT_MATERIAL_FLAG_INTERNAL_SCATTERING_MASK  0x300u
#define DCRT_MATERIAL_FLAG_TYPE_MASK         0xFu
#define DCRT_MATERIAL_TYPE_DIFFUSE          0
#define DCRT_MATERIAL_TYPE_PLASTIC          1
#define DCRT_MATERIAL_TYPE_CONDUCTOR        2
#define DCRT_MATERIAL_TYPE_DIELECTRIC       3
#define DCRT_MATERIAL_TYPE_THIN_DIELECTRIC  4
/* Shaders/InternalScatteringMode.inc.hlsl:4-6 */
#define DCRT_INTERNAL_SCATTERING_IGNORE   0
#define DCRT_INTERNAL_SCATTERING_SINGLE   1
#define DCRT_INTERNAL_SCATTERING_MULTIPLE 2
/* Shaders/InstanceSharedDef.inc.hlsl:4-5 */
#define DCRT_INSTANCE_FLAG_OPAQUE             0x1u
#define DCRT_INSTANCE_MATERIAL_OVERRIDE_NONE  0xFFFFFFFFu
/* Shaders/BVHSharedDef.inc.hlsl:4 */
#define DCRT_BVHNODE_MISC_MASK_PRIMITIVE_COUNT 0x1FFFFFFFu
/* Scene.h:108-109 */
#define DCRT_MAX_RAY_BOUNCE   20
#define DCRT_MAX_LIGHT_COUNT  5000
/* Shaders/BxDFTextureDef.inc.hlsl:4-9 */
#define DCRT_BXDFTEX_BRDF_SIZE_X 32
#define DCRT_BXDFTEX_BRDF_SIZE_Y 32
#define DCRT_BXDFTEX_BRDF_DIELECTRIC_SIZE_X 32
#define DCRT_BXDFTEX_BRDF_DIELECTRIC_SIZE_Y 16
#define DCRT_BXDFTEX_BRDF_DIELECTRIC_SIZE_Z 16

/* ---- feature variants (WavefrontPathTracer.cpp:554-590 shader defines) -- */
#define DCRT_FEATURE_GGX_SAMPLE_VNDF          0x01u  /* GGX_SAMPLE_VNDF (default on)            */
#define DCRT_FEATURE_NO_FRONT_TO_BACK         0x02u  /* BVH_NO_FRONT_TO_BACK_TRAVERSAL (off)    */
#define DCRT_FEATURE_LIGHT_VISIBLE            0x04u  /* LIGHT_VISIBLE (default on)              */
#define DCRT_FEATURE_WATERTIGHT               0x08u  /* WATERTIGHT_RAY_TRIANGLE_INTERSECTION(on)*/
#define DCRT_FEATURE_ALLOW_ANYHIT             0x10u  /* ALLOW_ANYHIT_SHADER (off): opacity test on
                                                        non-opaque instances (HitShader.inc.hlsl:86-113) */
#define DCRT_FEATURE_DEFAULT (DCRT_FEATURE_GGX_SAMPLE_VNDF | DCRT_FEATURE_LIGHT_VISIBLE | DCRT_FEATURE_WATERTIGHT)

/* ---- Appendix-B layouts ------------------------------------------------ */
/* Shaders/Vertex.inc.hlsl:8-14 -- 44 bytes */
typedef struct dcrt_vertex {
    float position[3];
    float normal[3];
    float tangent[3];
    float texcoord[2];
} dcrt_vertex;

/* Shaders/BVHNode.inc.hlsl:8-14 -- 32 bytes.
 * misc = primCount(or TLAS-leaf instance index) << 3 | (TLAS leaf ? 4 : 0) | split axis */
typedef struct dcrt_bvh_node {
    float bbox_min[3];
    float bbox_max[3];
    uint32_t right_child_or_prim_index;
    uint32_t misc;
} dcrt_bvh_node;

/* Shaders/Material.inc.hlsl:23-33 -- 52 bytes */
typedef struct dcrt_material {
    float albedo[3];
    int32_t albedo_texture_index;
    float ior[3];
    float roughness;
    float tex_tiling[2];
    float opacity;
    uint32_t flags;
    int32_t opacity_texture_index;
} dcrt_material;

/* Shaders/LightSharedDef.inc.hlsl:15-20 -- 28 bytes. For mesh lights the
 * second float3 holds (triangle offset, triangle count, instance) as uint bits. */
typedef struct dcrt_light {
    float radiance[3];
    float position_or_triangle_range[3];
    uint32_t flags;
} dcrt_light;

/* HLSL `float4x3` in a StructuredBuffer, column-major: m[c*4 + r] = M[r][c],
 * row-vector convention p' = mul(float4(p,1), M) (Scene.cpp:431-444). 48 bytes. */
typedef struct dcrt_float4x3 {
    float m[12];
} dcrt_float4x3;

/* Bindless scene texture (Texture2D<float4> g_Textures[], Scene.cpp:586-608). */
#define DCRT_TEXTURE_FORMAT_RGBA8_SRGB 0   /* DXGI_FORMAT_R8G8B8A8_UNORM_SRGB */
#define DCRT_TEXTURE_FORMAT_R8_UNORM   1   /* DXGI_FORMAT_R8_UNORM            */
typedef struct dcrt_texture {
    uint32_t width;
    uint32_t height;
    uint32_t format;            /* DCRT_TEXTURE_FORMAT_*            */
    const uint8_t* pixels;      /* tightly packed rows              */
} dcrt_texture;

/* The flattened scene: exactly what Scene.cpp:273-608 uploads. Host pointers. */
typedef struct dcrt_flat_scene {
    const dcrt_vertex* vertices;            uint32_t vertex_count;
    const uint32_t* triangles;              uint32_t triangle_count;   /* 3 indices / triangle */
    const dcrt_bvh_node* bvh_nodes;         uint32_t bvh_node_count;   /* TLAS first, then BLASes */
    uint32_t tlas_node_count;
    const uint32_t* material_ids;                                       /* one per triangle */
    const dcrt_float4x3* instance_transforms; uint32_t instance_count;  /* 2N: forward, inverse */
    const uint32_t* instance_light_indices;                             /* N */
    const uint32_t* instance_flags;                                     /* N */
    const uint32_t* instance_material_overrides;                        /* N */
    const dcrt_material* materials;         uint32_t material_count;
    const dcrt_light* lights;               uint32_t light_count;       /* mesh, env, punctual */
    uint32_t environment_light_index;       /* #mesh lights, or DCRT_LIGHT_INDEX_INVALID */
    const dcrt_texture* textures;           uint32_t texture_count;
    /* Environment cube (TextureCube<float3>): 6 faces (+X,-X,+Y,-Y,+Z,-Z) of
     * size x size texels, RGB float, NULL when the scene has none. */
    const float* env_cube_rgb;              uint32_t env_cube_size;
    uint32_t bvh_traversal_stack_size;      /* CScene::m_BVHTraversalStackSize */
} dcrt_flat_scene;

/* The six R16_UNORM BxDF lookup tables (BxDFTexturesBuilding.cpp:171-175,265-270,379-384). */
#define DCRT_LUT_BRDF_COUNT            (32 * 32)
#define DCRT_LUT_BRDF_AVG_COUNT        (32)
#define DCRT_LUT_BRDF_DIELECTRIC_COUNT (32 * 16 * 32)
#define DCRT_LUT_BRDF_DIELECTRIC_AVG_COUNT (16 * 16 * 2)
#define DCRT_LUT_BSDF_COUNT            (32 * 16 * 32)
#define DCRT_LUT_BSDF_AVG_COUNT        (16 * 16 * 2)
typedef struct dcrt_bxdf_luts {
    uint16_t brdf[DCRT_LUT_BRDF_COUNT];                         /* [alpha 32][cos 32]            */
    uint16_t brdf_avg[DCRT_LUT_BRDF_AVG_COUNT];                 /* [alpha 32]                    */
    uint16_t brdf_dielectric[DCRT_LUT_BRDF_DIELECTRIC_COUNT];   /* [slice 32][alpha 16][cos 32]  */
    uint16_t brdf_dielectric_avg[DCRT_LUT_BRDF_DIELECTRIC_AVG_COUNT]; /* [slice 2][ior 16][alpha 16] */
    uint16_t bsdf[DCRT_LUT_BSDF_COUNT];                         /* [slice 32][alpha 16][cos 32]  */
    uint16_t bsdf_avg[DCRT_LUT_BSDF_AVG_COUNT];                 /* [slice 2][ior 16][alpha 16]   */
} dcrt_bxdf_luts;

/* Union of SControlConstants / SNewPathConstants / SMaterialConstants
 * (WavefrontPathTracer.cpp:34-63,372-428). */
typedef struct dcrt_frame_params {
    float camera_transform[16];   /* row-major float4x4, translation in row 3 (Camera.cpp:87-96) */
    uint32_t resolution[2];       /* current film width, height                   */
    float film_size[2];
    float aperture_radius;        /* CalculateApertureDiameter() * 0.5            */
    float focal_distance;
    float film_distance;          /* CalculateFilmDistance()                      */
    uint32_t blade_count;
    float blade_vertex_pos[2];    /* cos/sin(pi / blades) * aperture radius       */
    float aperture_base_angle;
    uint32_t frame_seed;
    uint32_t max_bounce_count;
    uint32_t light_count;
    uint32_t environment_light_index;
    uint32_t features;            /* DCRT_FEATURE_* */
} dcrt_frame_params;

/* Film reconstruction (Scene.h:131-136, SampleConvolution.cpp:100-130). */
#define DCRT_FILTER_BOX      0
#define DCRT_FILTER_TRIANGLE 1
#define DCRT_FILTER_GAUSSIAN 2
#define DCRT_FILTER_MITCHELL 3
#define DCRT_FILTER_LANCZOS  4
typedef struct dcrt_filter_params {
    uint32_t filter;              /* DCRT_FILTER_* */
    float radius;
    float gaussian_alpha;
    float mitchell_b;
    float mitchell_c;
    uint32_t lanczos_tau;
} dcrt_filter_params;

/* Ray / hit records of the kernel-level boundary (WavefrontPathTracing.hlsl:3-17). */
typedef struct dcrt_ray {
    float origin[3];
    float t_max;
    float direction[3];
    float t_min;
} dcrt_ray;                       /* 32 bytes, SRay */
typedef struct dcrt_ray_hit {
    float t;                      /* +inf on a miss                                   */
    float u, v;
    uint32_t triangle_id;         /* bit 31 = backface                                */
    uint32_t instance_index;
} dcrt_ray_hit;                   /* 20 bytes, SRayHit */

/* Tracer configuration (CWavefrontPathTracer::Create, WavefrontPathTracer.cpp:25-28). */
typedef struct dcrt_tracer_config {
    uint32_t path_pool_size;      /* slots; 0 = default (2^20 on MI355X)             */
    uint32_t iterations_per_render; /* m_IterationPerFrame; 0 = default              */
    int32_t device;               /* HIP device ordinal                               */
    void* stream;                 /* hipStream_t or NULL                              */
    uint32_t debug_rng;           /* nonzero: keep each pixel's terminal RNG state    */
} dcrt_tracer_config;

/* Counters since the last dcrt_tracer_reset_stats (or create). */
typedef struct dcrt_ray_stats {
    uint64_t extension_rays;      /* EXTENSION_RAY_CAST rays traced                   */
    uint64_t shadow_rays;         /* SHADOW_RAY_CAST rays traced                      */
    uint64_t new_paths;           /* paths started by the completed images (one per
                                     rendered pixel, halo rows included, per image)   */
    uint64_t iterations;          /* RenderOneIteration equivalents launched          */
    uint64_t images_completed;    /* images finished by render / render_images        */
} dcrt_ray_stats;

/* Rows of the film a tracer renders and convolves (multi-GPU film tiling).
 * The H rows are cut into K = N * k stripes of floor/ceil(H / K) rows, k = round(H / (N *
 * stripe_height)) (at least 1); stripe j = rows [j*H/K, (j+1)*H/K) belongs to rank j % N.
 * A rank path-traces its rows plus halo_rows rows beyond each stripe edge and convolves
 * only its own rows, so the SUM of all ranks' films is the one-tracer film bit for bit. */
typedef struct dcrt_film_partition {
    uint32_t world_size;          /* N; 1 = whole film                                */
    uint32_t rank;
    uint32_t stripe_height;       /* target stripe height in rows                     */
    uint32_t halo_rows;           /* >= floor(filter radius + 0.5); 0 = 2             */
} dcrt_film_partition;

/* Traversal work counters of the extension / shadow casts
 * (SRayTraversalCounters semantics, SceneRayTrace.h:13-19): node visits =
 * iterationCounter (BVHAccel.inc.hlsl:121), triangle tests, BLAS entries. */
typedef struct dcrt_traversal_stats {
    uint64_t ext_node_visits, ext_triangle_tests, ext_blas_entries;
    uint64_t shadow_node_visits, shadow_triangle_tests, shadow_blas_entries;
    uint64_t ext_launches;
    double ext_kernel_ms;         /* summed HIP-event time of the timed EXTENSION_RAY_CAST launches */
    uint64_t ext_max_node_visits, shadow_max_node_visits;   /* the longest ray of each kind since
                                     the last reset (merged cast kernel, instrumented)      */
    uint64_t material_launches;   /* timed MATERIAL launches (ext_timing) and their summed   */
    double material_kernel_ms;    /* HIP-event time                                          */
    uint64_t control_launches;    /* timed CONTROL(+NEW_PATH) launches, likewise             */
    double control_kernel_ms;
} dcrt_traversal_stats;

/* What the tracer chose for the uploaded scene (diagnostics; bench.py reports it). */
typedef struct dcrt_tracer_info {
    uint32_t path_pool_size;      /* slots after rounding to whole CONTROL workgroups     */
    uint32_t scene_in_lds;        /* 1: the whole BVH + triangles sit in the cast kernel's
                                     LDS scene cache (the LDS-only cast variant)          */
    uint32_t cached_nodes, cached_triangles;   /* how much of the scene the LDS cache holds */
    uint32_t cast_block;          /* cast-kernel workgroup size                          */
    uint32_t traversal_stack;     /* LDS stack rows per lane                             */
    uint32_t material_generic;    /* 1: the any-scene MATERIAL variant                   */
    uint32_t pair_traversal;      /* 1: the cast kernel expands node pairs (scene beyond L2), over the device
                                     child-pair node order */
    uint32_t control_grid, material_grid;   /* CONTROL / MATERIAL workgroups per launch  */
    uint32_t cast_grid;           /* persistent cast-kernel workgroups (resident on the chip) */
    uint32_t material_lds;        /* bytes of MATERIAL's LDS scene copy (0: not used)      */
    uint32_t cast_identity;       /* 1: the cache-only cast kernel without instance space
                                     (every instance's inverse exactly the identity); 2: the
                                     same over the entry-free node order (no BLAS-entry step) */
    uint32_t stack_lds_rows;      /* LDS stack rows per lane of the launched cast kernel: traversal_stack + 2,
                                     or ring_rows                                          */
    uint32_t ring_rows;           /* 0, or the LDS window (rows) of a spilling traversal stack: deeper
                                     entries live in a per-lane global column              */
    uint32_t cast_waves_per_cu;   /* resident waves per CU of the launched cast kernel      */
} dcrt_tracer_info;

typedef struct dcrt_tracer dcrt_tracer;
typedef struct dcrt_scene dcrt_scene;

/* ===== version / device ================================================== */
/* ABI version of this header: bumped whenever a struct changes size or an entry point its
 * meaning (2: dcrt_tracer_info grew cast_waves_per_cu / ring_rows / stack_lds_rows). A caller
 * compiled against another header checks dcrt_abi_version() == DCRT_ABI_VERSION before it
 * passes any struct (a smaller dcrt_tracer_info would be written past its end). */
#define DCRT_ABI_VERSION 2
DCRT_API int dcrt_abi_version(void);
DCRT_API const char* dcrt_version(void);
DCRT_API const char* dcrt_last_error(void);
DCRT_API int dcrt_device_count(int* out_count);

/* ===== host scene: CScene + loaders + BVHAccel (Scene.cpp, BVHAccel.cpp) ==== */
DCRT_API int dcrt_scene_create(dcrt_scene** out_scene);
DCRT_API void dcrt_scene_destroy(dcrt_scene* scene);
/* CScene::Reset (Scene.cpp:626-660): resolution, camera defaults, clears content. */
DCRT_API int dcrt_scene_reset(dcrt_scene* scene, uint32_t resolution_width, uint32_t resolution_height);
/* CScene::LoadFromFile (Scene.cpp:103-624): .obj (WavefrontOBJLoading.cpp) or .xml (SceneXMLLoading.cpp). */
DCRT_API int dcrt_scene_load_from_file(dcrt_scene* scene, const char* path);
/* Equivalent of UI "Create -> Point/Directional Light" (ImGui.cpp:322-331). */
DCRT_API int dcrt_scene_add_punctual_light(dcrt_scene* scene, const float position[3], const float euler_angles[3],
                                           const float color[3], int is_directional);
/* Constant environment light (SceneXMLLoading.cpp:1454-1467); cube may be NULL. */
DCRT_API int dcrt_scene_set_environment_light(dcrt_scene* scene, const float color[3],
                                              const float* cube_rgb, uint32_t cube_size);
DCRT_API int dcrt_scene_set_camera(dcrt_scene* scene, const float position[3], const float euler_angles[3]);
/* Camera / film parameters (Scene.h:118-137): camera_type 0 = pinhole, 1 = thin lens. */
DCRT_API int dcrt_scene_set_lens(dcrt_scene* scene, int camera_type, float fov_x, float focal_length,
                                 float focal_distance, float relative_aperture, uint32_t blade_count,
                                 float aperture_rotation, const float film_size[2]);
DCRT_API int dcrt_scene_set_max_bounce(dcrt_scene* scene, uint32_t max_bounce);
DCRT_API int dcrt_scene_set_filter(dcrt_scene* scene, const dcrt_filter_params* filter);
DCRT_API int dcrt_scene_get_filter(const dcrt_scene* scene, dcrt_filter_params* out_filter);
DCRT_API int dcrt_scene_get_resolution(const dcrt_scene* scene, uint32_t* width, uint32_t* height);
/* Edit material i (UI material editing, ImGui.cpp:560-660). */
DCRT_API int dcrt_scene_get_material_count(const dcrt_scene* scene, uint32_t* out_count);
DCRT_API int dcrt_scene_set_material(dcrt_scene* scene, uint32_t index, int material_type, const float albedo[3],
                                     float roughness, const float ior[3], const float k[3],
                                     int multiscattering, int two_sided);
/* SMaterial as the scene holds it before UpdateMaterialGPUData translates it
 * (Material.h:14-30, Scene.cpp:742-774): the oracle's own flattening reads this. */
typedef struct dcrt_material_setting {
    float albedo[3];
    float roughness;
    float ior[3];
    float opacity;
    float k[3];
    float tiling[2];
    uint32_t material_type;               /* DCRT_MATERIAL_TYPE_* */
    int32_t albedo_texture_index;         /* -1 = INDEX_NONE */
    int32_t opacity_texture_index;
    uint32_t internal_scattering_mode;    /* DCRT_INTERNAL_SCATTERING_* */
    uint32_t multiscattering;             /* m_Multiscattering */
    uint32_t is_two_sided;
    uint32_t has_roughness_texture;
} dcrt_material_setting;
DCRT_API int dcrt_scene_get_material_setting(const dcrt_scene* scene, uint32_t index, dcrt_material_setting* out_setting);
/* The UI's "Multiscattering" checkbox (ImGui.cpp:620-626): only plastic, conductor and
 * dielectric materials have it (DCRT_E_INVALID_ARG for diffuse / thin dielectric). Both
 * loaders force the flag off (SceneXMLLoading.cpp:869, WavefrontOBJLoading.cpp:318). */
DCRT_API int dcrt_scene_set_material_multiscattering(dcrt_scene* scene, uint32_t index, int enable);
/* Material opacity and opacity texture (ImGui.cpp:630-650, SMaterial::m_Opacity /
 * m_OpacityTextureIndex); texture index -1 = none. Recomputes the instance OPAQUE flags
 * (Scene.cpp:57-80, 785-800). */
DCRT_API int dcrt_scene_set_material_opacity(dcrt_scene* scene, uint32_t index, float opacity,
                                             int32_t opacity_texture_index);
/* Shader feature toggles of the scene (Scene.h:140-146: m_IsGGXVNDFSamplingEnabled,
 * m_TraverseBVHFrontToBack, m_IsLightVisible, m_WatertightRayTriangleIntersection,
 * m_AllowAnyHitShader) as DCRT_FEATURE_* bits; get_frame_params reports them. */
DCRT_API int dcrt_scene_set_features(dcrt_scene* scene, uint32_t features);
DCRT_API int dcrt_scene_get_features(const dcrt_scene* scene, uint32_t* out_features);
/* Flattened buffers; pointers stay valid until the scene is modified or destroyed. */
DCRT_API int dcrt_scene_get_flat(dcrt_scene* scene, dcrt_flat_scene* out_flat);
/* The frame constants Render() would upload (WavefrontPathTracer.cpp:372-428). */
DCRT_API int dcrt_scene_get_frame_params(const dcrt_scene* scene, uint32_t frame_seed, dcrt_frame_params* out_params);
/* BVH statistics: node counts and depth (Scene.cpp:169-207). */
DCRT_API int dcrt_scene_get_bvh_info(const dcrt_scene* scene, uint32_t* tlas_nodes, uint32_t* total_nodes,
                                     uint32_t* max_stack_size);

/* The scene content as loaded, before BVHAccel reordered it -- the inputs of
 * Mesh::BuildBVH / BuildTLAS (Mesh.cpp:59-79, Scene.cpp:160-215): mesh i's vertices,
 * triangles (mesh-local vertex indices) and material ids in load order; instance j's
 * mesh index and XMFLOAT4X3 transform (4 rows of 3) in load order. Each mesh's pointers
 * stay valid until the scene is reset, loads more content or is destroyed. Used to check the BVH build against an independent one. */
typedef struct dcrt_obj_mesh dcrt_obj_mesh;
DCRT_API int dcrt_scene_get_content_counts(const dcrt_scene* scene, uint32_t* out_meshes, uint32_t* out_instances);
DCRT_API int dcrt_scene_get_loaded_mesh(dcrt_scene* scene, uint32_t mesh, dcrt_obj_mesh* out_mesh);
DCRT_API int dcrt_scene_get_instance(const dcrt_scene* scene, uint32_t instance, uint32_t* out_mesh_index,
                                     float out_transform[12]);

/* The rest of CScene's state before UpdateLight/Material/InstanceFlagsGPUData and
 * Render() flatten it (Scene.h:118-160, Camera.h, Scene.cpp:570-584, 672-807,
 * WavefrontPathTracer.cpp:372-428): what the oracle's own flattening is driven from. */
typedef struct dcrt_scene_settings {
    uint32_t resolution[2];
    uint32_t max_bounce_count;
    uint32_t camera_type;                 /* 0 = pinhole, 1 = thin lens */
    float fov_x, focal_length, focal_distance, relative_aperture;
    uint32_t aperture_blade_count;
    float aperture_rotation;
    float film_size[2];
    float camera_position[3];             /* CCamera::m_Position */
    float camera_euler_angles[3];         /* CCamera::m_EulerAngles (pitch, yaw, roll) */
    uint32_t features;                    /* DCRT_FEATURE_* */
    uint32_t has_environment_light;
    float environment_color[3];           /* SEnvironmentLight::m_Color */
    const float* env_cube_rgb;            /* the environment texture (NULL = none) */
    uint32_t env_cube_size;
    uint32_t mesh_light_count, punctual_light_count, material_count, texture_count;
} dcrt_scene_settings;
DCRT_API int dcrt_scene_get_settings(const dcrt_scene* scene, dcrt_scene_settings* out_settings);
/* SMeshLight i (Scene.h:42-46): the instance it lights (load order) and its radiance. */
DCRT_API int dcrt_scene_get_mesh_light(const dcrt_scene* scene, uint32_t index, uint32_t* out_instance,
                                       float out_color[3]);
/* SPunctualLight i (Scene.h:27-40). */
DCRT_API int dcrt_scene_get_punctual_light(const dcrt_scene* scene, uint32_t index, float out_position[3],
                                           float out_euler_angles[3], float out_color[3], int* out_is_directional);
/* SMeshInstance::m_MaterialIdOverride of instance j (load order; 0xFFFFFFFF = none). */
DCRT_API int dcrt_scene_get_instance_material_override(const dcrt_scene* scene, uint32_t instance,
                                                       uint32_t* out_override);

/* Standalone BVHAccel::BuildBLAS + PackBVH over one triangle soup
 * (BVHAccel.cpp:376-447). out_nodes holds 2*triangle_count-1 entries at most;
 * out_reordered_indices 3*triangle_count; out_reordered_triangles triangle_count. */
DCRT_API int dcrt_bvh_build_blas(const dcrt_vertex* vertices, const uint32_t* indices, uint32_t triangle_count,
                                 dcrt_bvh_node* out_nodes, uint32_t* out_node_count,
                                 uint32_t* out_reordered_indices, uint32_t* out_reordered_triangles,
                                 uint32_t* out_max_depth, uint32_t* out_max_stack_size);

/* OBJ loading into meshes, before any BVH build:
 *  - DCRT_OBJ_SCENE_LAYOUT: the meshes CScene::LoadFromWavefrontOBJFile builds
 *    (WavefrontOBJLoading.cpp:409-465): one mesh per OBJ shape, RH->LH transform
 *    (x negated), winding change, V flip, material ids offset by material_index_base;
 *  - 0: Mesh::LoadFromWavefrontOBJFile as the XML loader calls it
 *    (SceneXMLLoading.cpp:1334-1341): every shape into one mesh, no transform.
 * Vertices carry the MikkTSpace tangents (WavefrontOBJLoading.cpp:147-153). */
#define DCRT_OBJ_SCENE_LAYOUT 1u
typedef struct dcrt_obj_meshes dcrt_obj_meshes;
struct dcrt_obj_mesh {
    const dcrt_vertex* vertices;
    uint32_t vertex_count;
    const uint32_t* indices;          /* 3 per triangle                         */
    const uint32_t* material_ids;     /* 1 per triangle (0xFFFFFFFF = none)      */
    uint32_t triangle_count;
};
/* The translated OBJ materials (WavefrontOBJLoading.cpp:305-338) of a load. */
typedef struct dcrt_obj_material {
    float albedo[3], ior, roughness, opacity;
    int32_t albedo_texture_index, opacity_texture_index;
} dcrt_obj_material;
DCRT_API int dcrt_obj_load(const char* path, uint32_t flags, uint32_t material_index_base, dcrt_obj_meshes** out);
DCRT_API int dcrt_obj_mesh_count(const dcrt_obj_meshes* meshes, uint32_t* out_count);
DCRT_API int dcrt_obj_get_mesh(const dcrt_obj_meshes* meshes, uint32_t index, dcrt_obj_mesh* out_mesh);
DCRT_API int dcrt_obj_material_count(const dcrt_obj_meshes* meshes, uint32_t* out_count);
DCRT_API int dcrt_obj_get_material(const dcrt_obj_meshes* meshes, uint32_t index, dcrt_obj_material* out_material);
DCRT_API void dcrt_obj_free(dcrt_obj_meshes* meshes);
/* The element / attribute tree the Mitsuba XML loader parses from `path` (what
 * SceneXMLLoading.cpp's walk over rapidxml's DOM reads, :247-581): per element in document
 * order "E<name>\n", "A<name>=<value>\n" per attribute, its children, "/\n". Writes at most
 * `capacity` bytes; *out_length = the full length (DCRT_E_LIMIT if it did not fit). */
DCRT_API int dcrt_xml_dump_tree(const char* path, char* out, uint32_t capacity, uint32_t* out_length);

/* ===== tracer: CWavefrontPathTracer on MI355X ============================== */
DCRT_API int dcrt_tracer_create(const dcrt_tracer_config* config, dcrt_tracer** out_tracer);  /* Create()  */
DCRT_API void dcrt_tracer_destroy(dcrt_tracer* tracer);                                        /* Destroy() */
/* OnSceneLoaded + the uploads of Scene.cpp:273-608. Copies everything to HBM. */
DCRT_API int dcrt_tracer_upload_scene(dcrt_tracer* tracer, const dcrt_flat_scene* scene);
DCRT_API int dcrt_tracer_set_frame_params(dcrt_tracer* tracer, const dcrt_frame_params* params);
DCRT_API int dcrt_tracer_set_film_partition(dcrt_tracer* tracer, const dcrt_film_partition* partition);
/* Explicit film bands (cost-balanced film tiling): the tracer owns the rows of the
 * band_count ranges [bands[2i], bands[2i+1]) (ascending, disjoint, non-empty; rows past the film
 * are ignored), path-traces them plus halo_rows rows beyond each band (0 = 2) and convolves only
 * its own rows, so any cut of the film dealt to tracers sums to the one-tracer film bit for bit.
 * Replaces a dcrt_film_partition (and a later dcrt_tracer_set_film_partition replaces the bands). */
DCRT_API int dcrt_tracer_set_film_bands(dcrt_tracer* tracer, const uint32_t* bands, uint32_t band_count, uint32_t halo_rows);
/* Row-cost probe: enable != 0 clears and starts per-film-row counters of the rays the wavefront
 * casts (each MATERIAL pass adds its item's extension ray and, if it casts one, its shadow ray);
 * the counts are exact and schedule-independent. 0 stops them. Not a reference entry point: the
 * input of cost-balanced bands (directcomputeraytracing_amd/partition.py balanced_bands). */
DCRT_API int dcrt_tracer_set_row_cost_probe(dcrt_tracer* tracer, int enable);
DCRT_API int dcrt_tracer_read_row_cost(dcrt_tracer* tracer, uint32_t* out_rays_per_row);   /* film height entries */
/* Render(): run up to max_iterations wavefront iterations (0 = config value). */
DCRT_API int dcrt_tracer_render(dcrt_tracer* tracer, uint32_t max_iterations);
/* Render whole images: image s uses frame seed first_seed + s. Images are path-traced in
 * batches that share the path pool (new paths of the next image start as soon as slots
 * are idle); a completed batch is convolved into the film (SampleConvolution) image by
 * image, in order, so the film is the same as with one image at a time. */
DCRT_API int dcrt_tracer_render_images(dcrt_tracer* tracer, uint32_t first_seed, uint32_t image_count,
                                       const dcrt_filter_params* filter);
/* render_images generalised for pipelines that share a film's rows by interleaving images:
 * image k of the call has frame seed first_seed + k * seed_stride; with convolve == 0 the film
 * pass is skipped and image k's samples stay in slot k (at most 256 images, one batch) for
 * dcrt_tracer_image_sample_ptrs / dcrt_tracer_accumulate_images. No reference counterpart. */
DCRT_API int dcrt_tracer_render_images_strided(dcrt_tracer* tracer, uint32_t first_seed, uint32_t seed_stride,
                                               uint32_t image_count, int convolve, const dcrt_filter_params* filter);
/* Device pointers of image `image`'s sample textures (W*H R32G32F / RGBA32F) after a
 * render_images_strided call with convolve == 0. */
DCRT_API int dcrt_tracer_image_sample_ptrs(dcrt_tracer* tracer, uint32_t image, void** out_position, void** out_value);
/* SampleConvolution over image_count images whose sample textures sit at the given device
 * pointers (host arrays of image_count pointers each; every texture W*H of this tracer's film,
 * on its device), convolved in list order into this tracer's film (its own rows): the film of
 * several pipelines' interleaved images, bit for bit the one-pipeline film when the list is in
 * image order. Synchronous. */
DCRT_API int dcrt_tracer_accumulate_images(dcrt_tracer* tracer, const void* const* d_positions, const void* const* d_values,
                                           uint32_t image_count, const dcrt_filter_params* filter);
/* Allocate / capture now what dcrt_tracer_render_images(image_count) would on its first
 * call (the batch's sample textures, the iteration graph), e.g. before a timed region.
 * No reference counterpart (the reference allocates at Create and scene load). */
DCRT_API int dcrt_tracer_prepare_images(dcrt_tracer* tracer, uint32_t image_count);
/* Images per render_images batch (0 = automatic: as many as the path pool holds, at most
 * 64, the images cut into equal batches). */
DCRT_API int dcrt_tracer_set_image_batch(dcrt_tracer* tracer, uint32_t images);
/* 0 = wavefront (CWavefrontPathTracer, default), 1 = megakernel (CMegakernelPathTracer,
 * MegakernelPathTracing.hlsl) for dcrt_tracer_render_images. */
DCRT_API int dcrt_tracer_set_mode(dcrt_tracer* tracer, int mode);
DCRT_API int dcrt_tracer_reset_image(dcrt_tracer* tracer);                                     /* ResetImage() */
DCRT_API int dcrt_tracer_is_image_complete(dcrt_tracer* tracer, int* out_complete);           /* IsImageComplete() */
DCRT_API int dcrt_tracer_acquire_film_clear_trigger(dcrt_tracer* tracer, int* out_trigger);    /* AcquireFilmClearTrigger() */
DCRT_API int dcrt_tracer_clear_film(dcrt_tracer* tracer);
DCRT_API int dcrt_tracer_accumulate_film(dcrt_tracer* tracer, const dcrt_filter_params* filter);
DCRT_API int dcrt_tracer_read_film(dcrt_tracer* tracer, float* out_rgba);                      /* W*H*4 floats */
DCRT_API int dcrt_tracer_read_samples(dcrt_tracer* tracer, float* out_position, float* out_value); /* W*H*2, W*H*4 */
DCRT_API int dcrt_tracer_read_rng(dcrt_tracer* tracer, uint32_t* out_state);                   /* W*H*4 (debug_rng) */
DCRT_API int dcrt_tracer_film_device_ptr(dcrt_tracer* tracer, void** out_ptr);
/* The current image's sample textures in device memory (m_SamplePositionTexture R32G32F and
 * m_SampleValueTexture RGBA32F, row-major W x H of the frame resolution; Scene.cpp:863-885),
 * written by CONTROL / MATERIAL (WriteSample, RayTracingCommon.inc.hlsl:118-122): what the
 * reference's L1 SampleConvolution pass reads (SampleConvolution.cpp:89-170,
 * LaunchRendererLoop.cpp:295-297). Valid until the resolution or the image batch changes;
 * dcrt_tracer_accumulate_film is that pass on the tracer's own film. */
DCRT_API int dcrt_tracer_sample_device_ptrs(dcrt_tracer* tracer, void** out_position, void** out_value);
/* Device-to-device copy of the RGBA32F film (W*H*4 floats) into d_dst, e.g. an
 * RCCL buffer for the multi-GPU reduce; synchronous with the tracer stream. */
DCRT_API int dcrt_tracer_copy_film_device(dcrt_tracer* tracer, void* d_dst);
/* film += d_src (W*H*4 floats in device memory of the tracer's device), on the tracer
 * stream, synchronous. Combines the films of film partitions rendered by several
 * tracers of one GPU (concurrent pipelines): their supports are disjoint, so the sum
 * is the single-tracer film bit for bit. No reference counterpart (the reference has
 * one pipeline per device). */
DCRT_API int dcrt_tracer_add_film_device(dcrt_tracer* tracer, const void* d_src);
DCRT_API int dcrt_tracer_counters(dcrt_tracer* tracer, dcrt_ray_stats* out_stats);
/* counters != 0: traversal work counters in the cast kernels; ext_timing != 0: plain
 * (non-graph) launches with HIP events around every EXTENSION_RAY_CAST, MATERIAL and
 * CONTROL launch. */
DCRT_API int dcrt_tracer_set_instrumentation(dcrt_tracer* tracer, int counters, int ext_timing);
DCRT_API int dcrt_tracer_traversal_stats(dcrt_tracer* tracer, dcrt_traversal_stats* out_stats);
DCRT_API int dcrt_tracer_reset_stats(dcrt_tracer* tracer);
DCRT_API int dcrt_tracer_get_info(dcrt_tracer* tracer, dcrt_tracer_info* out_info);
/* Test hook of the spilling traversal stack (dcrt_tracer_info.ring_rows): the stack entries the
   ring cast kernel has moved to its spill columns since the scene upload (nonzero words of the
   zero-initialised columns; no stack entry is 0). 0 when the scene keeps its whole stack in LDS. */
DCRT_API int dcrt_tracer_debug_ring_spills(dcrt_tracer* tracer, uint64_t* out_words);
DCRT_API int dcrt_tracer_synchronize(dcrt_tracer* tracer);
DCRT_API int dcrt_tracer_get_luts(dcrt_tracer* tracer, dcrt_bxdf_luts* out_luts);
DCRT_API int dcrt_tracer_set_luts(dcrt_tracer* tracer, const dcrt_bxdf_luts* luts);

/* Kernel-level entry points used by the parity tests and the roofline bench:
 * one EXTENSION_RAY_CAST / SHADOW_RAY_CAST launch over a host ray batch. */
DCRT_API int dcrt_tracer_trace_rays(dcrt_tracer* tracer, const dcrt_ray* rays, uint32_t count, dcrt_ray_hit* out_hits,
                                    uint32_t features);
DCRT_API int dcrt_tracer_occluded(dcrt_tracer* tracer, const dcrt_ray* rays, uint32_t count, uint32_t* out_occluded,
                                  uint32_t features);
/* Device-resident variant for timing: rays/hits already in HBM, launched on the tracer stream. */
DCRT_API int dcrt_tracer_trace_rays_device(dcrt_tracer* tracer, const void* d_rays, uint32_t count, void* d_hits,
                                           uint32_t features);

/* ===== post-processing + image output (PostProcessing.cpp, PostProcessings.hlsl,
 *       SumLuminance.hlsl, SaveImageToFile.cpp) ============================== */
typedef struct dcrt_postfx_params {
    int32_t enabled;          /* m_IsPostFXEnabled (default 1); 0 = rgb / w only          */
    int32_t auto_exposure;    /* m_IsAutoExposureEnabled (default 1): log-average luminance */
    float ev100;              /* manual EV100: CalculateEV100(N, t, ISO) or m_ManualEV100  */
    float luminance_white;    /* m_LuminanceWhite (default 1), Reinhard max white          */
} dcrt_postfx_params;
/* Defaults of Scene.h:181-185 with EV100 from the scene's camera (PostProcessing.cpp:39-42). */
DCRT_API int dcrt_scene_get_postfx_params(const dcrt_scene* scene, dcrt_postfx_params* out_params);
/* The 255 linear thresholds between consecutive sRGB8 codes (R8G8B8A8_UNORM_SRGB encode). */
DCRT_API int dcrt_srgb_encode_thresholds(float out_thresholds[255]);
/* Tone-map the film into sRGB8 RGBA (W*H*4 bytes); optional sum of log luminance (auto exposure). */
DCRT_API int dcrt_tracer_resolve_image(dcrt_tracer* tracer, const dcrt_postfx_params* params, uint8_t* out_rgba8,
                                       float* out_sum_log_luminance);
/* 24-bit BMP writer ("Save Image to File", SaveImageToFile.cpp:92-182). */
DCRT_API int dcrt_write_bmp(const char* path, uint32_t width, uint32_t height, const uint8_t* rgba8);

/* Deterministic transcendental helpers shared by kernels (parity tests): function 0 sin, 1 cos,
   2 exp, 3 atan, 4 log (the det_* polynomials), 5 the fast reciprocal rcp_ieee, 6 IEEE 1/x. */
DCRT_API int dcrt_device_math_eval(dcrt_tracer* tracer, int function, const float* x, uint32_t count, float* out_y);

#ifdef __cplusplus
}
#endif

#endif /* DCRT_H_ */
