/*
 * nori_gpu.h -- C ABI of the MI355X wavefront path tracer (libnori_gpu.so).
 *
 * This is the drop-in boundary for Nori's render path.  The reference binds
 * the path through C++ virtuals, not an FFI; each entry point below names the
 * reference interface it replaces (paths relative to the reference checkout):
 *
 *   nori_scene_load_xml   <- loadFromXML()                src/parser.cpp:28-338
 *                            + NoriObjectFactory::createInstance  include/nori/object.h:160-165
 *                            + Scene::activate()          src/scene.cpp:43-61
 *   nori_gpu_create       <- Scene::activate's BVH::build src/bvh.cpp:329-382 (flatten + upload)
 *                            and Integrator::preprocess    src/photonmapper.cpp:41-117 (photon map)
 *   nori_gpu_render       <- RenderThread::renderScene's pass loop
 *                            src/render.cpp:173-250 (tbb::parallel_for over blocks,
 *                            renderBlock render.cpp:80-133, Integrator::Li
 *                            include/nori/integrator.h:55, ImageBlock::put
 *                            src/block.cpp:93-133)
 *   nori_gpu_trace        <- Scene::rayIntersect(ray, its) / rayIntersect(ray)
 *                            include/nori/scene.h:93-115 -> BVH::rayIntersect src/bvh.cpp:404-462
 *   nori_gpu_cancel       <- RenderThread::stopRendering  src/render.cpp:63-71
 *   nori_gpu_progress     <- RenderThread::getProgress    src/render.cpp:73-78
 *   nori_film_develop     <- ImageBlock::toBitmap         src/block.cpp:76-82
 *   nori_write_exr        <- Bitmap::save                 src/bitmap.cpp:82-107
 *   nori_read_exr         <- Bitmap::Bitmap(filename)     src/bitmap.cpp:23-80
 *   nori_read_image       <- stbi_load in ImageTexture / NormalMap  src/imagetexture.cpp:69-85
 *   nori_write_png        <- Bitmap::saveToLDR            src/bitmap.cpp:122-139
 *   nori_film_variance    <- renderScene's variance image src/render.cpp:164-169,190-245
 *   nori_denoise          <- denoiser/denoiser.py:53-66 (NL-means)
 *   nori_scene_bvh_info   <- BVH::build/statistics        src/bvh.cpp:329-402
 *   nori_scene_scan_list  (introspection: the small-scene scan list and its
 *                          exact in-plane filters, for the CPU tests)
 *   nori_gpu_comm_*, nori_gpu_render_sharded
 *                         <- the same pass loop spread over the GPUs of a node,
 *                            one process per GPU; the cross-GPU film merge is
 *                            ImageBlock::put(block) src/block.cpp:124-133 as an
 *                            RCCL sum over xGMI (the reference has no multi-device path)
 *
 * Rules of the ABI: plain C types only, no exceptions cross it, every call
 * returns an int status (NORI_OK = 0, negative = error) and the message of
 * the last failure on the calling thread is nori_gpu_last_error().  All
 * scene arrays are copied at nori_gpu_create(); the caller owns output
 * buffers.  Arithmetic on the path is fp32 (Eigen float in the reference).
 */
#ifndef NORI_GPU_H
#define NORI_GPU_H

#ifndef __HIPCC_RTC__  /* (the library compiles its scan kernels at run time with hipRTC, which has size_t built in) */
#include <stddef.h>
#endif
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Bumped whenever an exported signature or a shared struct changes (6: the
 * leading status argument of nori_gpu_comm_timeout; 7: nori_gpu_stats.nee_inline);
 * the Python binding and the C++ adapter refuse a library of another version. */
#define NORI_GPU_ABI_VERSION 7

/* ---- status codes ------------------------------------------------------ */
#define NORI_OK               0
#define NORI_ERR_INVALID     -1   /* bad argument                        */
#define NORI_ERR_IO          -2   /* file could not be read / written    */
#define NORI_ERR_PARSE       -3   /* XML / OBJ syntax or property error  */
#define NORI_ERR_UNSUPPORTED -4   /* plugin outside this path's scope    */
#define NORI_ERR_HIP         -5   /* HIP runtime failure / no device     */
#define NORI_ERR_CANCELLED   -6   /* nori_gpu_cancel() was honoured      */
#define NORI_ERR_OOM         -7   /* device allocation failed            */

/* ---- plugin kinds (XML `type` names in comments) ------------------------ */
enum { NORI_SHAPE_MESH = 0 /* "obj" */, NORI_SHAPE_SPHERE = 1 /* "sphere" */ };
enum {
    NORI_BSDF_DIFFUSE = 0,    /* "diffuse"    src/diffuse.cpp    */
    NORI_BSDF_MIRROR = 1,     /* "mirror"     src/mirror.cpp     */
    NORI_BSDF_DIELECTRIC = 2, /* "dielectric" src/dielectric.cpp */
    NORI_BSDF_MICROFACET = 3, /* "microfacet" src/microfacet.cpp */
    NORI_BSDF_DISNEY = 4      /* "disney"     src/disney.cpp     */
};
enum {
    NORI_EMITTER_AREA = 0,    /* "area"      src/arealight.cpp  */
    NORI_EMITTER_ENVMAP = 1,  /* "envmap"    src/envmap.cpp     */
    NORI_EMITTER_POINT = 2,   /* "point"     src/pointlight.cpp */
    NORI_EMITTER_SPOT = 3     /* "spotlight" src/spotlight.cpp  */
};
enum {
    NORI_TEXTURE_CONSTANT = 0,     /* "constant_color"     src/consttexture.cpp */
    NORI_TEXTURE_CHECKERBOARD = 1, /* "checkerboard_color" src/checkerboard.cpp */
    NORI_TEXTURE_IMAGE = 2         /* "ImageTexture"       src/imagetexture.cpp */
};
/* ImageWrap (include/nori/common.h:273-283): "repeat" | "clamp" */
enum { NORI_WRAP_REPEAT = 0, NORI_WRAP_CLAMP = 1 };
enum {
    NORI_CAMERA_PERSPECTIVE = 0,   /* "perspective"    src/perspective.cpp    */
    NORI_CAMERA_THINLENS = 1,      /* "thinlens"       src/thinlens.cpp       */
    NORI_CAMERA_ADVANCED = 2       /* "advancedCamera" src/advancedCamera.cpp */
};
enum {
    NORI_INTEGRATOR_PATH_MATS = 0,  /* "path_mats"  src/path_mats.cpp  */
    NORI_INTEGRATOR_PATH_MIS = 1,   /* "path_mis"   src/path_mis.cpp   */
    NORI_INTEGRATOR_VOLUMETRIC = 2, /* "volumetric" src/volumetric.cpp */
    /* one-bounce integrators (a fixed number of rays per camera sample) */
    NORI_INTEGRATOR_NORMALS = 3,    /* "normals"     src/normals.cpp           */
    NORI_INTEGRATOR_AV = 4,         /* "av"          src/averagevisibility.cpp */
    NORI_INTEGRATOR_DIRECT = 5,     /* "direct"      src/direct.cpp            */
    NORI_INTEGRATOR_DIRECT_EMS = 6, /* "direct_ems"  src/direct_ems.cpp        */
    NORI_INTEGRATOR_DIRECT_MATS = 7,/* "direct_mats" src/direct_mats.cpp       */
    NORI_INTEGRATOR_DIRECT_MIS = 8, /* "direct_mis"  src/direct_mis.cpp        */
    NORI_INTEGRATOR_PHOTONMAPPER = 9 /* "photonmapper" src/photonmapper.cpp    */
};
enum {
    NORI_FILTER_GAUSSIAN = 0, NORI_FILTER_MITCHELL = 1, NORI_FILTER_TENT = 2,
    NORI_FILTER_BOX = 3, NORI_FILTER_WINDOWED = 4     /* src/rfilter.cpp */
};
/* Random-number stream layout.
 *  WAVE : one pcg32 stream per (pass k, pixel) sample -- counter based, the
 *         layout the GPU uses; identical in the CPU oracle.
 *  BLOCK: the reference's layout: one stream per 32x32 block seeded with
 *         seed(offset.x, offset.y) and consumed serially over pixels and
 *         passes (src/independent.cpp:48-67, src/render.cpp:212-216).  CPU
 *         oracle only. */
enum { NORI_RNG_WAVE = 0, NORI_RNG_BLOCK = 1 };

#define NORI_BLOCK_SIZE 32           /* include/nori/block.h:30   */
#define NORI_FILTER_RESOLUTION 32    /* include/nori/rfilter.h:25 */
#define NORI_EPSILON 1e-4f           /* include/nori/common.h:52  */

/* ---- flattened scene (POD) ---------------------------------------------- */
typedef struct nori_shape_desc {
    int32_t type;                 /* NORI_SHAPE_*                              */
    uint32_t tri_offset;          /* mesh: first triangle in indices[]         */
    uint32_t tri_count;           /* mesh: triangle count (sphere: 1 primitive) */
    uint32_t vtx_offset;          /* mesh: first vertex in positions[]         */
    uint32_t vtx_count;
    int32_t has_normals;          /* mesh: per-vertex normals present          */
    int32_t has_uvs;              /* mesh: per-vertex uvs present              */
    float center[3];              /* sphere                                    */
    float radius;                 /* sphere                                    */
    int32_t bsdf;                 /* index into bsdfs[]                         */
    int32_t emitter;              /* index into emitters[] or -1               */
    int32_t normal_map;           /* "NormalMap" texture named "normal": index
                                     into images[] or -1 (shape.cpp:59-67;
                                     applied to meshes with normals, mesh.cpp:147-155) */
} nori_shape_desc;

typedef struct nori_bsdf_desc {
    int32_t type;                 /* NORI_BSDF_*                               */
    float albedo[3];              /* diffuse: constant_color albedo (def 0.5)  */
    float int_ior, ext_ior;       /* dielectric / microfacet                   */
    float alpha;                  /* microfacet                                */
    float kd[3];                  /* microfacet                                */
    float base_color[3];          /* disney                                    */
    float metallic, specular, roughness, sheen, sheen_tint, specular_tint;
    int32_t albedo_texture;       /* diffuse: NORI_TEXTURE_* of the albedo; a
                                     checkerboard uses albedo as value1        */
    float tex_value2[3];          /* checkerboard value2                        */
    float tex_delta[2], tex_scale[2]; /* checkerboard delta (def 0), scale (def 1) */
    int32_t albedo_image;         /* NORI_TEXTURE_IMAGE: index into images[], else -1 */
} nori_bsdf_desc;

/* An 8-bit RGB image of an ImageTexture or NormalMap, as stbi_load(path, ..,
 * STBI_rgb) returns it: width x height x 3 bytes, top row first. */
typedef struct nori_image_desc {
    int32_t width, height;
    int32_t wrap;                 /* NORI_WRAP_*                                */
    const uint8_t *rgb;
} nori_image_desc;

typedef struct nori_emitter_desc {
    int32_t type;                 /* NORI_EMITTER_*                            */
    int32_t shape;                /* attached shape index (area, envmap)       */
    float radiance[3];            /* area                                      */
    float weight;                 /* envmap                                    */
    float lum_scale[3];           /* envmap luminanceScale                     */
    int32_t env_rows, env_cols;   /* envmap: Bitmap rows x cols                */
    const float *env_rgb;         /* envmap: rows*cols*3 floats (row-major)    */
    float position[3];            /* point / spot                              */
    float power[3];               /* point: power | spot: color                */
    float direction[3];           /* spot: normalized direction                */
    float cos_falloff_start;      /* spot: cos(falloffStart deg)               */
    float cos_total_width;        /* spot: cos(totalWidth deg)                 */
} nori_emitter_desc;

typedef struct nori_camera_desc {
    int32_t width, height;
    float fov, near_clip, far_clip;
    float camera_to_world[16];    /* row-major 4x4                             */
    float sample_to_camera[16];   /* row-major 4x4 (perspective.cpp:53-82)     */
    int32_t filter_type;          /* NORI_FILTER_*                             */
    float filter_radius;
    float filter_p0, filter_p1;   /* gaussian: stddev | mitchell: B, C | windowed: tau */
    int32_t camera_type;          /* NORI_CAMERA_*                             */
    float lens_radius;            /* thinlens / advancedCamera "lensRadius"    */
    float focal_distance;         /* "focalDist"                               */
    float distortion[2];          /* advancedCamera barrel distortion k1, k2   */
    float chromatic[3];           /* advancedCamera "chromaticAberation"       */
} nori_camera_desc;

typedef struct nori_medium_desc {
    int32_t present;
    float sigma_a[3], sigma_s[3];
    float box_min[3], box_max[3]; /* origin -/+ |box_size| (medium.cpp:16-18)  */
} nori_medium_desc;

typedef struct nori_scene_desc {
    uint32_t abi_version;
    uint32_t num_vertices;
    const float *positions;       /* 3*num_vertices                            */
    const float *normals;         /* 3*num_vertices (zeros where absent)       */
    const float *uvs;             /* 2*num_vertices (zeros where absent)       */
    uint32_t num_triangles;
    const uint32_t *indices;      /* 3*num_triangles, global vertex ids        */
    uint32_t num_shapes;
    const nori_shape_desc *shapes;      /* BVH primitive order = shape order  */
    uint32_t num_bsdfs;
    const nori_bsdf_desc *bsdfs;
    uint32_t num_emitters;
    const nori_emitter_desc *emitters;  /* Scene::addChild order (scene.cpp:63-104) */
    nori_camera_desc camera;
    nori_medium_desc medium;
    int32_t integrator;           /* NORI_INTEGRATOR_*                          */
    uint32_t sample_count;        /* independent sampler sampleCount = spp      */
    float av_length;              /* "av" integrator ray length                 */
    uint32_t photon_count;        /* photonmapper "photonCount" (photons stored) */
    float photon_radius;          /* photonmapper "photonRadius" (0 in the XML:
                                     scene box diagonal / 500, photonmapper.cpp:55-56) */
    uint32_t num_images;          /* image textures and normal maps            */
    const nori_image_desc *images;
} nori_scene_desc;

/* ---- host-side scene loading (the plugin boundary) ----------------------- */
typedef struct nori_scene nori_scene;

/* Parse a Nori XML scene (same tags, `type` names, property names and
 * defaults as the reference).  width/height/spp > 0 override the XML. */
int nori_scene_load_xml(const char *path, int width, int height, int spp, nori_scene **out);
const nori_scene_desc *nori_scene_get_desc(const nori_scene *scene);
void nori_scene_free(nori_scene *scene);

/* Film border (ceil(radius - 0.5), block.cpp:57) and the 33-entry filter
 * table (block.cpp:59-64) for the scene's reconstruction filter. */
int nori_film_border(const nori_scene_desc *scene);
int nori_filter_table(const nori_scene_desc *scene, float table[NORI_FILTER_RESOLUTION + 1]);
/* RGBW film (H+2b)x(W+2b)x4 -> RGB bitmap HxWx3 divided by the filter weight
 * (ImageBlock::toBitmap, Color4f::divideByFilterWeight color.h:113-118). */
int nori_film_develop(const nori_scene_desc *scene, const float *rgbw, float *rgb);
/* Write an RGB float image as an uncompressed scanline OpenEXR file. */
int nori_write_exr(const char *path, const float *rgb, int width, int height);
/* Bitmap::saveToLDR (bitmap.cpp:109-139): sRGB transfer curve, x255 + 0.5,
 * clamp to [0, 255], 8-bit RGB PNG (zlib deflate, filter type 0). */
int nori_write_png(const char *path, const float *rgb, int width, int height);
/* Variance of each pixel's mean radiance from the statistics of
 * render_desc.variance_out (H x W x 8): out (H x W x 3) =
 * (sum L^2 - (sum L)^2 / n) / (n (n - 1)) per channel, in double precision;
 * 0 where n < 2.  The reference's own estimator (render.cpp:235-247,
 * 263-276: the spread of the running mean over the passes) does not estimate
 * the pixel variance; this one does (deviation D5). */
int nori_film_variance(const nori_scene_desc *scene, const float *stats, float *out);

/* NL-means denoiser <- denoiser/denoiser.py:53-66 on the GPU.  rgb: H x W x 3
 * image, variance: H x W per-pixel variance (the script's grey variance
 * image), out: H x W x 3.  radius = r (offsets in [-r, r]^2, <= 8), patch = f
 * (box filters of width 2(f-1)+1, 1 <= f <= 5), k = the script's k (0.02).
 * mode 0 reproduces the script's d2 (both variance terms 2 var(neighbour)),
 * mode 1 the textbook form (var_p + min(var_p, var_q), var_p + var_q).
 * Neighbours wrap around the image (np.roll), the box filters zero-pad
 * (convolve2d mode 'same').  Host buffers; runs on `device`. */
int nori_denoise(int device, const float *rgb, const float *variance, int width, int height, int radius,
                 int patch, float k, int mode, float *out);
/* Read the R, G, B planes of a scanline OpenEXR file (NONE/ZIPS/ZIP, HALF or
 * FLOAT) <- Bitmap::Bitmap (bitmap.cpp:23-80).  Call with rgb = NULL to get
 * the size, then with a buffer of 3*width*height floats (row-major). */
int nori_read_exr(const char *path, int *width, int *height, float *rgb);
/* Decode an image texture file as the reference's stbi_load(path, .., STBI_rgb)
 * does (stb_image v1.39: baseline JPEG, 8-bit PNG) <- ImageTexture / NormalMap
 * constructors (imagetexture.cpp:69-85, normalmap.cpp:69-85).  Call with
 * rgb = NULL to get the size, then with 3*width*height bytes (top row first). */
int nori_read_image(const char *path, int *width, int *height, uint8_t *rgb);

/* Host-side BVH build of the scene exactly as nori_gpu_create builds it (no
 * device needed) <- BVH::build + BVH::statistics (bvh.cpp:329-402): node count
 * and SAH cost of the reference-layout tree, device node count and depth, and
 * an FNV-1a hash of the leaf-order primitive ids. */
typedef struct nori_bvh_info {
    uint32_t ref_nodes;       /* nodes reachable in the reference layout      */
    uint32_t device_nodes;    /* 64-byte inner nodes of the device layout     */
    uint32_t depth;           /* inner-node depth of the device tree          */
    uint32_t num_prims;
    float sah_cost;           /* BVH::statistics cost of the root             */
    uint32_t pad;
    uint64_t order_hash;      /* FNV-1a over the leaf-order primitive ids     */
} nori_bvh_info;
int nori_scene_bvh_info(const nori_scene_desc *scene, nori_bvh_info *out);

/* Host-side scan list of a small scene (<= 64 primitives) exactly as
 * nori_gpu_create builds it (no device needed; introspection for tests -- no
 * reference counterpart): the primitive records in scan order (12 floats
 * each: v0 | prim id, e1 | sphere flag, e2 | leaf position; a sphere is
 * (centre | id, radius, ...)), per axis-plane pair the plane coordinate and
 * the in-plane filter of the binned extension kernel (8 floats: mid_B,
 * half_B + Kb, mid_C, half_C + Kb, Ka, c, 0, 0).  Call with null arrays for
 * the counts; records = 0 for a BVH scene. */
typedef struct nori_scan_info {
    uint32_t records;       /* 12-float records (pairs, other triangles padded, spheres) */
    uint32_t pairs;         /* axis-plane pairs: records 2g, 2g+1                          */
    uint32_t plane_end[3];  /* pairs of axis <= a                                          */
    uint32_t tris;          /* triangle records                                            */
} nori_scan_info;
int nori_scene_scan_list(const nori_scene_desc *scene, nori_scan_info *info, float *records, float *plane_c,
                         float *plane_f);

/* Compiles the scene's scan kernels specialised for its scan list (the
 * hipRTC program nori_gpu_create loads for scan-mode scenes, rtc.hip) for the
 * target `arch` (e.g. "gfx950"), without a device: *code_bytes = the code
 * object's size (0 for a BVH scene), *ms = the compile time (or cache read).
 * NORI_ERR_UNSUPPORTED when hipRTC is missing or the compile fails
 * (nori_gpu_last_error holds the log). */
int nori_scene_scan_rtc(const nori_scene_desc *scene, const char *arch, size_t *code_bytes, double *ms);

/* ---- GPU context ----------------------------------------------------------- */
typedef struct nori_gpu_ctx nori_gpu_ctx;

typedef struct nori_gpu_render_desc {
    uint32_t pass_begin;          /* first sample pass k                        */
    uint32_t pass_count;          /* passes to render (0 = scene spp)           */
    uint32_t num_blocks;          /* 0 = every 32x32 block of the frame         */
    const uint32_t *block_ids;    /* host array, id = by*nbx + bx (block.cpp:168) */
    uint64_t seed;                /* stream seed mixed into every sample id     */
    int32_t output_on_device;     /* rgbw_out is a device pointer on ctx device */
    uint32_t path_pool;           /* paths in flight (0 = default)              */
    int32_t timing;               /* nonzero: HIP events around every launch    */
    /* Optional per-pixel sample statistics, H x W x 8 floats ADDED into
     * (host or device memory like rgbw_out): sum of L (r, g, b), sum of L^2
     * (r, g, b), valid sample count, 0 -- of every valid sample in the pixel
     * it was taken in (unfiltered).  nori_film_variance turns them into the
     * variance of the pixel mean.  NULL: not collected. */
    float *variance_out;
} nori_gpu_render_desc;

typedef struct nori_gpu_stats {
    uint64_t samples;             /* camera samples completed                   */
    uint64_t invalid_samples;     /* NaN/Inf/negative radiance, dropped (block.cpp:94-98) */
    uint64_t rays_closest;        /* extension rays traced by k_extend          */
    uint64_t rays_shadow;         /* shadow rays traced (k_shadow, or k_shade itself) */
    uint64_t rays_finish;         /* rays traced inside the tail finisher       */
    uint64_t iterations;          /* wavefront iterations                       */
    uint64_t scene_bytes;         /* BVH nodes + primitive records in HBM       */
    uint32_t bvh_nodes, bvh_depth;
    uint32_t stream_parts;        /* pool parts on their own streams: each kernel
                                     runs stream_parts launches per iteration  */
    uint32_t path_pool;           /* paths in flight (the pool size used)     */
    double ms_total;              /* render wall time (host timer)              */
    /* with desc.timing: summed HIP-event time of each kernel, on the launch stream */
    double ms_extend, ms_shadow, ms_shade, ms_splat, ms_finish;
    /* scan-mode scenes: 1 when the context holds the scan kernels specialised
       for this scene (hipRTC at nori_gpu_create; the path integrators' trace
       launches and the trace API run them, the one-bounce integrators scan
       generically), the time that compile (or cache read) took then, and 1
       when its code object came from the cache */
    uint32_t scan_rtc, scan_rtc_cached;
    double ms_scan_rtc;
    /* 1 when the shade kernel traced its own next-event shadow rays instead of
       queueing them for k_shadow (scan-mode scenes with the basic plugins by
       default; NORI_NEE_INLINE=0/1 at nori_gpu_create) */
    uint32_t nee_inline, reserved0;
} nori_gpu_stats;

typedef struct nori_gpu_hit {
    float t;                      /* +inf on miss                               */
    int32_t prim;                 /* global primitive id (shape order), -1 miss */
    float u, v;                   /* barycentrics (mesh)                        */
} nori_gpu_hit;

const char *nori_gpu_last_error(void);
int nori_gpu_abi_version(void);
int nori_gpu_device_count(int *count);
int nori_gpu_create(const nori_scene_desc *scene, int device, nori_gpu_ctx **out);
/* Render passes [pass_begin, pass_begin+pass_count) of the given blocks and
 * ADD the filtered samples into rgbw_out ((H+2b)x(W+2b)x4 floats, caller
 * owned, host or device memory).  Blocking. */
int nori_gpu_render(nori_gpu_ctx *ctx, const nori_gpu_render_desc *desc,
                    float *rgbw_out, nori_gpu_stats *stats);
/* Trace n rays (host arrays; ray = o.xyz, mint, d.xyz, maxt) with the
 * reference's BVH semantics: closest hit, or any hit when any_hit != 0. */
int nori_gpu_trace(nori_gpu_ctx *ctx, const float *rays, uint32_t n, int any_hit,
                   nori_gpu_hit *hits);
int nori_gpu_cancel(nori_gpu_ctx *ctx);
float nori_gpu_progress(const nori_gpu_ctx *ctx);
void nori_gpu_destroy(nori_gpu_ctx *ctx);

/* ---- multi-GPU: one process per GPU, film sum over RCCL -------------------
 * Samples are independent, so a frame shards without any data-path
 * collective; the only exchange is the final film sum.  librccl is opened at
 * run time from the directory of the process's HIP runtime (fallback:
 * librccl.so.1); without it these calls fail with NORI_ERR_UNSUPPORTED and
 * everything else works. */
typedef struct nori_gpu_comm nori_gpu_comm;
#define NORI_COMM_ID_BYTES 128
/* Rank 0 makes the communicator id (ncclGetUniqueId); the caller hands the
 * bytes to every rank over any channel (torch.distributed store, MPI, file). */
int nori_gpu_comm_id(unsigned char id[NORI_COMM_ID_BYTES]);
/* Collective over the nranks processes (ncclCommInitRank); device = this
 * process's GPU (the device of the contexts used with the communicator). */
int nori_gpu_comm_create(const unsigned char id[NORI_COMM_ID_BYTES], int nranks, int rank, int device,
                         nori_gpu_comm **out);
int nori_gpu_comm_rank(const nori_gpu_comm *comm, int *nranks, int *rank);
void nori_gpu_comm_destroy(nori_gpu_comm *comm);
/* Path of the librccl opened (loading it if needed), NULL if none loads. */
const char *nori_gpu_comm_library(void);

#define NORI_SHARD_PASSES 0  /* rank r: passes [P*r/N, P*(r+1)/N) of every block (default) */
#define NORI_SHARD_BLOCKS 1  /* rank r: blocks r, r+N, r+2N, ... of the BlockGenerator's spiral
                                order (block.cpp:140-188), every pass */
/* The share of a whole-frame render `desc` that rank `rank` of `nranks`
 * renders: writes this rank's pass range and block ids into *out and
 * block_buf (capacity = the frame's block count).  desc->num_blocks != 0
 * restricts the frame to those blocks first (ids checked against the frame,
 * duplicates dropped); desc->pass_count == 0 means the scene's sampleCount.
 * out->pass_count == 0: the rank has no share (more ranks than passes /
 * blocks).  Pure host function. */
int nori_gpu_shard_desc(const nori_scene_desc *scene, const nori_gpu_render_desc *desc, int mode, int nranks,
                        int rank, nori_gpu_render_desc *out, uint32_t *block_buf);
/* Render this rank's share of `desc` into film_dev (device memory on the
 * context's device, (H+2b)x(W+2b)x4 floats; ZEROED first) and sum the films
 * of all ranks on the context's stream: into root's film_dev (ncclReduce), or
 * into every rank's when root < 0 (ncclAllReduce).  Returns after the sum has
 * completed on this rank.  stats: this rank's share.  desc->variance_out must
 * be NULL (per-pixel statistics are not summed across ranks).
 * Failure handling: every rank joins a status exchange before the film sum.
 * If any rank's share was cancelled (nori_gpu_cancel) every rank returns
 * NORI_ERR_CANCELLED; if any failed (bad arguments, allocation, a HIP error
 * that leaves the device usable, any exception of the render), the failing
 * rank returns its error and the others NORI_ERR_INVALID ("the frame is
 * incomplete"); no film sum runs and the communicator stays usable.  A rank
 * whose device faulted (a sticky HIP error) cannot join: it aborts the
 * communicator (ncclCommAbort) and returns NORI_ERR_HIP.  Its peers, and any
 * rank whose peers do not reach a collective, give up after the watchdog
 * bound nori_gpu_comm_timeout(own status, own render seconds, own samples,
 * largest share's samples) -- max(30 s, 20 x the own render time scaled to
 * the largest share) after a rendered share, 600 s for a rank whose share
 * failed, was cancelled or is empty, NORI_COMM_TIMEOUT_S seconds if set --
 * abort and return NORI_ERR_HIP; an aborted communicator fails every later
 * call. */
int nori_gpu_render_sharded(nori_gpu_ctx *ctx, nori_gpu_comm *comm, const nori_gpu_render_desc *desc, int mode,
                            int root, float *film_dev, nori_gpu_stats *stats);
/* The status word a rank contributes to the exchange (reduced by max):
 * severity << 16 | rank, severity 0 for NORI_OK, 1 for NORI_ERR_CANCELLED,
 * 2 for any other status.  Pure function. */
int nori_gpu_comm_status_word(int status, int rank);
/* The watchdog bound of a sharded render's collectives, in seconds (see
 * nori_gpu_render_sharded); status = the rank's own share's outcome.  Pure
 * function (reads NORI_COMM_TIMEOUT_S). */
double nori_gpu_comm_timeout(int status, double own_seconds, double own_samples, double max_samples);

#ifdef __cplusplus
}
#endif
#endif /* NORI_GPU_H */
