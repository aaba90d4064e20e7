/*
 * nori_oracle.h -- CPU restatement of Nori's render path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so; the product path
 * (libnori_gpu.so) never links or calls it.
 *
 * Parity status: the reference itself cannot be built here (SURVEY.md 8c:
 * compiling it was refused by the environment; the refusal binds every round),
 * so this restatement is pinned by the reference's own fixtures: the pcg32
 * known-answer vector (ext/pcg32/pcg32-demo.out:7-8), the furnace and
 * polygonal-light t-tests (scenes/pa4/tests/test-furnace.xml, test-direct.xml), the microfacet BSDF
 * t-test (scenes/pa3/tests/ttest-microfacet.xml) and image-level checks.
 */
#ifndef NORI_ORACLE_H
#define NORI_ORACLE_H

#include <stdint.h>
#include "../include/nori_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_scene oracle_scene;

typedef struct oracle_stats {
    uint64_t samples;
    uint64_t invalid_samples;
    uint64_t rays_closest;
    uint64_t rays_shadow;
    uint64_t bounces;            /* BSDF-sampled continuations */
    double ms_render;            /* "Rendering .. done (took ...)" scope */
    int threads;
} oracle_stats;

/* Build BVH (bvh.cpp:100-382 semantics), mesh area pdfs (mesh.cpp:30-38). */
int oracle_scene_create(const nori_scene_desc *desc, oracle_scene **out);
void oracle_scene_free(oracle_scene *s);
uint32_t oracle_scene_node_count(const oracle_scene *s);
/* reachable node count and BVH::statistics cost of the tree, FNV-1a hash of the leaf-order primitive ids */
int oracle_scene_bvh_stats(const oracle_scene *s, uint32_t *nodes, float *sah, uint64_t *order_hash);

/* render.cpp:173-250 pass loop.  Adds into rgbw ((H+2b)x(W+2b)x4).
 * rng_mode: NORI_RNG_WAVE or NORI_RNG_BLOCK.  nthreads<=0: all hw threads.
 * variance_pass: also run the reference's serial per-pass variance sweep. */
int oracle_render(const oracle_scene *s, int rng_mode, uint64_t seed,
                  uint32_t pass_begin, uint32_t pass_count,
                  const uint32_t *block_ids, uint32_t num_blocks,
                  int nthreads, int variance_pass, float *rgbw, oracle_stats *stats);

/* Scene::rayIntersect over a batch of rays (o.xyz, mint, d.xyz, maxt). */
int oracle_trace(const oracle_scene *s, const float *rays, uint32_t n, int any_hit,
                 nori_gpu_hit *hits);

/* Per-sample radiance for the given sample ids in WAVE mode: out = n x 5
 * (pixel-sample x, y, L r, g, b).  Used for sample-level parity. */
int oracle_wave_samples(const oracle_scene *s, uint64_t seed, const uint64_t *sample_ids,
                        uint32_t n, float *out);

/* photonmapper scenes: photons emitted to fill the map and the map itself
 * (n x 9 floats: position, direction, power as PhotonData returns them). */
int oracle_photon_map(const oracle_scene *s, uint64_t *emitted, uint32_t *count, const float **photons);

/* pcg32 (ext/pcg32/pcg32.h:51-110). state2 = {state, inc}. */
void oracle_pcg32_seed(uint64_t *state2, uint64_t initstate, uint64_t initseq);
uint32_t oracle_pcg32_next(uint64_t *state2);
float oracle_pcg32_next_float(uint64_t *state2);

/* StudentsTTest (ttest.cpp:147-194): n camera paths from an unseeded
 * independent sampler, luminance mean / unbiased variance. */
int oracle_scene_ttest(const oracle_scene *s, uint32_t n, double *mean, double *var);
/* StudentsTTest BSDF mode (ttest.cpp:107-145). */
int oracle_bsdf_ttest(const nori_bsdf_desc *bsdf, float angle_deg, uint32_t n,
                      double *mean, double *var);
/* BSDF sample / eval / pdf on local directions; used by the chi^2 test.
 * sample: out = n x 5 (wo.xyz, weight luminance, measure). */
int oracle_bsdf_sample(const nori_bsdf_desc *bsdf, const float *wi, const float *u2,
                       uint32_t n, float *out);
int oracle_bsdf_eval_pdf(const nori_bsdf_desc *bsdf, const float *wi, const float *wo,
                         uint32_t n, float *out /* n x 4: f.rgb, pdf */);

#ifdef __cplusplus
}
#endif
#endif
