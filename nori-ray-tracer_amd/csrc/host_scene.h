// host_scene.h -- host-side types of libnori_gpu: the loaded scene, errors,
// and the BVH in its device layout.
#pragma once
#include <stdint.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/nori_gpu.h"

namespace nori {

// NoriException (common.h:150-155) carrying the C-ABI status code.
struct NoriException : std::runtime_error {
    int code;
    NoriException(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

struct Vec3f {
    float x, y, z;
};
struct Mat4 {
    float m[16];  // row-major
};
Mat4 mat_identity();
Mat4 mat_mul(const Mat4 &a, const Mat4 &b);
bool mat_inverse(const Mat4 &a, Mat4 &out);
void compute_sample_to_camera(nori_camera_desc &d);
std::string resolve_path(const std::string &p);

// Owner of a flattened scene; `desc` points into the vectors.
struct HostScene {
    std::string source;
    std::vector<float> positions, normals, uvs;
    std::vector<uint32_t> indices;
    std::vector<nori_shape_desc> shapes;
    std::vector<nori_bsdf_desc> bsdfs;
    std::vector<nori_emitter_desc> emitters;
    std::vector<std::vector<float>> env_images;  // envmap texels, owned here (emitters[i].env_rgb)
    std::vector<std::vector<uint8_t>> image_rgb;   // ImageTexture / NormalMap texels (images[i].rgb)
    std::vector<nori_image_desc> images;
    nori_scene_desc desc{};
    float root_min[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
    float root_max[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    void expand_root(float x, float y, float z) {
        float p[3] = {x, y, z};
        for (int i = 0; i < 3; ++i) {
            root_min[i] = p[i] < root_min[i] ? p[i] : root_min[i];
            root_max[i] = p[i] > root_max[i] ? p[i] : root_max[i];
        }
    }
    void finalize();
};
HostScene *load_scene_xml(const std::string &path, int width, int height, int spp);
// stbi_load(path, .., STBI_rgb) of the reference's stb_image v1.39: baseline
// JPEG or 8-bit PNG -> width x height x 3 bytes (image_decode.cpp); throws.
void decode_image_rgb8(const std::string &path, int &width, int &height, std::vector<uint8_t> &rgb);
// R, G, B planes of an OpenEXR file, rows = image height (image_io.cpp); throws NoriException.
int load_exr(const std::string &path, int &width, int &height, std::vector<float> &rgb);

// ---- BVH in device layout -------------------------------------------------
// The reference's binary tree is collapsed into a 4-wide tree (each node takes
// the inner children of largest surface area apart until it holds 4).  Inner
// node = 8 x float4 (128 B), children in SoA form:
//   [0] min.x of children 0..3  [1] min.y  [2] min.z
//   [3] max.x                   [4] max.y  [5] max.z
//   [6] child refs (uint bits)  [7] unused
// Unused child slots have NaN boxes (every slab test fails).  A child ref with
// bit 31 clear is an inner-node index; with bit 31 set it is a leaf: bits 0-24
// first primitive record, bits 25-30 count-1 (<= 64 prims).
// Primitive record = 3 x float4 (48 B), in leaf order:
//   triangle: (v0.xyz, prim id), (e1.xyz, 0), (e2.xyz, 0)   e1=p1-p0, e2=p2-p0
//   sphere  : (center.xyz, prim id), (radius, 0, 0, 1), (0, 0, 0, 0)
constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kLeafMaxPrims = 64;
struct DeviceBvh {
    std::vector<float> nodes;   // 32 floats per 4-wide node
    std::vector<float> prims;   // 12 floats per primitive
    uint32_t num_nodes = 0;
    uint32_t depth = 0;          // max inner-node depth of the 4-wide tree (stack bound: 3 per level)
    uint32_t ref_nodes = 0;      // nodes of the reference-layout tree
    float sah_cost = 0;
};
// Binned-SAH build with the reference's algorithm (bvh.cpp:100-382).
void build_device_bvh(const nori_scene_desc &d, const float root_min[3], const float root_max[3], DeviceBvh &out);

// Photon map (photon_map.cpp): raw = n photons x 12 floats (position, 0,
// direction towards the light, 0, power, 0) in emission order -> photons as
// (x, y, z, theta | phi << 8) and RGBE words (the reference's PhotonData),
// sorted by hash-grid bucket of cell size `radius`; tables = PhotonData's
// 5 x 256 decode tables; start = bucket offsets (mask + 2 entries).
void build_photon_map(const std::vector<float> &raw, uint32_t n, float radius, std::vector<float> &photons,
                      std::vector<uint32_t> &rgbe, std::vector<float> &tables, std::vector<uint32_t> &start,
                      uint32_t &mask);

}  // namespace nori
