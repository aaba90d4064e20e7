// nori_gpu_euler.cpp -- the reference's RenderThread (include/nori/render.h,
// src/render.cpp:63-276) and its `nori_euler` driver (src/main_euler.cpp)
// written against the C ABI of libnori_gpu only (include/nori_gpu.h): the
// binding INTEGRATION.md section 2 describes, compiled and run by the tests.
//
//   nori_gpu_euler scene.xml [--device D] [--spp N] [--size W H] [--png] [--out stem]
//
// renderScene() starts the render on its own std::thread (render.cpp:173),
// getProgress()/isRenderingDone() poll nori_gpu_progress and the thread's
// status, stopRendering() is nori_gpu_cancel (checked between wavefront
// iterations, as render.cpp:196 checks between passes).  The image is the
// full-frame ImageBlock (RGBW + filter border, block.h:48) the GPU adds into;
// it is developed (ImageBlock::toBitmap) and saved next to the scene as
// <stem>.exr (+ <stem>.png with --png), render.cpp:256-261.
#include <nori_gpu.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace {

struct GpuError : std::runtime_error {
    int code;
    GpuError(int c, const std::string &what) : std::runtime_error(what + ": " + nori_gpu_last_error()), code(c) {}
};
void check(int rc, const char *what) {
    if (rc != NORI_OK) throw GpuError(rc, what);
}

class RenderThread {
public:
    RenderThread(int device, int spp, int width, int height, bool png, std::string out)
        : device_(device), spp_(spp), width_(width), height_(height), png_(png), out_(std::move(out)) {}
    ~RenderThread() {
        stopRendering();
        if (thread_.joinable()) thread_.join();
        if (ctx_) nori_gpu_destroy(ctx_);
        if (scene_) nori_scene_free(scene_);
    }

    // render.cpp:158-250: load the scene, size the block, render on a thread
    void renderScene(const std::string &filename) {
        check(nori_scene_load_xml(filename.c_str(), width_, height_, spp_, &scene_), "loading the scene");
        desc_ = nori_scene_get_desc(scene_);
        const int b = nori_film_border(desc_);
        W_ = desc_->camera.width;
        H_ = desc_->camera.height;
        block_.assign(4 * (size_t)(W_ + 2 * b) * (H_ + 2 * b), 0.0f);  // ImageBlock::clear
        check(nori_gpu_create(desc_, device_, &ctx_), "creating the GPU context");
        stem_ = out_.empty() ? filename.substr(0, filename.rfind('.')) : out_;
        status_ = 1;
        thread_ = std::thread([this] {
            nori_gpu_render_desc rd;
            std::memset(&rd, 0, sizeof(rd));
            rd.pass_count = desc_->sample_count;  // sampler->getSampleCount() passes
            rc_ = nori_gpu_render(ctx_, &rd, block_.data(), &stats_);
            if (rc_ != NORI_OK) err_ = nori_gpu_last_error();  // (thread-local: read it here)
            if (rc_ == NORI_OK) {
                try {
                    save();
                } catch (const GpuError &e) {
                    rc_ = e.code;
                    err_ = e.what();
                }
            }
            status_ = rc_ == NORI_ERR_CANCELLED ? 2 : 3;
        });
    }
    bool isBusy() const { return status_ == 1; }
    void stopRendering() {
        if (ctx_ && status_ == 1) nori_gpu_cancel(ctx_);
    }
    float getProgress() const { return ctx_ ? nori_gpu_progress(ctx_) : 0.0f; }
    bool isRenderingDone() const { return status_ >= 2; }
    int result() const { return rc_; }
    const std::string &error() const { return err_; }
    const nori_gpu_stats &stats() const { return stats_; }

private:
    void save() {  // render.cpp:252-261: toBitmap, then Bitmap::save / saveToLDR
        std::vector<float> rgb(3 * (size_t)W_ * H_);
        check(nori_film_develop(desc_, block_.data(), rgb.data()), "developing the film");
        check(nori_write_exr((stem_ + ".exr").c_str(), rgb.data(), W_, H_), "writing the EXR");
        if (png_) check(nori_write_png((stem_ + ".png").c_str(), rgb.data(), W_, H_), "writing the PNG");
    }

    int device_, spp_, width_, height_;
    bool png_;
    std::string out_;
    nori_scene *scene_ = nullptr;
    const nori_scene_desc *desc_ = nullptr;
    nori_gpu_ctx *ctx_ = nullptr;
    std::vector<float> block_;
    std::string stem_;
    int W_ = 0, H_ = 0;
    std::thread thread_;
    std::atomic<int> status_{0};  // 0 free, 1 busy, 2 interrupted, 3 done (render.h:55)
    int rc_ = NORI_OK;
    std::string err_;
    nori_gpu_stats stats_{};
};

}  // namespace

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s scene.xml [--device D] [--spp N] [--size W H] [--png] [--out stem]\n", argv[0]);
        return 2;
    }
    int device = 0, spp = 0, width = 0, height = 0;
    bool png = false;
    std::string out;
    for (int i = 2; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--device" && i + 1 < argc) device = std::atoi(argv[++i]);
        else if (a == "--spp" && i + 1 < argc) spp = std::atoi(argv[++i]);
        else if (a == "--size" && i + 2 < argc) width = std::atoi(argv[++i]), height = std::atoi(argv[++i]);
        else if (a == "--png") png = true;
        else if (a == "--out" && i + 1 < argc) out = argv[++i];
        else {
            std::fprintf(stderr, "unknown argument %s\n", a.c_str());
            return 2;
        }
    }
    if (nori_gpu_abi_version() != NORI_GPU_ABI_VERSION) {
        std::fprintf(stderr, "libnori_gpu ABI %d, header %d\n", nori_gpu_abi_version(), NORI_GPU_ABI_VERSION);
        return 3;
    }
    try {
        RenderThread rt(device, spp, width, height, png, out);
        rt.renderScene(argv[1]);
        // main_euler.cpp: poll the progress until the render is done
        while (!rt.isRenderingDone()) {
            std::printf("Progress of the rendering : %.2f%%\n", 100.0 * rt.getProgress());
            std::fflush(stdout);
            std::this_thread::sleep_for(std::chrono::milliseconds(200));
        }
        if (rt.result() != NORI_OK) {
            std::fprintf(stderr, "render failed (%d): %s\n", rt.result(), rt.error().c_str());
            return 1;
        }
        const nori_gpu_stats &st = rt.stats();
        std::printf("Rendering done: %llu samples, %llu invalid, %.1f ms, %.1f Msamples/s\n",
                    (unsigned long long)st.samples, (unsigned long long)st.invalid_samples, st.ms_total,
                    st.samples / (st.ms_total * 1e3));
    } catch (const GpuError &e) {
        std::fprintf(stderr, "%s\n", e.what());
        return e.code == NORI_ERR_HIP ? 4 : 1;
    }
    return 0;
}
