// loader.hip -- the training image path: ImageReader (conerf/base/task_queue.py:89-152) +
// read_image (:13-27) + the trainer's copy of the float image to the device (gaussian_trainer.py:346-358).
//
// The reference decodes each image in a Python thread into a float32 HWC CPU tensor and later copies that tensor
// (12 B/pixel) to the GPU on the compute stream.  Here:
//   * C++ reader threads fill pinned host slots with the image's raw u8 HWC bytes (a decoded .npy cache: no decode
//     on the hot path);
//   * dg_ring_upload copies the u8 bytes (3-4 B/pixel) with hipMemcpyAsync on the caller's stream and a kernel
//     turns them into the float CHW image the loss reads (x / 255, RGBA composited over black exactly as
//     read_image does), so PCIe carries a quarter of the bytes and nothing waits on the host;
//   * a slot returns to the pool when the event recorded after its copy has completed.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "loader.h"

namespace gs {

namespace {

// read_image: (image / 255.0).clamp(0, 1) (float32), RGBA: rgb * a + [0,0,0] * (1 - a) in float64 (numpy with the
// int64 background), then .float(); the trainer's permute(2, 0, 1) makes it CHW.
__global__ void __launch_bounds__(256) k_u8_to_chw(const uint8_t* __restrict__ in, int H, int W, int Cin,
                                                   int composite, float* __restrict__ out) {
    const size_t npix = (size_t)H * W;
    const size_t p = (size_t)blockIdx.x * 256u + threadIdx.x;
    if (p >= npix) return;
    const uint8_t* px = in + p * Cin;
    if (Cin == 4 && composite) {
        const float a = fminf(fmaxf((float)px[3] / 255.0f, 0.0f), 1.0f);
        for (int c = 0; c < 3; c++) {
            const float v = fminf(fmaxf((float)px[c] / 255.0f, 0.0f), 1.0f);
            out[c * npix + p] = (float)((double)v * (double)a + 0.0 * (1.0 - (double)a));
        }
    } else {
        for (int c = 0; c < Cin; c++) out[c * npix + p] = fminf(fmaxf((float)px[c] / 255.0f, 0.0f), 1.0f);
    }
}

}  // namespace

void launch_u8_to_chw(const uint8_t* in, int H, int W, int C, int composite, float* out, hipStream_t s) {
    const size_t npix = (size_t)H * W;
    if (npix) k_u8_to_chw<<<(unsigned)((npix + 255) / 256), 256, 0, s>>>(in, H, W, C, composite, out);
}

struct ImageRing {
    struct Job { std::string path; uint64_t offset; int index, h, w, c; };
    struct Done { int index, h, w, c, slot; bool ok; };
    std::vector<uint8_t*> slot_mem;
    std::vector<hipEvent_t> slot_ev;  // recorded after the slot's upload; the slot is free once it completed
    std::vector<int> slot_state;      // 0 free, 1 reading / ready, 2 uploading
    uint64_t slot_bytes = 0;
    std::deque<Job> jobs;
    std::deque<Done> done;
    std::mutex mu;
    std::condition_variable cv_jobs, cv_done, cv_slots;
    std::vector<std::thread> workers;
    bool stop = false;
    std::string err;

    int acquire_slot(std::unique_lock<std::mutex>& lk) {  // called with mu held
        for (;;) {
            for (size_t i = 0; i < slot_state.size(); i++) {
                if (slot_state[i] == 2 && hipEventQuery(slot_ev[i]) == hipSuccess) slot_state[i] = 0;
                if (slot_state[i] == 0) { slot_state[i] = 1; return (int)i; }
            }
            if (stop) return -1;
            cv_slots.wait_for(lk, std::chrono::microseconds(200));
        }
    }

    void worker() {
        for (;;) {
            Job j;
            int slot;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv_jobs.wait(lk, [&] { return stop || !jobs.empty(); });
                if (stop) return;
                j = jobs.front();
                jobs.pop_front();
                slot = acquire_slot(lk);
                if (slot < 0) return;
            }
            const uint64_t n = (uint64_t)j.h * j.w * j.c;
            bool ok = n <= slot_bytes;
            if (ok) {
                FILE* f = fopen(j.path.c_str(), "rb");
                ok = f && fseeko(f, (off_t)j.offset, SEEK_SET) == 0 && fread(slot_mem[slot], 1, n, f) == n;
                if (f) fclose(f);
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                done.push_back({j.index, j.h, j.w, j.c, slot, ok});
                if (!ok) err = "could not read " + j.path;
            }
            cv_done.notify_one();
        }
    }
};

}  // namespace gs

extern "C" {

dg_image_ring* dg_ring_create(int slots, uint64_t max_bytes, int threads) {
    if (slots <= 0 || threads <= 0 || max_bytes == 0) return nullptr;
    auto* r = new gs::ImageRing();
    r->slot_bytes = max_bytes;
    for (int i = 0; i < slots; i++) {
        uint8_t* p = nullptr;
        hipEvent_t e = nullptr;
        if (hipHostMalloc((void**)&p, max_bytes, hipHostMallocDefault) != hipSuccess ||
            hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            dg_ring_destroy(reinterpret_cast<dg_image_ring*>(r));
            return nullptr;
        }
        r->slot_mem.push_back(p);
        r->slot_ev.push_back(e);
        r->slot_state.push_back(0);
    }
    for (int t = 0; t < threads; t++) r->workers.emplace_back([r] { r->worker(); });
    return reinterpret_cast<dg_image_ring*>(r);
}

int dg_ring_submit(dg_image_ring* ring, const char* path, uint64_t offset, int index, int h, int w, int c) {
    auto* r = reinterpret_cast<gs::ImageRing*>(ring);
    if (!r || !path || h <= 0 || w <= 0 || (c != 1 && c != 3 && c != 4)) return 1;
    if ((uint64_t)h * w * c > r->slot_bytes) return 2;
    {
        std::lock_guard<std::mutex> lk(r->mu);
        r->jobs.push_back({path, offset, index, h, w, c});
    }
    r->cv_jobs.notify_one();
    return 0;
}

int dg_ring_next(dg_image_ring* ring, int* index, int* h, int* w, int* c, int* slot) {
    auto* r = reinterpret_cast<gs::ImageRing*>(ring);
    if (!r) return 1;
    std::unique_lock<std::mutex> lk(r->mu);
    r->cv_done.wait(lk, [&] { return !r->done.empty(); });
    const auto d = r->done.front();
    r->done.pop_front();
    *index = d.index; *h = d.h; *w = d.w; *c = d.c; *slot = d.slot;
    if (!d.ok) {
        r->slot_state[d.slot] = 0;
        r->cv_slots.notify_all();
        return 3;
    }
    return 0;
}

int dg_ring_upload(dg_image_ring* ring, int slot, int h, int w, int c, int rgba_composite, uint8_t* dev_staging,
                   float* out_chw, dg_stream_t stream) {
    auto* r = reinterpret_cast<gs::ImageRing*>(ring);
    if (!r || slot < 0 || slot >= (int)r->slot_mem.size() || !dev_staging || !out_chw) return 1;
    if (h <= 0 || w <= 0 || (uint64_t)h * w * c > r->slot_bytes) return 2;
    hipStream_t s = (hipStream_t)stream;
    const size_t n = (size_t)h * w * c;
    if (hipMemcpyAsync(dev_staging, r->slot_mem[slot], n, hipMemcpyHostToDevice, s) != hipSuccess) return 4;
    gs::launch_u8_to_chw(dev_staging, h, w, c, rgba_composite, out_chw, s);
    if (hipEventRecord(r->slot_ev[slot], s) != hipSuccess) return 4;
    {
        std::lock_guard<std::mutex> lk(r->mu);
        r->slot_state[slot] = 2;  // free once the copy has completed
    }
    r->cv_slots.notify_all();
    return hipGetLastError() == hipSuccess ? 0 : 4;
}

int dg_ring_pending(dg_image_ring* ring) {
    auto* r = reinterpret_cast<gs::ImageRing*>(ring);
    if (!r) return 0;
    std::lock_guard<std::mutex> lk(r->mu);
    return (int)(r->jobs.size() + r->done.size());
}

void dg_ring_destroy(dg_image_ring* ring) {
    auto* r = reinterpret_cast<gs::ImageRing*>(ring);
    if (!r) return;
    {
        std::lock_guard<std::mutex> lk(r->mu);
        r->stop = true;
    }
    r->cv_jobs.notify_all();
    r->cv_slots.notify_all();
    for (auto& t : r->workers) t.join();
    for (size_t i = 0; i < r->slot_mem.size(); i++) {
        if (r->slot_ev[i]) {
            (void)hipEventSynchronize(r->slot_ev[i]);
            (void)hipEventDestroy(r->slot_ev[i]);
        }
        (void)hipHostFree(r->slot_mem[i]);
    }
    delete r;
}

int dg_image_u8_to_chw(const uint8_t* dev_hwc, int h, int w, int c, int rgba_composite, float* out_chw,
                       dg_stream_t stream) {
    if (h < 0 || w < 0 || (c != 1 && c != 3 && c != 4)) return 1;
    gs::launch_u8_to_chw(dev_hwc, h, w, c, rgba_composite, out_chw, (hipStream_t)stream);
    return hipGetLastError() == hipSuccess ? 0 : 4;
}

}  // extern "C"
