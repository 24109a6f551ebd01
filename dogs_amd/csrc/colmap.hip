// colmap.hip -- host-side readers of COLMAP's binary model (cameras.bin, images.bin, points3D.bin), the input of the
// block split (load_colmap.py:180-260 -> conerf/pycolmap/pycolmap/scene_manager.py:137-310).
//
// The reference parses every record with Python struct.unpack (one call per point, plus one per track, plus one
// byte-at-a-time read per image name): minutes for a city-scale points3D.bin.  Here each file is mapped once and
// walked twice in C++ -- a count pass that sizes the caller's arrays, and a fill pass -- with the reference's
// record layouts and filters:
//   cameras.bin   u64 n; per camera: u32 id, i32 model, u64 width, u64 height, f64 params[num_params(model)]
//   images.bin    u64 n; per image: u32 id, f64 qvec[4], f64 tvec[3], u32 camera_id, name\0, u64 n2d,
//                 n2d x (f64 x, f64 y, i64 point3D_id); points with point3D_id == -1 are dropped (:204-207)
//   points3D.bin  u64 n; per point: u64 id, f64 xyz[3], u8 rgb[3], f64 error, u64 track_len,
//                 track_len x (u32 image_id, u32 point2D_idx); points with track_len < min_track_length are
//                 skipped (:288-291)
// Host code only: it runs on the CPU and touches no device.
#include <fcntl.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../../include/dogs_hip.h"

namespace {

struct Mapped {
    const uint8_t* p = nullptr;
    size_t n = 0;
    int fd = -1;
    explicit Mapped(const char* path) {
        fd = open(path, O_RDONLY);
        if (fd < 0) return;
        struct stat st;
        if (fstat(fd, &st) != 0 || st.st_size <= 0) return;
        n = (size_t)st.st_size;
        void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) { n = 0; return; }
        p = (const uint8_t*)m;
    }
    ~Mapped() {
        if (p) munmap((void*)p, n);
        if (fd >= 0) close(fd);
    }
};

// bounds-checked little-endian reads (x86 and gfx hosts are little-endian)
struct Cursor {
    const uint8_t* p;
    size_t n, off = 0;
    bool bad = false;
    template <typename T>
    T get() {
        T v{};
        if (off + sizeof(T) > n) { bad = true; return v; }
        memcpy(&v, p + off, sizeof(T));
        off += sizeof(T);
        return v;
    }
    bool skip(size_t b) {
        if (off + b > n) { bad = true; return false; }
        off += b;
        return true;
    }
};

int num_params(int model) {  // Camera.GetNumParams (pycolmap/camera.py)
    switch (model) {
        case 0: return 3;   // SIMPLE_PINHOLE
        case 1: return 4;   // PINHOLE
        case 2: return 4;   // SIMPLE_RADIAL
        case 3: return 5;   // RADIAL
        case 4: return 8;   // OPENCV
        default: return -1;
    }
}

}  // namespace

extern "C" {

int dg_colmap_cameras(const char* path, uint64_t* n_out, uint32_t* ids, int32_t* models, uint64_t* wh,
                      double* params8) {
    Mapped m(path);
    if (!m.p) return 1;
    Cursor c{m.p, m.n};
    const uint64_t n = c.get<uint64_t>();
    if (c.bad) return 2;
    if (!ids) { *n_out = n; }
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t id = c.get<uint32_t>();
        const int32_t model = c.get<int32_t>();
        const uint64_t w = c.get<uint64_t>(), h = c.get<uint64_t>();
        const int np = num_params(model);
        if (c.bad || np < 0) return 3;
        if (ids) {
            ids[i] = id; models[i] = model; wh[2 * i] = w; wh[2 * i + 1] = h;
            for (int k = 0; k < 8; k++) params8[8 * i + k] = 0.0;
            for (int k = 0; k < np; k++) params8[8 * i + k] = c.get<double>();
        } else {
            c.skip(8 * (size_t)np);
        }
        if (c.bad) return 2;
    }
    *n_out = n;
    return 0;
}

int dg_colmap_images(const char* path, uint64_t* n_out, uint64_t* name_bytes, uint64_t* n_points2d, uint32_t* ids,
                     double* qt7, uint32_t* camera_ids, uint64_t* name_offsets, char* names, uint64_t* p2d_offsets,
                     double* xy, int64_t* point3d_ids) {
    Mapped m(path);
    if (!m.p) return 1;
    Cursor c{m.p, m.n};
    const uint64_t n = c.get<uint64_t>();
    if (c.bad) return 2;
    const bool fill = ids != nullptr;
    uint64_t nb = 0, np2 = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t id = c.get<uint32_t>();
        double qt[7];
        for (int k = 0; k < 7; k++) qt[k] = c.get<double>();
        const uint32_t cam = c.get<uint32_t>();
        if (c.bad) return 2;
        const uint8_t* s = m.p + c.off;
        const uint8_t* z = (const uint8_t*)memchr(s, 0, m.n - c.off);
        if (!z) return 2;
        const size_t len = (size_t)(z - s);
        if (fill) {
            ids[i] = id; camera_ids[i] = cam;
            for (int k = 0; k < 7; k++) qt7[7 * i + k] = qt[k];
            name_offsets[i] = nb;
            memcpy(names + nb, s, len);
            p2d_offsets[i] = np2;
        }
        nb += len;
        c.skip(len + 1);
        const uint64_t k2 = c.get<uint64_t>();
        if (c.bad || c.off > m.n || k2 > (m.n - c.off) / 24) return 2;   // no wrap-around on a hostile count
        for (uint64_t j = 0; j < k2; j++) {
            double x, y;
            int64_t pid;
            memcpy(&x, m.p + c.off, 8); memcpy(&y, m.p + c.off + 8, 8); memcpy(&pid, m.p + c.off + 16, 8);
            c.off += 24;
            if (pid == -1) continue;  // no associated 3D point (scene_manager.py:204-207)
            if (fill) { xy[2 * np2] = x; xy[2 * np2 + 1] = y; point3d_ids[np2] = pid; }
            np2++;
        }
    }
    if (fill) { name_offsets[n] = nb; p2d_offsets[n] = np2; }
    *n_out = n; *name_bytes = nb; *n_points2d = np2;
    return 0;
}

int dg_colmap_points3d(const char* path, int min_track_length, uint64_t* n_out, uint64_t* n_track, uint64_t* ids,
                       double* xyz, uint8_t* rgb, double* err, uint64_t* track_offsets, uint32_t* tracks) {
    Mapped m(path);
    if (!m.p) return 1;
    Cursor c{m.p, m.n};
    const uint64_t n = c.get<uint64_t>();
    if (c.bad) return 2;
    const bool fill = ids != nullptr;
    uint64_t kept = 0, nt = 0;
    constexpr size_t REC = 8 + 24 + 3 + 8 + 8;  // '<Q 3d 3B d Q', packed
    for (uint64_t i = 0; i < n; i++) {
        if (c.off + REC > m.n) return 2;
        const uint8_t* r = m.p + c.off;
        uint64_t tl;
        memcpy(&tl, r + 43, 8);
        c.off += REC;
        if (c.off > m.n || tl > (m.n - c.off) / 8) return 2;
        if ((int64_t)tl >= (int64_t)min_track_length) {
            if (fill) {
                memcpy(ids + kept, r, 8);
                memcpy(xyz + 3 * kept, r + 8, 24);
                memcpy(rgb + 3 * kept, r + 32, 3);
                memcpy(err + kept, r + 35, 8);
                track_offsets[kept] = nt;
                memcpy(tracks + 2 * nt, m.p + c.off, 8 * tl);
            }
            kept++;
            nt += tl;
        }
        c.off += 8 * tl;
    }
    if (fill) track_offsets[kept] = nt;
    *n_out = kept; *n_track = nt;
    return 0;
}

}  // extern "C"
