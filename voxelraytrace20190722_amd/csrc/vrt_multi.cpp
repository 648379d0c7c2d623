// vrt_multi.cpp -- the multi-device frame of include/vrt.h (SURVEY §8(b),
// §8(e)): the reference's render_mt (VRT/camera.h:42-68) spreads one frame's
// 8x8 tiles over the CPU's threads; here the tiles are dealt over the GPUs of
// one node.  The scene is built once and replicated per device; each rank
// renders its share of the tile deal into a packed buffer on its own stream,
// one RCCL ncclGather brings the shares to rank 0 over xGMI (rank 0's share
// is rendered in place into the receive buffer), and rank 0 re-assembles the
// image with the same unpack kernel as the torch.distributed path of
// bench.py.  The collective is the frame's only exchange.
//
// VRT/x = /root/reference/VoxelRayTrace20190722/x
#include "../../include/vrt.h"
#include "vrt_error.h"
#include "vrt_internal.h"

#include <rccl/rccl.h>

#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

using namespace vrt;

struct vrt_multi {
        std::vector<int> devs;          // rank i -> HIP device
        std::vector<vrt_scene *> sc;    // rank i's replica of the scene
        std::vector<ncclComm_t> comm;   // ncclCommInitAll over devs (empty: virtual ranks)
        bool virt = false;              // VRT_TEST_VIRTUAL_RANKS: n ranks on one device, copies for the gather
        std::vector<hipStream_t> st;    // rank i's render + collective stream
        std::vector<hipEvent_t> ev;     // rank i: its part of a frame queued
        std::vector<float *> send;      // ranks >= 1: packed tile buffer (tpr * 192 floats)
        float *gath = nullptr;          // rank 0: n * tpr * 192 floats (its own share in place)
        size_t tpr_cap = 0;             // tiles per rank the buffers hold
        float *d_img = nullptr;         // vrt_render_multi: image on rank 0's device
        float *h_pin = nullptr;         // and its pinned staging copy
        size_t img_bytes = 0;
        hipEvent_t ev_in = nullptr;     // caller's stream -> rank 0's stream
        std::mutex mu;
};

namespace {

#define HIPCHK(expr)                                                                              \
        do {                                                                                      \
                hipError_t e_ = (expr);                                                           \
                if (e_ != hipSuccess)                                                             \
                        return set_error(VRT_E_DEVICE, "%s failed: %s", #expr, hipGetErrorString(e_)); \
        } while (0)

#define NCCLCHK(expr)                                                                             \
        do {                                                                                      \
                ncclResult_t r_ = (expr);                                                         \
                if (r_ != ncclSuccess)                                                            \
                        return set_error(VRT_E_DEVICE, "%s failed: %s", #expr, ncclGetErrorString(r_)); \
        } while (0)

// the caller's current device is restored on every return
struct DeviceGuard {
        int dev = -1;
        DeviceGuard() { (void)hipGetDevice(&dev); }
        ~DeviceGuard()
        {
                if (dev >= 0)
                        (void)hipSetDevice(dev);
        }
};

std::vector<int> mask_devices(uint32_t mask)
{
        std::vector<int> d;
        for (int i = 0; i < 32; ++i)
                if (mask & (1u << i))
                        d.push_back(i);
        return d;
}

void free_buffers(vrt_multi *m)
{
        for (size_t i = 0; i < m->send.size(); ++i)
                if (m->send[i]) {
                        (void)hipSetDevice(m->devs[i]);
                        (void)hipFree(m->send[i]);
                        m->send[i] = nullptr;
                }
        if (m->gath) {
                (void)hipSetDevice(m->devs[0]);
                (void)hipFree(m->gath);
                m->gath = nullptr;
        }
        m->tpr_cap = 0;
}

int sync_all(vrt_multi *m)
{
        for (size_t i = 0; i < m->st.size(); ++i)
                if (m->st[i]) {
                        HIPCHK(hipSetDevice(m->devs[i]));
                        HIPCHK(hipStreamSynchronize(m->st[i]));
                }
        return VRT_OK;
}

// The ranks' packed buffers into rank 0's receive buffer m->gath (rank-major,
// `count` floats each), after each rank's render on its stream; rank 0's
// stream then holds the complete buffer.
int gather(vrt_multi *m, size_t count)
{
        const int n = (int)m->devs.size();
        if (m->virt) {
                // VRT_TEST_VIRTUAL_RANKS: rank i's buffer into its slot on rank
                // i's stream (after its render, where the collective's send
                // runs), and -- as the collective waits for the root -- only
                // once rank 0's stream has reached this frame's gather (so the
                // previous frame's unpack has read the slot); rank 0's stream
                // then waits for every copy
                HIPCHK(hipSetDevice(m->devs[0]));
                HIPCHK(hipEventRecord(m->ev[0], m->st[0]));
                for (int i = 1; i < n; ++i)
                        HIPCHK(hipStreamWaitEvent(m->st[i], m->ev[0], 0));
                for (int i = 1; i < n; ++i) {
                        HIPCHK(hipMemcpyAsync(m->gath + (size_t)i * count, m->send[i], count * sizeof(float),
                                              hipMemcpyDeviceToDevice, m->st[i]));
                        HIPCHK(hipEventRecord(m->ev[i], m->st[i]));
                        HIPCHK(hipStreamWaitEvent(m->st[0], m->ev[i], 0));
                }
                return VRT_OK;
        }
        // one RCCL gather to rank 0 (in place for rank 0: sendbuff == recvbuff + 0)
        NCCLCHK(ncclGroupStart());
        for (int i = 0; i < n; ++i) {
                const ncclResult_t r = ncclGather(i == 0 ? m->gath : m->send[i], i == 0 ? m->gath : nullptr, count,
                                                  ncclFloat32, 0, m->comm[i], m->st[i]);
                if (r != ncclSuccess) {
                        (void)ncclGroupEnd();
                        return set_error(VRT_E_DEVICE, "ncclGather (rank %d): %s", i, ncclGetErrorString(r));
                }
        }
        NCCLCHK(ncclGroupEnd());
        return VRT_OK;
}

// One frame into d_image on rank 0's device (caller holds m->mu).
int render_multi(vrt_multi *m, const vrt_camera *cam, const vrt_film *film, float *d_image, hipStream_t caller)
{
        const int n = (int)m->devs.size();
        const int tpr = vrt_tiles_per_rank(film, n);
        const size_t count = (size_t)tpr * 192;  // floats per rank buffer (8x8 pixels x RGB per tile)
        if (tpr > 0 && (size_t)tpr > m->tpr_cap) {
                if (int rc = sync_all(m))
                        return rc;
                free_buffers(m);
                for (int i = 1; i < n; ++i) {
                        HIPCHK(hipSetDevice(m->devs[i]));
                        HIPCHK(hipMalloc(&m->send[i], count * sizeof(float)));
                }
                HIPCHK(hipSetDevice(m->devs[0]));
                HIPCHK(hipMalloc(&m->gath, (size_t)n * count * sizeof(float)));
                m->tpr_cap = (size_t)tpr;
        }
        HIPCHK(hipSetDevice(m->devs[0]));
        if (caller) {  // rank 0's stream follows the caller's
                HIPCHK(hipEventRecord(m->ev_in, caller));
                HIPCHK(hipStreamWaitEvent(m->st[0], m->ev_in, 0));
        }
        if (tpr > 0) {
                // each rank's share, packed tile-major (vrt_render_tiles_device)
                for (int i = 0; i < n; ++i) {
                        float *dst = i == 0 ? m->gath : m->send[i];
                        if (int rc = vrt_render_tiles_device(m->sc[i], cam, film, i, n, 0, dst, m->st[i]))
                                return rc;
                }
                if (int rc = gather(m, count))
                        return rc;
        }
        HIPCHK(hipSetDevice(m->devs[0]));
        if (tpr > 0) {
                if (int rc = vrt_unpack_tiles_device(film, n, m->gath, d_image, m->st[0]))
                        return rc;
        } else {
                HIPCHK(hipMemsetAsync(d_image, 0, (size_t)film->nx * film->ny * 12, m->st[0]));
        }
        if (caller) {
                HIPCHK(hipEventRecord(m->ev[0], m->st[0]));
                HIPCHK(hipStreamWaitEvent(caller, m->ev[0], 0));
        }
        return VRT_OK;
}

}  // namespace

extern "C" void vrt_multi_destroy(vrt_multi *m)
{
        if (!m)
                return;
        DeviceGuard g;
        (void)sync_all(m);
        for (ncclComm_t c : m->comm)
                if (c)
                        (void)ncclCommDestroy(c);
        free_buffers(m);
        if (m->d_img || m->h_pin || m->ev_in) {
                (void)hipSetDevice(m->devs[0]);
                if (m->d_img)
                        (void)hipFree(m->d_img);
                if (m->h_pin)
                        (void)hipHostFree(m->h_pin);
                if (m->ev_in)
                        (void)hipEventDestroy(m->ev_in);
        }
        for (size_t i = 0; i < m->st.size(); ++i) {
                (void)hipSetDevice(m->devs[i]);
                if (m->ev[i])
                        (void)hipEventDestroy(m->ev[i]);
                if (m->st[i])
                        (void)hipStreamDestroy(m->st[i]);
        }
        for (vrt_scene *s : m->sc)
                vrt_scene_destroy(s);
        delete m;
}

extern "C" int vrt_scene_create_multi(const vrt_scene_desc *desc, int max_depth, uint32_t device_mask, int flags,
                                      vrt_multi **out)
{
        if (!out)
                return set_error(VRT_E_INVALID, "null out");
        *out = nullptr;
        std::vector<int> devs = mask_devices(device_mask);
        if (devs.empty())
                return set_error(VRT_E_INVALID, "empty device mask");
        const int tf = test_flags();
        const bool virt = (tf & VRT_TEST_VIRTUAL_RANKS) != 0;
        if (virt) {
                const int nv = (tf >> 8) & 0xff;
                if (devs.size() != 1 || nv < 2 || nv > 16)
                        return set_error(VRT_E_INVALID, "virtual ranks need a one-device mask and 2..16 ranks (got %d)", nv);
                devs.assign(nv, devs[0]);
        }
        int nvis = 0;
        if (hipGetDeviceCount(&nvis) != hipSuccess || devs.back() >= nvis)
                return set_error(VRT_E_NODEVICE, "device mask %#x names device %d, %d visible", device_mask,
                                 devs.back(), nvis);
        DeviceGuard g;
        std::unique_ptr<vrt_multi, void (*)(vrt_multi *)> m(new (std::nothrow) vrt_multi, vrt_multi_destroy);
        if (!m)
                return set_error(VRT_E_NOMEM, "vrt_multi alloc");
        const int n = (int)devs.size();
        m->devs = devs;
        m->sc.assign(n, nullptr);
        m->st.assign(n, nullptr);
        m->ev.assign(n, nullptr);
        m->send.assign(n, nullptr);
        // build once (host, or rank 0's device with VRT_BUILD_DEVICE) ...
        if (int rc = vrt_scene_create_ex(desc, max_depth, devs[0], flags, &m->sc[0]))
                return rc;
        // ... and upload the same build to every other device, in parallel
        std::vector<int> rcs(n, VRT_OK);
        std::vector<std::string> errs(n);
        {
                std::vector<std::thread> th;
                for (int i = 1; i < n; ++i)
                        th.emplace_back([&, i] {
                                rcs[i] = scene_replicate(m->sc[0], desc, devs[i], &m->sc[i]);
                                if (rcs[i])
                                        errs[i] = vrt_last_error();
                        });
                for (auto &t : th)
                        t.join();
        }
        for (int i = 1; i < n; ++i)
                if (rcs[i])
                        return set_error(rcs[i], "replica on device %d: %s", devs[i], errs[i].c_str());
        for (int i = 0; i < n; ++i) {
                HIPCHK(hipSetDevice(devs[i]));
                HIPCHK(hipStreamCreateWithFlags(&m->st[i], hipStreamNonBlocking));
                HIPCHK(hipEventCreateWithFlags(&m->ev[i], hipEventDisableTiming));
        }
        HIPCHK(hipSetDevice(devs[0]));
        HIPCHK(hipEventCreateWithFlags(&m->ev_in, hipEventDisableTiming));
        m->virt = virt;
        if (!virt) {
                m->comm.assign(n, nullptr);
                NCCLCHK(ncclCommInitAll(m->comm.data(), n, m->devs.data()));
        }
        *out = m.release();
        return VRT_OK;
}

extern "C" int vrt_multi_devices(const vrt_multi *m, int *n, int32_t *devices)
{
        if (!m || !n)
                return set_error(VRT_E_INVALID, "null argument");
        *n = (int)m->devs.size();
        if (devices)
                for (size_t i = 0; i < m->devs.size(); ++i)
                        devices[i] = m->devs[i];
        return VRT_OK;
}

extern "C" int vrt_multi_scene(vrt_multi *m, int rank, vrt_scene **out)
{
        if (!m || !out || rank < 0 || rank >= (int)m->sc.size())
                return set_error(VRT_E_INVALID, "bad argument");
        *out = m->sc[rank];
        return VRT_OK;
}

extern "C" int vrt_render_multi_device(vrt_multi *m, const vrt_camera *cam, const vrt_film *film, float *d_image,
                                       void *stream)
{
        if (!m || !cam || !film || !d_image)
                return set_error(VRT_E_INVALID, "null argument");
        if (film->nx < 1 || film->ny < 1 || film->nx > 32768 || film->ny > 32768)
                return set_error(VRT_E_INVALID, "bad film");
        std::lock_guard<std::mutex> lk(m->mu);
        DeviceGuard g;
        if (int rc = render_multi(m, cam, film, d_image, static_cast<hipStream_t>(stream)))
                return rc;
        if (!stream)  // no caller stream: the image is complete on return
                return sync_all(m);
        return VRT_OK;
}

extern "C" int vrt_render_multi(vrt_multi *m, const vrt_camera *cam, const vrt_film *film, float *rgb)
{
        if (!m || !cam || !film || !rgb)
                return set_error(VRT_E_INVALID, "null argument");
        if (film->nx < 1 || film->ny < 1 || film->nx > 32768 || film->ny > 32768)
                return set_error(VRT_E_INVALID, "bad film");
        std::lock_guard<std::mutex> lk(m->mu);
        DeviceGuard g;
        const size_t bytes = (size_t)film->nx * film->ny * 12;
        HIPCHK(hipSetDevice(m->devs[0]));
        if (bytes > m->img_bytes) {
                HIPCHK(hipStreamSynchronize(m->st[0]));
                if (m->d_img)
                        (void)hipFree(m->d_img);
                if (m->h_pin)
                        (void)hipHostFree(m->h_pin);
                m->d_img = nullptr;
                m->h_pin = nullptr;
                m->img_bytes = 0;
                HIPCHK(hipMalloc(&m->d_img, bytes));
                HIPCHK(hipHostMalloc(&m->h_pin, bytes, hipHostMallocDefault));
                m->img_bytes = bytes;
        }
        // the unpack writes every pixel (zero outside the tile grid)
        if (int rc = render_multi(m, cam, film, m->d_img, nullptr))
                return rc;
        HIPCHK(hipSetDevice(m->devs[0]));
        HIPCHK(hipMemcpyAsync(m->h_pin, m->d_img, bytes, hipMemcpyDeviceToHost, m->st[0]));
        if (int rc = sync_all(m))
                return rc;
        par_memcpy(rgb, m->h_pin, bytes);
        return VRT_OK;
}

extern "C" int vrt_multi_tile_map(const vrt_film *film, uint32_t device_mask, int32_t *device_of_tile,
                                  int32_t *slot_of_tile)
{
        const std::vector<int> devs = mask_devices(device_mask);
        if (devs.empty() || !device_of_tile || !slot_of_tile)
                return set_error(VRT_E_INVALID, "bad argument");
        if (int rc = vrt_tile_deal_map(film, (int)devs.size(), device_of_tile, slot_of_tile))
                return rc;
        const int64_t nt = (int64_t)(film->nx / 8) * (film->ny / 8);
        for (int64_t t = 0; t < nt; ++t)
                device_of_tile[t] = devs[device_of_tile[t]];
        return VRT_OK;
}
