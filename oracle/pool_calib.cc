// oracle/pool_calib.cc -- TEST INFRASTRUCTURE ONLY (CPU-baseline calibration).
//
// Drives the oracle's per-pixel primary render (vrt_oracle.c,
// ora_render_tile) with the reference's OWN scheduler: render_mt's 64 tile
// tasks (VRT/camera.h:42-68) posted to a tp::ThreadPool built from the
// reference's thread_pool_cpp headers, included unmodified from
// /root/reference by oracle/Makefile (-I$(REF)); a new pool per frame and one
// std::promise per task, as render_mt does.  Built into oracle/_ref/ (never
// shipped to the GPU box); tools/cpu_calibration.py times it against the
// oracle's own atomic-counter scheduler (ora_render_rows) on the same frames,
// which gives BASELINE.md's calibration ratio for bench.py's cpu_baseline.
//
// VRT/x = /root/reference/VoxelRayTrace20190722/x
#include <chrono>
#include <cstring>
#include <future>
#include <vector>

#include "thread_pool_cpp/thread_pool.hpp"  // VRT/thread_pool_cpp (unmodified)
#include "vrt_oracle.h"

extern "C" {

// One render_mt frame (VRT/camera.h:42-68): pt = n / 8 pixels per tile side,
// task (tx, ty) posted in tx-major order, each running its rows then columns;
// workers = 0: ThreadPoolOptions' default (hardware_concurrency,
// thread_pool_options.hpp:50-54).  rgb (nx*ny*3) is zeroed first.  Returns
// the frame's wall seconds, pool construction and teardown included (the
// reference builds the pool inside render_mt, per frame).
double pc_render_mt(const ora_scene *s, const float cam[19], float film_w, float film_h, int nx, int ny,
                    int workers, float *rgb)
{
        std::memset(rgb, 0, sizeof(float) * 3 * (size_t)nx * ny);
        const auto t0 = std::chrono::steady_clock::now();
        {
                const int ntx = 8, nty = 8;
                const int ptx = nx / ntx, pty = ny / nty;
                std::vector<std::promise<void>> waiters(ntx * nty);
                tp::ThreadPoolOptions opt;
                if (workers > 0)
                        opt.setThreadCount((size_t)workers);
                tp::ThreadPool pool(opt);
                for (int tx = 0; tx < ntx; ++tx)
                        for (int ty = 0; ty < nty; ++ty) {
                                std::promise<void> *w = &waiters[tx + ty * ntx];
                                const int x0 = ptx * tx, y0 = pty * ty;
                                pool.post([=]() {
                                        ora_render_tile(s, cam, film_w, film_h, nx, ny, x0, y0, x0 + ptx, y0 + pty,
                                                        rgb);
                                        w->set_value();
                                });
                        }
                for (auto &w : waiters)
                        w.get_future().wait();
        }
        const auto t1 = std::chrono::steady_clock::now();
        return std::chrono::duration<double>(t1 - t0).count();
}

// The pool's default worker count (ThreadPoolOptions().threadCount()).
int pc_default_workers(void)
{
        return (int)tp::ThreadPoolOptions().threadCount();
}
}
