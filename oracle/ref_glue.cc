// ref_glue.cc -- TEST INFRASTRUCTURE ONLY.
//
// C-linkage entry points onto the reference's own, unmodified sources, which
// oracle/Makefile compiles in place from /root/reference into
// oracle/_ref/libvrtref.so (never shipped, never loaded by the product):
//   - intersect_triangle3   VRT/raytri.cc:197-249   (declared in VRT/raytri.h:5-7)
//   - triBoxOverlap         VRT/tribox2.cc:122-196  (declared in VRT/tribox2.h:6)
//   - stbi_write_hdr_to_func / stbi_write_hdr  VRT/stb_image_write.h:178,757
// Nothing here re-implements reference behaviour; it only forwards.
#include "raytri.h"
#include "tribox2.h"

#include <cstdlib>
#include <cstring>
#include <vector>

#define STB_IMAGE_WRITE_IMPLEMENTATION
#include "stb_image_write.h"

extern "C" {

int ref_intersect_triangle3(const double orig[3], const double dir[3],
                            const double v0[3], const double v1[3],
                            const double v2[3], double out[3], int *wrote)
{
        double o[3], d[3], a[3], b[3], c[3];
        std::memcpy(o, orig, sizeof o);
        std::memcpy(d, dir, sizeof d);
        std::memcpy(a, v0, sizeof a);
        std::memcpy(b, v1, sizeof b);
        std::memcpy(c, v2, sizeof c);
        out[0] = out[1] = out[2] = 0.0;
        int r = intersect_triangle3(o, d, a, b, c, &out[0], &out[1], &out[2]);
        if (wrote)
                *wrote = r;
        return r;
}

int ref_tri_box_overlap(const float center[3], const float half[3],
                        const float tri[9])
{
        float c[3], h[3], t[3][3];
        std::memcpy(c, center, sizeof c);
        std::memcpy(h, half, sizeof h);
        std::memcpy(t, tri, sizeof t);
        return triBoxOverlap(c, h, t);
}

static void collect(void *ctx, void *data, int size)
{
        auto *v = static_cast<std::vector<unsigned char> *>(ctx);
        auto *p = static_cast<unsigned char *>(data);
        v->insert(v->end(), p, p + size);
}

// Encode with the reference writer into memory.  Returns the byte count
// (or -needed when cap is too small, 0 on writer failure).
long ref_write_hdr_mem(int w, int h, int comp, const float *data,
                       unsigned char *out, long cap)
{
        std::vector<unsigned char> buf;
        if (!stbi_write_hdr_to_func(collect, &buf, w, h, comp, data))
                return 0;
        if ((long)buf.size() > cap)
                return -(long)buf.size();
        std::memcpy(out, buf.data(), buf.size());
        return (long)buf.size();
}

int ref_write_hdr_file(const char *path, int w, int h, int comp,
                       const float *data)
{
        return stbi_write_hdr(path, w, h, comp, data);
}
}
