// vrt_hdr.cpp -- Radiance .hdr output, byte-identical to the reference's
// stbi_write_hdr (VRT/stb_image_write.h v1.13, :595-757): header, per-row
// "2 2 hi lo" scanline header, and per-component RLE of the RGBE bytes.
// Two entry paths: float pixels (RGBE packing here, as stb does), or RGBE
// bytes already packed on the device by k_rgbe (vrt_rgbe_device), which
// leaves only the serial RLE to the host.
#include "../../include/vrt.h"

#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

namespace {

// (unsigned char)(float) as the reference's x86-64 build executes it:
// cvttss2si to int32 (INT_MIN when out of range / NaN), low byte kept.
inline unsigned char to_uchar(float f)
{
        int i;
        if (!(f >= -2147483648.0f && f < 2147483648.0f))
                i = INT_MIN;
        else
                i = (int)f;
        return (unsigned char)i;
}

// stbiw__linear_to_rgbe (:601-616)
void linear_to_rgbe(unsigned char *rgbe, const float *lin)
{
        const float m12 = lin[1] > lin[2] ? lin[1] : lin[2];
        const float maxcomp = lin[0] > m12 ? lin[0] : m12;
        if (maxcomp < 1e-32f) {
                rgbe[0] = rgbe[1] = rgbe[2] = rgbe[3] = 0;
        } else {
                int e;
                const float nrm = (float)std::frexp(maxcomp, &e) * 256.0f / maxcomp;
                rgbe[0] = to_uchar(lin[0] * nrm);
                rgbe[1] = to_uchar(lin[1] * nrm);
                rgbe[2] = to_uchar(lin[2] * nrm);
                rgbe[3] = (unsigned char)(e + 128);
        }
}

struct Out {
        std::vector<unsigned char> b;
        void put(const void *p, size_t n)
        {
                const unsigned char *c = static_cast<const unsigned char *>(p);
                b.insert(b.end(), c, c + n);
        }
};

void pixel_linear(const float *scan, int x, int ncomp, float lin[3])
{
        if (ncomp >= 3) {
                lin[2] = scan[x * ncomp + 2];
                lin[1] = scan[x * ncomp + 1];
                lin[0] = scan[x * ncomp + 0];
        } else {
                lin[0] = lin[1] = lin[2] = scan[x * ncomp + 0];
        }
}

// RLE of one scanline held as 4 component planes (scratch[x + width*c]),
// the second half of stbiw__write_hdr_scanline (:651-718)
void rle_planes(Out &o, int width, const unsigned char *scratch)
{
        const unsigned char hdr[4] = { 2, 2, (unsigned char)((width & 0xff00) >> 8),
                                       (unsigned char)(width & 0x00ff) };
        o.put(hdr, 4);
        for (int c = 0; c < 4; ++c) {
                const unsigned char *comp = &scratch[width * c];
                int x = 0;
                while (x < width) {
                        int r = x;  // first run of >= 3 equal bytes at/after x
                        while (r + 2 < width) {
                                if (comp[r] == comp[r + 1] && comp[r] == comp[r + 2])
                                        break;
                                ++r;
                        }
                        if (r + 2 >= width)
                                r = width;
                        while (x < r) {  // literal dump, <= 128 per packet
                                int len = r - x;
                                if (len > 128)
                                        len = 128;
                                const unsigned char lb = (unsigned char)len;
                                o.put(&lb, 1);
                                o.put(&comp[x], (size_t)len);
                                x += len;
                        }
                        if (r + 2 < width) {  // run, <= 127 per packet
                                while (r < width && comp[r] == comp[x])
                                        ++r;
                                while (x < r) {
                                        int len = r - x;
                                        if (len > 127)
                                                len = 127;
                                        const unsigned char pk[2] = { (unsigned char)(len + 128), comp[x] };
                                        o.put(pk, 2);
                                        x += len;
                                }
                        }
                }
        }
}

// stbiw__write_hdr_scanline (:634-719) from float pixels
void scanline(Out &o, int width, int ncomp, unsigned char *scratch,
              const float *scan)
{
        unsigned char rgbe[4];
        float lin[3];
        if (width < 8 || width >= 32768) {  // no RLE
                for (int x = 0; x < width; ++x) {
                        pixel_linear(scan, x, ncomp, lin);
                        linear_to_rgbe(rgbe, lin);
                        o.put(rgbe, 4);
                }
                return;
        }
        for (int x = 0; x < width; ++x) {
                pixel_linear(scan, x, ncomp, lin);
                linear_to_rgbe(rgbe, lin);
                for (int c = 0; c < 4; ++c)
                        scratch[x + width * c] = rgbe[c];
        }
        rle_planes(o, width, scratch);
}

// the same scanline from RGBE bytes packed on the device (vrt_rgbe_device)
void scanline_rgbe(Out &o, int width, unsigned char *scratch, const unsigned char *rgbe)
{
        if (width < 8 || width >= 32768) {
                o.put(rgbe, (size_t)width * 4);
                return;
        }
        for (int x = 0; x < width; ++x)
                for (int c = 0; c < 4; ++c)
                        scratch[x + width * c] = rgbe[4 * x + c];
        rle_planes(o, width, scratch);
}

void header(Out &o, int w, int h)
{
        static const char head[] =
                "#?RADIANCE\n# Written by stb_image_write.h\nFORMAT=32-bit_rle_rgbe\n";
        o.put(head, sizeof(head) - 1);
        char buf[128];
        const int len = std::snprintf(buf, sizeof buf,
                                      "EXPOSURE=          1.0000000000000\n\n-Y %d +X %d\n", h, w);
        o.put(buf, (size_t)len);
}

// stbi_write_hdr_core (:723-747)
bool encode(int w, int h, int comp, const float *data, Out &o)
{
        if (h <= 0 || w <= 0 || data == nullptr)
                return false;
        std::vector<unsigned char> scratch((size_t)w * 4);
        header(o, w, h);
        for (int i = 0; i < h; ++i)
                scanline(o, w, comp, scratch.data(), data + (size_t)comp * w * i);
        return true;
}

bool encode_rgbe(int w, int h, const unsigned char *rgbe, Out &o)
{
        if (h <= 0 || w <= 0 || rgbe == nullptr)
                return false;
        std::vector<unsigned char> scratch((size_t)w * 4);
        header(o, w, h);
        for (int i = 0; i < h; ++i)
                scanline_rgbe(o, w, scratch.data(), rgbe + (size_t)4 * w * i);
        return true;
}

int64_t to_mem(const Out &o, uint8_t *out, int64_t cap)
{
        if ((int64_t)o.b.size() > cap || !out)
                return -(int64_t)o.b.size();
        std::memcpy(out, o.b.data(), o.b.size());
        return (int64_t)o.b.size();
}

int to_file(const Out &o, const char *filename)
{
        std::FILE *f = std::fopen(filename, "wb");
        if (!f)
                return 0;
        const size_t n = std::fwrite(o.b.data(), 1, o.b.size(), f);
        const int ok = (n == o.b.size()) && std::fclose(f) == 0;
        if (n != o.b.size())
                std::fclose(f);
        return ok ? 1 : 0;
}

}  // namespace

extern "C" int64_t vrt_write_hdr_rgbe_mem(int w, int h, const uint8_t *rgbe, uint8_t *out, int64_t cap)
{
        Out o;
        if (!encode_rgbe(w, h, rgbe, o))
                return 0;
        return to_mem(o, out, cap);
}

extern "C" int vrt_write_hdr_rgbe(const char *filename, int w, int h, const uint8_t *rgbe)
{
        Out o;
        if (!filename || !encode_rgbe(w, h, rgbe, o))
                return 0;
        return to_file(o, filename);
}

extern "C" int64_t vrt_write_hdr_mem(int w, int h, int comp, const float *data,
                                     uint8_t *out, int64_t cap)
{
        Out o;
        if (comp < 1 || comp > 4 || !encode(w, h, comp, data, o))
                return 0;
        return to_mem(o, out, cap);
}

extern "C" int vrt_write_hdr(const char *filename, int w, int h, int comp,
                             const float *data)
{
        if (!filename || comp < 1 || comp > 4)
                return 0;
        Out o;
        if (!encode(w, h, comp, data, o))
                return 0;
        return to_file(o, filename);
}

// the reference's own entry point (VRT/stb_image_write.h:178): same writer
extern "C" int stbi_write_hdr(char const *filename, int w, int h, int comp, const float *data)
{
        return vrt_write_hdr(filename, w, h, comp, data);
}
