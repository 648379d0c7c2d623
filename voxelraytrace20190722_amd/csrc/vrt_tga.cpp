// vrt_tga.cpp -- TGA decode for the texture pipeline.
//
// The reference loads every diffuse texture with stbi_load(path, &w, &h,
// &channels, 0) (VRT/voxel_octree.cc:373-388, stb_image v2.x bundled as
// VRT/stb_image.h).  Sponza's textures are TGA, and a file whose second byte
// (colour-map type) is 0 or 1 is never claimed by stb's earlier format probes
// (JPEG FF D8, PNG 89 50, BMP 'BM', GIF 'GI', PSD '8B', PIC 53 80, PNM 'P5/6',
// HDR '#?'), so for TGA input stbi_load == stbi__tga_test + stbi__tga_load.
// This file restates those two (VRT/stb_image.h:5323-5335 get_comp,
// 5404-5432 test, 5436-5452 rgb16, 5455-5640 load) over an in-memory
// buffer with stb's read semantics: get8 past the end yields 0, a short
// palette read is an error.  Raw (uncompressed) pixel rows cut short by EOF
// are left uninitialised by stb; here they are zero.  Output = 8-bit
// interleaved, row 0 = top (stbi_set_flip_vertically_on_load is off).
#include "../../include/vrt.h"
#include "vrt_error.h"

#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

struct ByteReader {
        const uint8_t *p, *end;
        int get8()
        {
                return p < end ? *p++ : 0;
        }
        int get16le()
        {
                int lo = get8();
                return lo + (get8() << 8);
        }
        void skip(int64_t n)
        {
                p = (end - p) < n ? end : p + n;
        }
        // all-or-nothing copy; false (nothing consumed past end) when short
        bool getn(uint8_t *dst, int64_t n)
        {
                if (end - p < n) {
                        int64_t have = end - p;
                        memcpy(dst, p, (size_t)have);
                        memset(dst + have, 0, (size_t)(n - have));
                        p = end;
                        return false;
                }
                memcpy(dst, p, (size_t)n);
                p += n;
                return true;
        }
};

// stbi__tga_get_comp: channels for a pixel / palette-entry size
int tga_channels(int bits, bool grey, bool *rgb16)
{
        *rgb16 = false;
        switch (bits) {
        case 8: return 1;
        case 16:
                if (grey) return 2;
                *rgb16 = true;
                return 3;
        case 15: *rgb16 = true; return 3;
        case 24: return 3;
        case 32: return 4;
        default: return 0;
        }
}

bool bits_ok(int b)
{
        return b == 8 || b == 15 || b == 16 || b == 24 || b == 32;
}

// stbi__tga_test: header sanity, no side effects
bool tga_header_ok(const uint8_t *buf, int64_t len)
{
        ByteReader r{buf, buf + len};
        r.get8();
        int cmap = r.get8();
        if (cmap > 1) return false;
        int type = r.get8();
        if (cmap == 1) {
                if (type != 1 && type != 9) return false;
                r.skip(4);
                if (!bits_ok(r.get8())) return false;
                r.skip(4);
        } else {
                if (type != 2 && type != 3 && type != 10 && type != 11) return false;
                r.skip(9);
        }
        if (r.get16le() < 1 || r.get16le() < 1) return false;
        int bpp = r.get8();
        if (cmap == 1 && bpp != 8 && bpp != 16) return false;
        return bits_ok(bpp);
}

// 5-5-5 little-endian pixel -> RGB (stored already in RGB order)
void rgb555(ByteReader &r, uint8_t *out)
{
        int px = r.get16le() & 0xffff;
        out[0] = (uint8_t)((((px >> 10) & 31) * 255) / 31);
        out[1] = (uint8_t)((((px >> 5) & 31) * 255) / 31);
        out[2] = (uint8_t)(((px & 31) * 255) / 31);
}

}  // namespace

extern "C" int vrt_tga_decode(const uint8_t *buf, int64_t len, int *w, int *h,
                              int *comp, uint8_t **out)
{
        if (!buf || len < 0 || !w || !h || !comp || !out)
                return vrt::set_error(VRT_E_INVALID, "vrt_tga_decode: null argument");
        *out = nullptr;
        if (!tga_header_ok(buf, len))
                return vrt::set_error(VRT_E_INVALID, "not a TGA image stb_image would accept");

        ByteReader r{buf, buf + len};
        const int id_len = r.get8();
        const bool indexed = r.get8() != 0;
        int type = r.get8();
        const int pal_start = r.get16le();
        const int pal_len = r.get16le();
        const int pal_bits = r.get8();
        r.get16le();  // x origin
        r.get16le();  // y origin
        const int width = r.get16le();
        const int height = r.get16le();
        const int bpp = r.get8();
        const int desc = r.get8();
        const bool rle = type >= 8;
        if (rle) type -= 8;
        const bool bottom_up = ((desc >> 5) & 1) == 0;  // stb: "inverted"

        bool rgb16 = false;
        const int nc = indexed ? tga_channels(pal_bits, false, &rgb16)
                               : tga_channels(bpp, type == 3, &rgb16);
        if (nc == 0) return vrt::set_error(VRT_E_INVALID, "TGA: bad pixel format");
        // stbi__mad3sizes_valid(w, h, comp, 0)
        if (width > INT_MAX / height || width * height > INT_MAX / nc)
                return vrt::set_error(VRT_E_INVALID, "TGA: image too large");

        const int64_t row = (int64_t)width * nc;
        const int64_t npx = (int64_t)width * height;
        uint8_t *img = (uint8_t *)malloc((size_t)(npx * nc));
        if (!img) return vrt::set_error(VRT_E_NOMEM, "TGA: out of memory");
        r.skip(id_len);

        if (!indexed && !rle && !rgb16) {
                // raw rows straight into place (flipped when stored bottom-up)
                for (int y = 0; y < height; ++y) {
                        int dst = bottom_up ? height - 1 - y : y;
                        r.getn(img + dst * row, row);
                }
        } else {
                std::vector<uint8_t> pal;
                if (indexed) {
                        r.skip(pal_start);  // stb skips this many BYTES
                        pal.assign((size_t)pal_len * nc, 0);
                        if (rgb16) {
                                for (int i = 0; i < pal_len; ++i) rgb555(r, &pal[(size_t)i * nc]);
                        } else if (!r.getn(pal.data(), (int64_t)pal_len * nc)) {
                                free(img);
                                return vrt::set_error(VRT_E_INVALID, "TGA: corrupt palette");
                        }
                }
                uint8_t px[4] = {0, 0, 0, 0};
                int run_left = 0;
                bool run_repeat = false;
                for (int64_t i = 0; i < npx; ++i) {
                        bool fetch = true;
                        if (rle) {
                                if (run_left == 0) {
                                        int cmd = r.get8();
                                        run_left = 1 + (cmd & 127);
                                        run_repeat = (cmd >> 7) != 0;
                                } else if (run_repeat) {
                                        fetch = false;
                                }
                        }
                        if (fetch) {
                                if (indexed) {
                                        int k = bpp == 8 ? r.get8() : r.get16le();
                                        if (k >= pal_len) k = 0;
                                        for (int j = 0; j < nc; ++j)
                                                px[j] = pal.empty() ? 0 : pal[(size_t)k * nc + j];
                                } else if (rgb16) {
                                        rgb555(r, px);
                                } else {
                                        for (int j = 0; j < nc; ++j) px[j] = (uint8_t)r.get8();
                                }
                        }
                        memcpy(img + i * nc, px, (size_t)nc);
                        --run_left;
                }
                if (bottom_up) {
                        std::vector<uint8_t> tmp((size_t)row);
                        for (int y = 0; 2 * y < height; ++y) {
                                uint8_t *a = img + y * row, *b = img + (height - 1 - y) * row;
                                if (a == b) continue;
                                memcpy(tmp.data(), a, (size_t)row);
                                memcpy(a, b, (size_t)row);
                                memcpy(b, tmp.data(), (size_t)row);
                        }
                }
        }
        // BGR(A) -> RGB(A); 5-5-5 sources are already RGB
        if (nc >= 3 && !rgb16)
                for (int64_t i = 0; i < npx; ++i) {
                        uint8_t t = img[i * nc];
                        img[i * nc] = img[i * nc + 2];
                        img[i * nc + 2] = t;
                }
        *w = width;
        *h = height;
        *comp = nc;
        *out = img;
        return VRT_OK;
}

extern "C" int vrt_tga_load(const char *path, int *w, int *h, int *comp, uint8_t **out)
{
        if (!path || !out) return vrt::set_error(VRT_E_INVALID, "vrt_tga_load: null argument");
        *out = nullptr;
        FILE *f = fopen(path, "rb");
        if (!f) return vrt::set_error(VRT_E_IO, "cannot open image '%s'", path);
        std::vector<uint8_t> bytes;
        uint8_t chunk[1 << 16];
        size_t n;
        while ((n = fread(chunk, 1, sizeof chunk, f)) > 0) bytes.insert(bytes.end(), chunk, chunk + n);
        fclose(f);
        int rc = vrt_tga_decode(bytes.data(), (int64_t)bytes.size(), w, h, comp, out);
        if (rc != VRT_OK && rc != VRT_E_NOMEM)
                return vrt::set_error(rc, "image '%s': %s", path, vrt_last_error());
        return rc;
}

extern "C" void vrt_image_free(uint8_t *p)
{
        free(p);
}
