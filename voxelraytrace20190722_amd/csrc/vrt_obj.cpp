// vrt_obj.cpp -- scene ingest: OBJ/MTL -> triangle soup + textures
// (SURVEY.md §8 row f2).
//
// The reference gets its soup from obj2voxel (VRT/voxel_octree.cc:305-371):
// tinyobj::LoadObj(attrib, shapes, materials, .., path, mtldir, triangulate =
// true) from tinyobjloader v1.4.0 (bundled as VRT/tiny_obj_loader.h), then
// one Triangle per (shape, face) with positions / normals / texcoords copied
// through the face's index triples and the face's material; textures are
// read lazily with stbi_load (VRT/voxel_octree.cc:373-411).  This file
// restates the parts of LoadObj that decide the soup bit for bit:
//   * tryParseDouble (tiny_obj_loader.h:567-703) -- NOT correctly rounded,
//     so strtod would differ in the last bit for many inputs;
//   * the line loop (:1813-2278): v/vn/vt/f/usemtl/mtllib/g/o/l and the
//     shape-export rules, including the ones that drop faces (an `o` line
//     after a material change with no new faces loses that shape);
//   * ear-clipping triangulation (exportGroupsToShape, :1080-1339) in float,
//     with its axis choice, signed area, pnpoly ear test and iteration cap;
//   * LoadMtl (:1353-1727) for newmtl / Kd / map_Kd incl. texture options
//     (ParseTextureNameAndOption, :906-990) and first-wins name mapping.
// Statements that cannot change the soup (t, s, vertex colours, other MTL
// keys) are skipped.  Deviations, all where the reference has undefined
// behaviour or exits (DESIGN.md "Ingest"):
//   * faces without a normal index or with an out-of-range index fail with
//     VRT_E_INVALID (reference: assert / out-of-bounds read);
//   * faces with no material (-1) get an extra default material (Kd 0, no
//     texture) instead of reading materials[-1];
//   * a path with no directory part uses "" as mtldir (reference: "/");
//   * an empty map_Kd stays untextured (reference: stbi_load(mtldir) fails
//     and exits) and textures load eagerly, TGA only (vrt_tga.cpp); a texture
//     path with '\\' separators that does not open is retried with '/'.
#include "../../include/vrt.h"
#include "vrt_error.h"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <new>
#include <string>
#include <vector>

namespace {

inline bool blank(char c) { return c == ' ' || c == '\t'; }
inline bool eol(char c) { return c == '\r' || c == '\n' || c == '\0'; }
inline bool digit(char c) { return (unsigned)(c - '0') < 10u; }

// tryParseDouble (tiny_obj_loader.h:567-703).  *e is always one of
// ' ', '\t', '\r', '\0' (parse_real's field end), never a digit.
bool parse_double(const char *s, const char *e, double *out)
{
        static const double kFrac[8] = {1.0, 1e-1, 1e-2, 1e-3, 1e-4, 1e-5, 1e-6, 1e-7};
        if (s >= e) return false;
        const char *p = s;
        bool neg = false;
        if (*p == '+' || *p == '-') {
                neg = *p == '-';
                ++p;
        } else if (!digit(*p)) {
                return false;
        }
        double m = 0.0;
        int n = 0;
        for (; p != e && digit(*p); ++p, ++n) {
                m *= 10;
                m += static_cast<int>(*p - '0');
        }
        if (n == 0) return false;
        int ex = 0;
        bool has_exp = false;
        if (p != e) {
                if (*p == '.') {
                        ++p;
                        for (n = 1; p != e && digit(*p); ++p, ++n)
                                m += static_cast<int>(*p - '0') * (n < 8 ? kFrac[n] : std::pow(10.0, -n));
                        has_exp = p != e && (*p == 'e' || *p == 'E');
                } else {
                        has_exp = *p == 'e' || *p == 'E';
                }
        }
        if (has_exp) {
                ++p;
                bool eneg = false;
                if (p != e && (*p == '+' || *p == '-')) {
                        eneg = *p == '-';
                        ++p;
                } else if (!digit(*p)) {
                        return false;
                }
                for (n = 0; p != e && digit(*p); ++p, ++n) {
                        ex *= 10;
                        ex += static_cast<int>(*p - '0');
                }
                ex *= eneg ? -1 : 1;
                if (n == 0) return false;
        }
        *out = (neg ? -1 : 1) * (ex ? std::ldexp(m * std::pow(5.0, ex), ex) : m);
        return true;
}

// parseReal (tiny_obj_loader.h:705-714): one blank-delimited field
float parse_real(const char **t, double dflt = 0.0)
{
        *t += strspn(*t, " \t");
        const char *end = *t + strcspn(*t, " \t\r");
        double v = dflt;
        parse_double(*t, end, &v);
        *t = end;
        return static_cast<float>(v);
}

// skip one field the way parseOnOff / parseReal / parseString advance
void skip_field(const char **t)
{
        *t += strspn(*t, " \t");
        *t += strcspn(*t, " \t\r");
}

// safeGetline (tiny_obj_loader.h:461-493) over an in-memory file:
// "\n", "\r\n" and a lone "\r" end a line; NULs stay in the line.
struct Lines {
        const std::string &s;
        size_t i = 0;
        bool next(std::string &line)
        {
                if (i >= s.size()) return false;
                line.clear();
                while (i < s.size()) {
                        char c = s[i++];
                        if (c == '\n') break;
                        if (c == '\r') {
                                if (i < s.size() && s[i] == '\n') ++i;
                                break;
                        }
                        line += c;
                }
                return true;
        }
};

// std::ifstream semantics: a directory opens but reads nothing
bool read_file(const std::string &path, std::string *out)
{
        FILE *f = fopen(path.c_str(), "rb");
        if (!f) return false;
        out->clear();
        char buf[1 << 16];
        size_t n;
        while ((n = fread(buf, 1, sizeof buf, f)) > 0) out->append(buf, n);
        fclose(f);
        return true;
}

struct Corner {
        int v = -1, vn = -1, vt = -1;
};

struct Material {
        std::string name;
        float kd[3] = {0.f, 0.f, 0.f};
        std::string tex;  // diffuse_texname
};

// ParseTextureNameAndOption (tiny_obj_loader.h:906-990): options are
// skipped; the name is the rest of the line after them.
void parse_texname(const char *t, std::string *name)
{
        struct Opt {
                const char *key;
                int len, adv, fields;
        };
        static const Opt kOpts[] = {
                {"-blendu", 7, 8, 1}, {"-blendv", 7, 8, 1}, {"-clamp", 6, 7, 1},
                {"-boost", 6, 7, 1},  {"-bm", 3, 4, 1},     {"-o", 2, 3, 3},
                {"-s", 2, 3, 3},      {"-t", 2, 3, 3},      {"-type", 5, 5, 1},
                {"-imfchan", 8, 9, 1}, {"-mm", 3, 4, 2},    {"-colorspace", 11, 12, 1},
        };
        bool found = false;
        std::string got;
        while (!eol(*t)) {
                t += strspn(t, " \t");
                const Opt *hit = nullptr;
                for (const Opt &o : kOpts)
                        if (strncmp(t, o.key, (size_t)o.len) == 0 && blank(t[o.len])) {
                                hit = &o;
                                break;
                        }
                if (hit) {
                        t += hit->adv;
                        for (int k = 0; k < hit->fields; ++k) skip_field(&t);
                } else {
                        got = t;
                        t += got.size();
                        found = true;
                }
        }
        if (found) *name = got;
}

// LoadMtl (tiny_obj_loader.h:1353-1727), reduced to the fields the
// reference renders with (name, diffuse, diffuse_texname).
void load_mtl(const std::string &text, std::map<std::string, int> *map, std::vector<Material> *mats)
{
        Material cur;
        Lines in{text};
        std::string line;
        while (in.next(line)) {
                if (!line.empty()) line = line.substr(0, line.find_last_not_of(" \t") + 1);
                if (line.empty()) continue;
                const char *t = line.c_str();
                t += strspn(t, " \t");
                if (*t == '\0' || *t == '#') continue;
                if (strncmp(t, "newmtl", 6) == 0 && blank(t[6])) {
                        if (!cur.name.empty()) {
                                map->insert({cur.name, (int)mats->size()});
                                mats->push_back(cur);
                        }
                        cur = Material();
                        cur.name = t + 7;
                        continue;
                }
                if (t[0] == 'K' && t[1] == 'd' && blank(t[2])) {
                        t += 2;
                        for (int k = 0; k < 3; ++k) cur.kd[k] = parse_real(&t);
                        continue;
                }
                if (strncmp(t, "map_Kd", 6) == 0 && blank(t[6])) parse_texname(t + 7, &cur.tex);
        }
        map->insert({cur.name, (int)mats->size()});
        mats->push_back(cur);
}

// pnpoly (tiny_obj_loader.h:1063-1076) for a triangle
bool in_tri(const float *vx, const float *vy, float tx, float ty)
{
        bool c = false;
        for (int i = 0, j = 2; i < 3; j = i++)
                if (((vy[i] > ty) != (vy[j] > ty)) &&
                    (tx < (vx[j] - vx[i]) * (ty - vy[i]) / (vy[j] - vy[i]) + vx[i]))
                        c = !c;
        return c;
}

struct Shape {
        std::vector<Corner> idx;   // 3 per triangle
        std::vector<int> mat;      // per triangle
        size_t path = 0;           // mesh.path.indices.size()
        bool empty() const { return idx.empty(); }
};

// exportGroupsToShape (tiny_obj_loader.h:1080-1339), triangulate = true.
// `v` is the position array as parsed SO FAR (forward references read as
// absent, exactly like the reference).  `lines` models lineGroup's size,
// which is swapped into the shape's path.
bool export_faces(Shape *sh, const std::vector<std::vector<Corner>> &faces, size_t *lines, int material,
                  const std::vector<float> &v)
{
        if (faces.empty() && *lines == 0) return false;
        const size_t nv = v.size();
        auto ok2 = [&](int vi, size_t a0, size_t a1) {
                size_t s = size_t(vi);
                return !((s * 3 + a0) >= nv || (s * 3 + a1) >= nv);
        };
        auto emit = [&](const Corner &a, const Corner &b, const Corner &c) {
                sh->idx.push_back(a);
                sh->idx.push_back(b);
                sh->idx.push_back(c);
                sh->mat.push_back(material);
        };
        for (const std::vector<Corner> &face : faces) {
                size_t np = face.size();
                if (np < 3) continue;
                // axis pair from the first corner with a non-tiny cross product
                size_t ax[2] = {1, 2};
                for (size_t k = 0; k < np; ++k) {
                        size_t a = size_t(face[k % np].v), b = size_t(face[(k + 1) % np].v),
                               c = size_t(face[(k + 2) % np].v);
                        if ((3 * a + 2) >= nv || (3 * b + 2) >= nv || (3 * c + 2) >= nv) continue;
                        float e0x = v[b * 3 + 0] - v[a * 3 + 0], e0y = v[b * 3 + 1] - v[a * 3 + 1],
                              e0z = v[b * 3 + 2] - v[a * 3 + 2];
                        float e1x = v[c * 3 + 0] - v[b * 3 + 0], e1y = v[c * 3 + 1] - v[b * 3 + 1],
                              e1z = v[c * 3 + 2] - v[b * 3 + 2];
                        float cx = std::fabs(e0y * e1z - e0z * e1y);
                        float cy = std::fabs(e0z * e1x - e0x * e1z);
                        float cz = std::fabs(e0x * e1y - e0y * e1x);
                        const float eps = 1.1920928955078125e-7f;  // FLT_EPSILON
                        if (cx > eps || cy > eps || cz > eps) {
                                if (!(cx > cy && cx > cz)) {
                                        ax[0] = 0;
                                        if (cz > cx && cz > cy) ax[1] = 1;
                                }
                                break;
                        }
                }
                float area = 0;
                for (size_t k = 0; k < np; ++k) {
                        int a = face[k % np].v, b = face[(k + 1) % np].v;
                        if (!ok2(a, ax[0], ax[1]) || !ok2(b, ax[0], ax[1])) continue;
                        float x0 = v[size_t(a) * 3 + ax[0]], y0 = v[size_t(a) * 3 + ax[1]];
                        float x1 = v[size_t(b) * 3 + ax[0]], y1 = v[size_t(b) * 3 + ax[1]];
                        area += (x0 * y1 - y0 * x1) * 0.5f;
                }
                std::vector<Corner> rem = face;
                size_t guess = 0;
                size_t iters = face.size();
                size_t prev = rem.size();
                Corner ind[3];
                float vx[3], vy[3];
                while (rem.size() > 3 && iters > 0) {
                        np = rem.size();
                        if (guess >= np) guess -= np;
                        if (prev != np) {
                                prev = np;
                                iters = np;
                        } else {
                                --iters;
                        }
                        for (size_t k = 0; k < 3; ++k) {
                                ind[k] = rem[(guess + k) % np];
                                if (ok2(ind[k].v, ax[0], ax[1])) {
                                        vx[k] = v[size_t(ind[k].v) * 3 + ax[0]];
                                        vy[k] = v[size_t(ind[k].v) * 3 + ax[1]];
                                } else {
                                        vx[k] = vy[k] = 0.f;
                                }
                        }
                        float cross = (vx[1] - vx[0]) * (vy[2] - vy[1]) - (vy[1] - vy[0]) * (vx[2] - vx[1]);
                        if (cross * area < 0.f) {
                                ++guess;
                                continue;
                        }
                        bool overlap = false;
                        for (size_t o = 3; o < np; ++o) {
                                size_t i = (guess + o) % np;
                                int ov = rem[i].v;
                                if (!ok2(ov, ax[0], ax[1])) continue;
                                if (in_tri(vx, vy, v[size_t(ov) * 3 + ax[0]], v[size_t(ov) * 3 + ax[1]])) {
                                        overlap = true;
                                        break;
                                }
                        }
                        if (overlap) {
                                ++guess;
                                continue;
                        }
                        emit(ind[0], ind[1], ind[2]);
                        rem.erase(rem.begin() + (long)((guess + 1) % np));
                }
                if (rem.size() == 3) emit(rem[0], rem[1], rem[2]);
        }
        if (*lines) std::swap(*lines, sh->path);
        return true;
}

// fixIndex (tiny_obj_loader.h:501-525)
bool fix_index(int idx, int n, int *ret)
{
        if (idx > 0) {
                *ret = idx - 1;
                return true;
        }
        if (idx == 0) return false;
        *ret = n + idx;
        return true;
}

// parseTriple (tiny_obj_loader.h:820-876): v, v/vt, v//vn, v/vt/vn
bool parse_corner(const char **t, int nv, int nvn, int nvt, Corner *out)
{
        Corner c;
        if (!fix_index(atoi(*t), nv, &c.v)) return false;
        *t += strcspn(*t, "/ \t\r");
        if (**t != '/') {
                *out = c;
                return true;
        }
        ++*t;
        if (**t == '/') {
                ++*t;
                if (!fix_index(atoi(*t), nvn, &c.vn)) return false;
                *t += strcspn(*t, "/ \t\r");
                *out = c;
                return true;
        }
        if (!fix_index(atoi(*t), nvt, &c.vt)) return false;
        *t += strcspn(*t, "/ \t\r");
        if (**t == '/') {
                ++*t;
                if (!fix_index(atoi(*t), nvn, &c.vn)) return false;
                *t += strcspn(*t, "/ \t\r");
        }
        *out = c;
        return true;
}

// std::getline(ss, item, ' ') split used for `mtllib a b c`
std::vector<std::string> split_space(const std::string &s)
{
        std::vector<std::string> out;
        size_t i = 0;
        while (i < s.size()) {
                size_t k = s.find(' ', i);
                if (k == std::string::npos) {
                        out.push_back(s.substr(i));
                        break;
                }
                out.push_back(s.substr(i, k - i));
                i = k + 1;
        }
        return out;
}

}  // namespace

struct __attribute__((visibility("hidden"))) vrt_obj {
        // tinyobj::LoadObj outputs
        std::vector<float> v, vn, vt;
        std::vector<Shape> shapes;
        std::vector<Material> mats;
        std::string warn;
        // obj2voxel soup (absent with VRT_OBJ_PARSE_ONLY)
        bool has_soup = false;
        std::vector<float> pos, nrm, uv;
        std::vector<int32_t> mat, mat_tex;
        std::vector<float> mat_kd;
        std::vector<std::string> tex_path;
        std::vector<int32_t> tex_dims;
        std::vector<int64_t> tex_off;
        std::vector<uint8_t> tex_data;
        int64_t ntri = 0;
};

namespace {

// tinyobj::LoadObj(.., filename, mtl_basedir, triangulate = true)
// (tiny_obj_loader.h:1777-1811 + 1813-2278)
int load_obj(const std::string &path, const std::string &mtldir, vrt_obj *o)
{
        std::string text;
        if (!read_file(path, &text)) return vrt::set_error(VRT_E_IO, "cannot open '%s'", path.c_str());
        std::map<std::string, int> matmap;
        std::vector<std::vector<Corner>> faces;
        size_t lines = 0;
        int material = -1;
        Shape sh;
        Lines in{text};
        std::string line;
        size_t lineno = 0;
        while (in.next(line)) {
                ++lineno;
                if (!line.empty() && line.back() == '\n') line.pop_back();
                if (!line.empty() && line.back() == '\r') line.pop_back();
                if (line.empty()) continue;
                const char *t = line.c_str();
                t += strspn(t, " \t");
                if (*t == '\0' || *t == '#') continue;
                if (t[0] == 'v' && blank(t[1])) {
                        t += 2;
                        for (int k = 0; k < 3; ++k) o->v.push_back(parse_real(&t));
                        continue;
                }
                if (t[0] == 'v' && t[1] == 'n' && blank(t[2])) {
                        t += 3;
                        for (int k = 0; k < 3; ++k) o->vn.push_back(parse_real(&t));
                        continue;
                }
                if (t[0] == 'v' && t[1] == 't' && blank(t[2])) {
                        t += 3;
                        for (int k = 0; k < 2; ++k) o->vt.push_back(parse_real(&t));
                        continue;
                }
                if (t[0] == 'l' && blank(t[1])) {
                        // only the pair count matters (it decides shape export)
                        t += 2;
                        size_t k = 0;
                        while (!eol(*t)) {
                                skip_field(&t);
                                t += strspn(t, " \t\r");
                                ++k;
                        }
                        lines += 2 * (k / 2);
                        continue;
                }
                if (t[0] == 'f' && blank(t[1])) {
                        t += 2;
                        t += strspn(t, " \t");
                        std::vector<Corner> face;
                        face.reserve(3);
                        while (!eol(*t)) {
                                Corner c;
                                if (!parse_corner(&t, (int)(o->v.size() / 3), (int)(o->vn.size() / 3),
                                                  (int)(o->vt.size() / 2), &c))
                                        return vrt::set_error(VRT_E_INVALID,
                                                              "%s:%zu: failed to parse `f' line (zero index?)",
                                                              path.c_str(), lineno);
                                face.push_back(c);
                                t += strspn(t, " \t\r");
                        }
                        faces.push_back(std::move(face));
                        continue;
                }
                if (strncmp(t, "usemtl", 6) == 0 && blank(t[6])) {
                        auto it = matmap.find(std::string(t + 7));
                        int id = it == matmap.end() ? -1 : it->second;
                        if (id != material) {
                                export_faces(&sh, faces, &lines, material, o->v);
                                faces.clear();
                                material = id;
                        }
                        continue;
                }
                if (strncmp(t, "mtllib", 6) == 0 && blank(t[6])) {
                        std::vector<std::string> names = split_space(std::string(t + 7));
                        bool found = false;
                        for (const std::string &n : names) {
                                std::string mtext;
                                if (read_file(mtldir + n, &mtext)) {
                                        load_mtl(mtext, &matmap, &o->mats);
                                        found = true;
                                        break;
                                }
                        }
                        if (!names.empty() && !found)
                                o->warn += "failed to load material file(s) named on line " +
                                           std::to_string(lineno) + "\n";
                        continue;
                }
                if (t[0] == 'g' && blank(t[1])) {
                        export_faces(&sh, faces, &lines, material, o->v);
                        if (!sh.empty()) o->shapes.push_back(std::move(sh));
                        sh = Shape();
                        faces.clear();
                        continue;
                }
                if (t[0] == 'o' && blank(t[1])) {
                        if (export_faces(&sh, faces, &lines, material, o->v)) o->shapes.push_back(std::move(sh));
                        faces.clear();
                        sh = Shape();
                        continue;
                }
        }
        bool ret = export_faces(&sh, faces, &lines, material, o->v);
        if (ret || !sh.empty()) o->shapes.push_back(std::move(sh));
        return VRT_OK;
}

std::string base_dir(const std::string &p)
{
        size_t k = p.find_last_of("/\\");
        return k == std::string::npos ? std::string() : p.substr(0, k);
}

// obj2voxel's soup (VRT/voxel_octree.cc:336-368) + load_image of every
// texture a face uses (VRT/voxel_octree.cc:373-411, texel_fetch cache).
int build_soup(vrt_obj *o, const std::string &mtldir)
{
        const int64_t nv = (int64_t)o->v.size() / 3, nvn = (int64_t)o->vn.size() / 3,
                      nvt = (int64_t)o->vt.size() / 2;
        int64_t ntri = 0;
        for (const Shape &s : o->shapes) ntri += (int64_t)s.mat.size();
        if (ntri > INT32_MAX) return vrt::set_error(VRT_E_INVALID, "too many triangles (%lld)", (long long)ntri);
        const int nmat = (int)o->mats.size();
        int default_mat = -1;
        o->pos.resize((size_t)ntri * 9);
        o->nrm.resize((size_t)ntri * 9);
        o->uv.assign((size_t)ntri * 6, 0.f);
        o->mat.resize((size_t)ntri);
        std::vector<char> used((size_t)nmat + 1, 0);
        int64_t t = 0;
        for (size_t si = 0; si < o->shapes.size(); ++si) {
                const Shape &s = o->shapes[si];
                for (size_t f = 0; f < s.mat.size(); ++f, ++t) {
                        for (int k = 0; k < 3; ++k) {
                                const Corner &c = s.idx[f * 3 + k];
                                if (c.v < 0 || c.v >= nv)
                                        return vrt::set_error(VRT_E_INVALID,
                                                              "shape %zu face %zu: vertex index %d out of range",
                                                              si, f, c.v);
                                if (c.vn < 0 || c.vn >= nvn)
                                        return vrt::set_error(VRT_E_INVALID,
                                                              "shape %zu face %zu: missing or out-of-range normal "
                                                              "index %d (obj2voxel requires normals)",
                                                              si, f, c.vn);
                                if (c.vt >= nvt)
                                        return vrt::set_error(VRT_E_INVALID,
                                                              "shape %zu face %zu: texcoord index %d out of range",
                                                              si, f, c.vt);
                                memcpy(&o->pos[t * 9 + k * 3], &o->v[(size_t)c.v * 3], 12);
                                memcpy(&o->nrm[t * 9 + k * 3], &o->vn[(size_t)c.vn * 3], 12);
                                if (c.vt >= 0) memcpy(&o->uv[t * 6 + k * 2], &o->vt[(size_t)c.vt * 2], 8);
                        }
                        int m = s.mat[f];
                        if (m < 0) {
                                if (default_mat < 0) default_mat = nmat;
                                m = default_mat;
                        }
                        o->mat[t] = m;
                        used[(size_t)m] = 1;
                }
        }
        o->ntri = ntri;
        const int nm = nmat + (default_mat >= 0 ? 1 : 0);
        o->mat_kd.assign((size_t)nm * 3, 0.f);
        o->mat_tex.assign((size_t)nm, -1);
        std::map<std::string, int> texid;
        for (int m = 0; m < nmat; ++m) {
                Material &mt = o->mats[(size_t)m];
                memcpy(&o->mat_kd[(size_t)m * 3], mt.kd, 12);
                if (!used[(size_t)m] || mt.tex.empty()) continue;
                std::string p = mt.tex.rfind(mtldir, 0) == 0 ? mt.tex : mtldir + mt.tex;
                auto it = texid.find(p);
                if (it != texid.end()) {
                        o->mat_tex[(size_t)m] = it->second;
                        continue;
                }
                int w = 0, h = 0, c = 0;
                uint8_t *img = nullptr;
                int rc = vrt_tga_load(p.c_str(), &w, &h, &c, &img);
                if (rc == VRT_E_IO && p.find('\\') != std::string::npos) {
                        std::string q = p;
                        for (char &ch : q)
                                if (ch == '\\') ch = '/';
                        rc = vrt_tga_load(q.c_str(), &w, &h, &c, &img);
                }
                if (rc != VRT_OK) return vrt::set_error(rc, "material '%s': %s", mt.name.c_str(), vrt_last_error());
                int id = (int)o->tex_path.size();
                texid[p] = id;
                o->tex_path.push_back(p);
                o->tex_dims.insert(o->tex_dims.end(), {w, h, c});
                o->tex_off.push_back((int64_t)o->tex_data.size());
                o->tex_data.insert(o->tex_data.end(), img, img + (size_t)w * h * c);
                vrt_image_free(img);
                o->mat_tex[(size_t)m] = id;
        }
        o->has_soup = true;
        return VRT_OK;
}

}  // namespace

extern "C" int vrt_obj_load(const char *obj_path, int flags, vrt_obj **out)
{
        if (!obj_path || !out) return vrt::set_error(VRT_E_INVALID, "vrt_obj_load: null argument");
        *out = nullptr;
        if (flags & ~VRT_OBJ_PARSE_ONLY) return vrt::set_error(VRT_E_INVALID, "vrt_obj_load: unknown flags %#x", flags);
        std::unique_ptr<vrt_obj> o(new (std::nothrow) vrt_obj);
        if (!o) return vrt::set_error(VRT_E_NOMEM, "vrt_obj_load: out of memory");
        const std::string path(obj_path);
        const std::string dir = base_dir(path);
        const std::string mtldir = dir.empty() ? std::string() : dir + "/";
        try {
                int rc = load_obj(path, mtldir, o.get());
                if (rc != VRT_OK) return rc;
                if (!(flags & VRT_OBJ_PARSE_ONLY)) {
                        rc = build_soup(o.get(), mtldir);
                        if (rc != VRT_OK) return rc;
                }
        } catch (const std::bad_alloc &) {
                return vrt::set_error(VRT_E_NOMEM, "vrt_obj_load: out of memory");
        }
        *out = o.release();
        return VRT_OK;
}

extern "C" void vrt_obj_free(vrt_obj *o)
{
        delete o;
}

extern "C" int vrt_obj_info(const vrt_obj *o, vrt_obj_info_t *info)
{
        if (!o || !info) return vrt::set_error(VRT_E_INVALID, "vrt_obj_info: null argument");
        info->nvert = (int64_t)o->v.size() / 3;
        info->nnormal = (int64_t)o->vn.size() / 3;
        info->ntexcoord = (int64_t)o->vt.size() / 2;
        info->nshape = (int32_t)o->shapes.size();
        int64_t nf = 0;
        for (const Shape &s : o->shapes) nf += (int64_t)s.mat.size();
        info->nface = nf;
        info->nmat = (int32_t)o->mats.size();
        info->has_soup = o->has_soup ? 1 : 0;
        info->nsoup_mat = (int32_t)o->mat_tex.size();
        info->ntex = (int32_t)o->tex_path.size();
        info->tex_bytes = (int64_t)o->tex_data.size();
        return VRT_OK;
}

extern "C" int vrt_obj_attrib(const vrt_obj *o, const float **v, const float **vn, const float **vt)
{
        if (!o) return vrt::set_error(VRT_E_INVALID, "vrt_obj_attrib: null argument");
        if (v) *v = o->v.data();
        if (vn) *vn = o->vn.data();
        if (vt) *vt = o->vt.data();
        return VRT_OK;
}

extern "C" int vrt_obj_faces(const vrt_obj *o, int32_t *idx, int32_t *mat, int32_t *shape)
{
        if (!o) return vrt::set_error(VRT_E_INVALID, "vrt_obj_faces: null argument");
        int64_t f = 0;
        for (size_t s = 0; s < o->shapes.size(); ++s) {
                const Shape &sh = o->shapes[s];
                for (size_t k = 0; k < sh.mat.size(); ++k, ++f) {
                        if (idx)
                                for (int c = 0; c < 3; ++c) {
                                        const Corner &q = sh.idx[k * 3 + c];
                                        idx[f * 9 + c * 3 + 0] = q.v;
                                        idx[f * 9 + c * 3 + 1] = q.vn;
                                        idx[f * 9 + c * 3 + 2] = q.vt;
                                }
                        if (mat) mat[f] = sh.mat[k];
                        if (shape) shape[f] = (int32_t)s;
                }
        }
        return VRT_OK;
}

extern "C" int vrt_obj_material(const vrt_obj *o, int i, const char **name, float kd[3], const char **texname)
{
        if (!o || i < 0 || i >= (int)o->mats.size())
                return vrt::set_error(VRT_E_INVALID, "vrt_obj_material: bad handle or index %d", i);
        const Material &m = o->mats[(size_t)i];
        if (name) *name = m.name.c_str();
        if (kd) memcpy(kd, m.kd, 12);
        if (texname) *texname = m.tex.c_str();
        return VRT_OK;
}

extern "C" int vrt_obj_texture_path(const vrt_obj *o, int i, const char **path)
{
        if (!o || !path || i < 0 || i >= (int)o->tex_path.size())
                return vrt::set_error(VRT_E_INVALID, "vrt_obj_texture_path: bad handle or index %d", i);
        *path = o->tex_path[(size_t)i].c_str();
        return VRT_OK;
}

extern "C" const char *vrt_obj_warnings(const vrt_obj *o)
{
        return o ? o->warn.c_str() : "";
}

extern "C" int vrt_obj_scene_desc(const vrt_obj *o, vrt_scene_desc *d)
{
        if (!o || !d) return vrt::set_error(VRT_E_INVALID, "vrt_obj_scene_desc: null argument");
        if (!o->has_soup) return vrt::set_error(VRT_E_INVALID, "vrt_obj_scene_desc: loaded with VRT_OBJ_PARSE_ONLY");
        if (o->mat_tex.empty()) return vrt::set_error(VRT_E_INVALID, "vrt_obj_scene_desc: model has no faces");
        memset(d, 0, sizeof *d);
        d->ntri = (int32_t)o->ntri;
        d->pos = o->pos.data();
        d->nrm = o->nrm.data();
        d->uv = o->uv.data();
        d->mat = o->mat.data();
        d->nmat = (int32_t)o->mat_tex.size();
        d->mat_tex = o->mat_tex.data();
        d->mat_kd = o->mat_kd.data();
        d->ntex = (int32_t)o->tex_path.size();
        d->tex_dims = o->tex_dims.empty() ? nullptr : o->tex_dims.data();
        d->tex_off = o->tex_off.empty() ? nullptr : o->tex_off.data();
        d->tex_data = o->tex_data.empty() ? nullptr : o->tex_data.data();
        d->tex_bytes = (int64_t)o->tex_data.size();
        return VRT_OK;
}
