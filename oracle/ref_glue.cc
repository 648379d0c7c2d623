// ref_glue.cc -- TEST INFRASTRUCTURE ONLY.
//
// C-linkage entry points onto the reference's own, unmodified sources, which
// oracle/Makefile compiles in place from /root/reference into
// oracle/_ref/libvrtref.so (never shipped, never loaded by the product):
//   - intersect_triangle3   VRT/raytri.cc:197-249   (declared in VRT/raytri.h:5-7)
//   - triBoxOverlap         VRT/tribox2.cc:122-196  (declared in VRT/tribox2.h:6)
//   - stbi_write_hdr_to_func / stbi_write_hdr  VRT/stb_image_write.h:178,757
//   - tinyobj::LoadObj      VRT/tiny_obj_loader.cc (v1.4.0 implementation),
//                           called with obj2voxel's arguments
//                           (VRT/voxel_octree.cc:316-317); its attrib /
//                           shapes / materials are flattened to C arrays
//   - stbi_load / stbi_load_from_memory  VRT/stb_image.h (load_image's call,
//                           VRT/voxel_octree.cc:377)
// Nothing here re-implements reference behaviour; it only forwards.
#include "raytri.h"
#include "tribox2.h"
#include "tiny_obj_loader.h"

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define STB_IMAGE_WRITE_IMPLEMENTATION
#include "stb_image_write.h"
#define STB_IMAGE_IMPLEMENTATION
#include "stb_image.h"

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

// ---- tinyobj::LoadObj, flattened ------------------------------------------
struct ref_obj {
        int32_t ok;
        int64_t nv, nvn, nvt;           // attrib sizes / 3, / 3, / 2
        float *v, *vn, *vt;
        int32_t nshape;
        int64_t nface;
        int32_t *fv;                    // num_face_vertices (all 3 here)
        int32_t *idx;                   // nface*9 {vertex, normal, texcoord} x 3
        int32_t *mat;                   // material_ids
        int32_t *shape;                 // owning shape
        int32_t nmat;
        float *kd;                      // nmat*3 material_t::diffuse
        char **name, **tex;             // material_t::name / diffuse_texname
        char *warn, *err;
};

}  // extern "C"

static char *dup(const std::string &s)
{
        char *p = (char *)std::malloc(s.size() + 1);
        std::memcpy(p, s.c_str(), s.size() + 1);
        return p;
}

template <class T>
static T *copy_vec(const std::vector<T> &v)
{
        T *p = (T *)std::malloc(v.size() * sizeof(T) + 1);
        if (!v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
        return p;
}

extern "C" {

ref_obj *ref_load_obj(const char *path, const char *mtl_basedir)
{
        tinyobj::attrib_t attrib;
        std::vector<tinyobj::shape_t> shapes;
        std::vector<tinyobj::material_t> materials;
        std::string warn, err;
        bool ok = tinyobj::LoadObj(&attrib, &shapes, &materials, &warn, &err, path, mtl_basedir, true);
        ref_obj *o = (ref_obj *)std::calloc(1, sizeof(ref_obj));
        o->ok = ok ? 1 : 0;
        o->nv = (int64_t)attrib.vertices.size() / 3;
        o->nvn = (int64_t)attrib.normals.size() / 3;
        o->nvt = (int64_t)attrib.texcoords.size() / 2;
        o->v = copy_vec(attrib.vertices);
        o->vn = copy_vec(attrib.normals);
        o->vt = copy_vec(attrib.texcoords);
        o->nshape = (int32_t)shapes.size();
        std::vector<int32_t> fv, idx, mat, shp;
        for (size_t s = 0; s < shapes.size(); ++s) {
                const tinyobj::mesh_t &m = shapes[s].mesh;
                size_t base = 0;
                for (size_t f = 0; f < m.num_face_vertices.size(); ++f) {
                        int n = m.num_face_vertices[f];
                        fv.push_back(n);
                        for (int k = 0; k < 3; ++k) {
                                const tinyobj::index_t &q = m.indices[base + (k < n ? k : 0)];
                                idx.push_back(q.vertex_index);
                                idx.push_back(q.normal_index);
                                idx.push_back(q.texcoord_index);
                        }
                        base += (size_t)n;
                        mat.push_back(m.material_ids[f]);
                        shp.push_back((int32_t)s);
                }
        }
        o->nface = (int64_t)fv.size();
        o->fv = copy_vec(fv);
        o->idx = copy_vec(idx);
        o->mat = copy_vec(mat);
        o->shape = copy_vec(shp);
        o->nmat = (int32_t)materials.size();
        o->kd = (float *)std::malloc(materials.size() * 3 * sizeof(float) + 1);
        o->name = (char **)std::malloc(materials.size() * sizeof(char *) + 1);
        o->tex = (char **)std::malloc(materials.size() * sizeof(char *) + 1);
        for (size_t m = 0; m < materials.size(); ++m) {
                std::memcpy(o->kd + 3 * m, materials[m].diffuse, 3 * sizeof(float));
                o->name[m] = dup(materials[m].name);
                o->tex[m] = dup(materials[m].diffuse_texname);
        }
        o->warn = dup(warn);
        o->err = dup(err);
        return o;
}

void ref_free_obj(ref_obj *o)
{
        if (!o) return;
        for (int32_t m = 0; m < o->nmat; ++m) {
                std::free(o->name[m]);
                std::free(o->tex[m]);
        }
        void *ps[] = {o->v, o->vn, o->vt, o->fv, o->idx, o->mat, o->shape, o->kd, o->name, o->tex, o->warn, o->err};
        for (void *p : ps) std::free(p);
        std::free(o);
}

// ---- stbi_load (load_image's call: req_comp = 0) ---------------------------
unsigned char *ref_stbi_load(const char *path, int *w, int *h, int *comp)
{
        return stbi_load(path, w, h, comp, 0);
}

unsigned char *ref_stbi_load_mem(const unsigned char *buf, int len, int *w, int *h, int *comp)
{
        return stbi_load_from_memory(buf, len, w, h, comp, 0);
}

void ref_stbi_free(unsigned char *p)
{
        stbi_image_free(p);
}

const char *ref_stbi_failure(void)
{
        const char *r = stbi_failure_reason();
        return r ? r : "";
}
}
