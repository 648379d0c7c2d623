// A reference-side caller of the two legacy primitives, built and linked
// against libvrt.so alone by tests/test_prims.py.
//
// The declarations are the reference's (VRT/raytri.h:5-7, VRT/tribox2.h:6):
// C++ linkage, no extern "C" -- exactly what VRT/voxel_octree.cc:446,490
// import.  If libvrt.so did not define the mangled names this would not link.
//
// stdin : u32 n_mt, n_mt x 15 f64 (orig, dir, v0, v1, v2),
//         u32 n_sat, n_sat x 15 f32 (centre, half size, 3 vertices)
// stdout: n_mt x 4 f64 (ret, t, u, v; zeros after a miss), n_sat x i32
#include <cstdint>
#include <cstdio>
#include <vector>

int intersect_triangle3(double orig[3], double dir[3], double vert0[3],
                        double vert1[3], double vert2[3], double* t, double* u,
                        double* v);
int triBoxOverlap(float boxcenter[3], float boxhalfsize[3], float triverts[3][3]);

int main()
{
        uint32_t n = 0;
        if (fread(&n, 4, 1, stdin) != 1)
                return 2;
        std::vector<double> q(size_t(n) * 15);
        if (fread(q.data(), 8, q.size(), stdin) != q.size())
                return 2;
        std::vector<double> out(size_t(n) * 4, 0.0);
        for (uint32_t i = 0; i < n; ++i) {
                double *p = &q[size_t(i) * 15], t, u, v;
                const int r = intersect_triangle3(p, p + 3, p + 6, p + 9, p + 12, &t, &u, &v);
                double *o = &out[size_t(i) * 4];
                o[0] = r;
                if (r == 1) {
                        o[1] = t;
                        o[2] = u;
                        o[3] = v;
                }
        }
        uint32_t m = 0;
        if (fread(&m, 4, 1, stdin) != 1)
                return 2;
        std::vector<float> b(size_t(m) * 15);
        if (fread(b.data(), 4, b.size(), stdin) != b.size())
                return 2;
        std::vector<int32_t> sat(m);
        for (uint32_t i = 0; i < m; ++i) {
                float *p = &b[size_t(i) * 15];
                float tv[3][3] = { { p[6], p[7], p[8] }, { p[9], p[10], p[11] }, { p[12], p[13], p[14] } };
                sat[i] = triBoxOverlap(p, p + 3, tv);
        }
        fwrite(out.data(), 8, out.size(), stdout);
        fwrite(sat.data(), 4, sat.size(), stdout);
        return 0;
}
