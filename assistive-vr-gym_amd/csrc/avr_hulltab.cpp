// avr_hulltab.cpp -- host builder of the support-mapping tables for large convex hulls.
//
// GJK/EPA query support(d) = the first hull vertex with the strictly largest projection on d
// (Bullet's btConvexHullShape::localGetSupportingVertexWithoutMargin scans every point; the CPU
// oracle does the same).  For the Jaco link hulls (296..1067 vertices) that full scan was the
// dominant cost of the collision phase.  This table makes the query exact and sub-linear:
//
//   * directions are bucketed by a cube map: face f = 2 * axis + (component < 0), then a G x G
//     grid over the other two components divided by the major one (the same convention as the
//     device lookup `tab_cell` in avr_kernel.hip);
//   * each cell lies inside a spherical cap (centre c, radius theta: the largest angle from c to
//     the cell's corners, plus a guard for float cell selection);
//   * a vertex v is listed for the cell unless, for some other vertex w, EVERY direction d of the
//     cap prefers w by more than the tolerance: max_{d in cap} d.(v - w) < -tol.  A vertex that
//     is a support point (or a float near-tie of one) for some d in the cap always passes, so the
//     list is a superset of the possible winners for every direction of the cell, kept in
//     ascending vertex order -- scanning it with the same strict ">" gives the same vertex as
//     scanning the whole hull.
//
// The pairwise test runs over a slab prefilter (c.v >= h(c) - 2 sin(theta/2) * 2R - tol, which
// every winner satisfies); testing against fewer w only keeps more candidates.  Built once per
// avr_create from the float vertices the device sees (the same bits), in double precision.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "../../include/avr.h"

namespace {

struct D3 { double x, y, z; };
inline D3 d3(double x, double y, double z) { return D3{x, y, z}; }
inline double ddot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline D3 dsub(D3 a, D3 b) { return d3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline D3 dnorm(D3 a) { const double l = std::sqrt(ddot(a, a)); return d3(a.x / l, a.y / l, a.z / l); }

// direction of face f at face coordinates (u, v) (see the header comment)
D3 face_dir(int f, double u, double v) {
    const int ax = f >> 1;
    const double s = (f & 1) ? -1.0 : 1.0;
    double c[3];
    const int o0 = ax == 0 ? 1 : 0, o1 = ax == 2 ? 1 : 2;
    c[ax] = s; c[o0] = u; c[o1] = v;
    return dnorm(d3(c[0], c[1], c[2]));
}

}  // namespace

extern "C" int32_t avr_hull_support_table(const float *verts, int32_t nv, int32_t G, int32_t *cell, int32_t *idx, int32_t cap) {
    if (!verts || nv <= 0 || G <= 0 || G > 64 || !cell) return -1;
    std::vector<D3> P((size_t)nv);
    D3 cen = d3(0, 0, 0);
    for (int i = 0; i < nv; i++) {
        P[i] = d3(verts[3 * i], verts[3 * i + 1], verts[3 * i + 2]);
        cen.x += P[i].x; cen.y += P[i].y; cen.z += P[i].z;
    }
    cen = d3(cen.x / nv, cen.y / nv, cen.z / nv);
    double R = 0.0;
    for (int i = 0; i < nv; i++) R = std::max(R, std::sqrt(ddot(dsub(P[i], cen), dsub(P[i], cen))));
    const double tol = 1e-6 * (1.0 + 2.0 * R);
    const double guard = 1e-4;            // rad: float cell selection near cell borders
    std::vector<int> slab, keep;
    int total = 0;
    for (int f = 0; f < 6; f++) {
        for (int i = 0; i < G; i++) {
            for (int j = 0; j < G; j++) {
                const double u0 = -1.0 + 2.0 * i / G, u1 = -1.0 + 2.0 * (i + 1) / G;
                const double v0 = -1.0 + 2.0 * j / G, v1 = -1.0 + 2.0 * (j + 1) / G;
                const D3 c = face_dir(f, 0.5 * (u0 + u1), 0.5 * (v0 + v1));
                double th = 0.0;
                const double uu[2] = {u0, u1}, vv[2] = {v0, v1};
                for (int a = 0; a < 2; a++)
                    for (int b = 0; b < 2; b++)
                        th = std::max(th, std::acos(std::min(1.0, std::max(-1.0, ddot(c, face_dir(f, uu[a], vv[b]))))));
                th += guard;
                double h = -1e300;
                for (int k = 0; k < nv; k++) h = std::max(h, ddot(c, P[k]));
                const double lim = h - 2.0 * std::sin(0.5 * th) * 2.0 * R - tol;
                slab.clear();
                for (int k = 0; k < nv; k++)
                    if (ddot(c, P[k]) >= lim) slab.push_back(k);
                keep.clear();
                for (int a : slab) {
                    bool ok = true;
                    for (int b : slab) {
                        if (a == b) continue;
                        const D3 uvec = dsub(P[a], P[b]);
                        const double nu = std::sqrt(ddot(uvec, uvec));
                        if (nu < 1e-15) continue;
                        const double ang = std::acos(std::min(1.0, std::max(-1.0, ddot(c, uvec) / nu)));
                        // max over the cap of d.(v - w)
                        const double best = nu * std::cos(std::max(0.0, ang - th));
                        if (best < -tol) { ok = false; break; }
                    }
                    if (ok) keep.push_back(a);
                }
                const int ci = (f * G + i) * G + j;
                cell[2 * ci] = total;
                cell[2 * ci + 1] = (int)keep.size();
                for (size_t q = 0; q < keep.size(); q++)
                    if (idx && total + (int)q < cap) idx[total + q] = keep[q];
                total += (int)keep.size();
            }
        }
    }
    return total;
}
