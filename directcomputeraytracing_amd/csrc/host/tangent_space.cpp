// tangent_space.cpp -- per-corner tangents exactly as MikkTSpace's genTangSpaceDefault
// computes them for a triangle list (/root/reference/MikkTSpace/mikktspace.c, called by
// Source/WavefrontOBJLoading.cpp:147-153,195). The tangent of every corner feeds the
// TBN frame of each BSDF evaluation and sample (Shaders/BSDFs.inc.hlsl:44-45,167-168,
// 303-304, HitShader.inc.hlsl:34-51) and the loader's vertex-dedup key
// (WavefrontOBJLoading.cpp:45-74,217), so it is parity-defining.
//
// Stages (triangles only: the OBJ path hands MikkTSpace triangulated faces,
// WavefrontOBJLoading.cpp:95-100, so the quad handling never runs):
//   1. weld corners with bit-identical (position, normal, uv) -- a 2048-cell grid on the
//      widest axis, then recursive midpoint splits (mikktspace.c:451-692);
//   2. flag degenerate triangles and move them behind the good ones (:278-302,1737-1818);
//   3. per-triangle texture-space derivatives and orientation (:944-1007);
//   4. edge adjacency from a sort of (min, max, triangle) keys (:1501-1594) -- the
//      reference's seeded quicksort is reproduced because its sub-sort passes leave the
//      last run unsorted, so the pairing order depends on it;
//   5. vertex groups grown over neighbours with the same orientation (:1069-1189);
//   6. one angle-weighted frame per group subset (:1198-1439);
//   7. degenerate corners copy a frame from a good corner of the same welded vertex
//      (:1820-1860).
// Floating-point order follows the reference expression by expression (single precision,
// no contraction; acos in double) so the result is bit-identical.
#include "scene.h"

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>

namespace dcrt {
namespace {

constexpr int kGridCells = 2048;
constexpr uint32_t kSortSeed = 39871946u;
constexpr uint32_t kTriDegenerate = 1u, kTriGroupWithAny = 4u, kTriOrientPreserving = 8u;

inline bool Same(const Float3& a, const Float3& b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
inline bool AboveMin(float v) { return std::fabs(v) > FLT_MIN; }
inline bool AboveMin(const Float3& v) { return AboveMin(v.x) || AboveMin(v.y) || AboveMin(v.z); }
inline float Len(const Float3& v) { return std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z); }
inline Float3 Unit(const Float3& v) { return v * (1.0f / Len(v)); }
inline Float3 UnitIfNonZero(const Float3& v) { return AboveMin(v) ? Unit(v) : v; }
inline Float3 Tangential(const Float3& v, const Float3& n) { return v - n * Dot(n, v); }

// x86 cvttss2si: out-of-range and NaN give INT_MIN (the reference casts with (int))
inline int TruncToInt(float f) { return (f >= -2147483648.0f && f < 2147483648.0f) ? (int)f : INT_MIN; }

__attribute__((noinline)) int GridCell(float lo, float hi, float v)
{
    const float f = (float)kGridCells * ((v - lo) / (hi - lo));
    const int i = TruncToInt(f);
    return i < kGridCells ? (i >= 0 ? i : 0) : kGridCells - 1;
}

// rotate the seed left by its low 5 bits and step it (one pivot draw)
inline uint32_t NextSeed(uint32_t s)
{
    const uint32_t r = s & 31u;
    const uint32_t rot = (s << r) | (s >> ((32u - r) & 31u));
    return s + rot + 3u;
}

struct EdgeKey { int lo, hi, tri; int Get(int ch) const { return ch == 0 ? lo : (ch == 1 ? hi : tri); } };

void SortEdges(std::vector<EdgeKey>& e, int left, int right, int ch, uint32_t seed)
{
    const int n = right - left + 1;
    if (n < 2) return;
    if (n == 2) {
        if (e[left].Get(ch) > e[right].Get(ch)) std::swap(e[left], e[right]);
        return;
    }
    seed = NextSeed(seed);
    const int pivot = e[left + (int)(seed % (uint32_t)n)].Get(ch);
    int l = left, r = right;
    do {
        while (e[l].Get(ch) < pivot) ++l;
        while (e[r].Get(ch) > pivot) --r;
        if (l <= r) { std::swap(e[l], e[r]); ++l; --r; }
    } while (l <= r);
    if (left < r) SortEdges(e, left, r, ch, seed);
    if (l < right) SortEdges(e, l, right, ch, seed);
}

struct Frame {
    Float3 os{ 1.0f, 0.0f, 0.0f };
    float magS = 1.0f;
    Float3 ot{ 0.0f, 1.0f, 0.0f };
    float magT = 1.0f;
    int uses = 0;
};

struct TriState {
    int neighbor[3] = { -1, -1, -1 };
    int group[3] = { -1, -1, -1 };
    Float3 os, ot;
    float magS = 0.0f, magT = 0.0f;
    int srcTri = 0;          // triangle of the input list (its frames live at 3 * srcTri)
    uint32_t flags = 0;
};

struct VertexGroup { int rep; bool orient; std::vector<int> tris; };

class MikkTangents {
public:
    MikkTangents(const Float3* pos, const Float3* nrm, const Float3* uvw, int triCount)
        : pos_(pos), nrm_(nrm), uvw_(uvw), n_(triCount) {}

    bool Run(std::vector<Float3>* out)
    {
        if (n_ <= 0) return false;
        corners_.resize((size_t)n_ * 3);
        tris_.assign(n_, TriState());
        for (int t = 0; t < n_; ++t) {
            tris_[t].srcTri = t;
            for (int k = 0; k < 3; ++k) corners_[t * 3 + k] = (t << 2) | k;
        }
        Weld();
        good_ = n_;
        for (int t = 0; t < n_; ++t) {
            const Float3 &a = P(corners_[t * 3]), &b = P(corners_[t * 3 + 1]), &c = P(corners_[t * 3 + 2]);
            if (Same(a, b) || Same(a, c) || Same(b, c)) { tris_[t].flags |= kTriDegenerate; --good_; }
        }
        MoveDegenerateLast();
        Derivatives();
        Adjacency();
        BuildGroups();
        frames_.assign((size_t)n_ * 3, Frame());
        EvaluateGroups();
        PatchDegenerate();
        out->resize((size_t)n_ * 3);
        for (int t = 0; t < n_; ++t)
            for (int k = 0; k < 3; ++k) (*out)[t * 3 + k] = frames_[t * 3 + k].os;
        return true;
    }

private:
    // corner code = triangle << 2 | corner (the code's value orders the adjacency sort)
    const Float3& P(int code) const { return pos_[(code >> 2) * 3 + (code & 3)]; }
    const Float3& N(int code) const { return nrm_[(code >> 2) * 3 + (code & 3)]; }
    const Float3& T(int code) const { return uvw_[(code >> 2) * 3 + (code & 3)]; }
    bool SameCorner(int a, int b) const { return Same(P(a), P(b)) && Same(N(a), N(b)) && Same(T(a), T(b)); }

    struct Probe { float p[3]; int slot; };

    void Weld()
    {
        const int m = (int)corners_.size();
        Float3 lo = P(0), hi = lo;
        for (int i = 1; i < m; ++i) {
            const Float3& p = P(corners_[i]);
            for (int a = 0; a < 3; ++a) {
                if (lo[a] > p[a]) lo[a] = p[a];
                else if (hi[a] < p[a]) hi[a] = p[a];
            }
        }
        const Float3 ext = hi - lo;
        int axis = 0;
        if (ext.y > ext.x && ext.y > ext.z) axis = 1;
        else if (ext.z > ext.x) axis = 2;
        std::vector<int> cell(m), start(kGridCells + 1, 0);
        for (int i = 0; i < m; ++i) {
            cell[i] = GridCell(lo[axis], hi[axis], P(corners_[i])[axis]);
            ++start[cell[i] + 1];
        }
        for (int c = 0; c < kGridCells; ++c) start[c + 1] += start[c];
        std::vector<int> bucket(m), fill(start.begin(), start.end() - 1);
        for (int i = 0; i < m; ++i) bucket[fill[cell[i]]++] = i;
        std::vector<Probe> probes;
        for (int c = 0; c < kGridCells; ++c) {
            const int count = start[c + 1] - start[c];
            if (count < 2) continue;
            probes.resize(count);
            for (int e = 0; e < count; ++e) {
                const int slot = bucket[start[c] + e];
                const Float3& p = P(corners_[slot]);
                probes[e] = { { p.x, p.y, p.z }, slot };
            }
            SplitWeld(probes, 0, count - 1);
        }
    }

    void SplitWeld(std::vector<Probe>& v, int left, int right)
    {
        float mn[3], mx[3];
        for (int a = 0; a < 3; ++a) mn[a] = mx[a] = v[left].p[a];
        for (int l = left + 1; l <= right; ++l)
            for (int a = 0; a < 3; ++a) {
                if (mn[a] > v[l].p[a]) mn[a] = v[l].p[a];
                if (mx[a] < v[l].p[a]) mx[a] = v[l].p[a];
            }
        const float dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
        int ch = 0;
        if (dy > dx && dy > dz) ch = 1;
        else if (dz > dx) ch = 2;
        const float sep = 0.5f * (mx[ch] + mn[ch]);
        if (!std::isfinite(sep)) return;
        if (sep >= mx[ch] || sep <= mn[ch]) {
            // a leaf: each corner takes the code of the first identical corner before it
            for (int l = left; l <= right; ++l) {
                const int slot = v[l].slot;
                for (int l2 = left; l2 < l; ++l2) {
                    const int slot2 = v[l2].slot;
                    if (SameCorner(corners_[slot], corners_[slot2])) { corners_[slot] = corners_[slot2]; break; }
                }
            }
            return;
        }
        int l = left, r = right;
        while (l < r) {
            bool leftReady = false, rightReady = false;
            while (!leftReady && l < r) {
                leftReady = !(v[l].p[ch] < sep);
                if (!leftReady) ++l;
            }
            while (!rightReady && l < r) {
                rightReady = v[r].p[ch] < sep;
                if (!rightReady) --r;
            }
            if (leftReady && rightReady) { std::swap(v[l], v[r]); ++l; --r; }
        }
        if (l == r) {
            if (v[r].p[ch] < sep) ++l;
            else --r;
        }
        if (left < r) SplitWeld(v, left, r);
        if (l < right) SplitWeld(v, l, right);
    }

    void SwapTris(int a, int b)
    {
        for (int k = 0; k < 3; ++k) std::swap(corners_[a * 3 + k], corners_[b * 3 + k]);
        std::swap(tris_[a], tris_[b]);
    }

    // good triangles keep their order at the front; each degenerate one swaps with the
    // next good triangle found after it
    void MoveDegenerateLast()
    {
        int nextGood = 1;
        for (int t = 0; t < good_; ++t) {
            if (!(tris_[t].flags & kTriDegenerate)) {
                nextGood = std::max(nextGood, t + 2);
                continue;
            }
            while (nextGood < n_ && (tris_[nextGood].flags & kTriDegenerate)) ++nextGood;
            if (nextGood >= n_) break;
            SwapTris(t, nextGood);
            ++nextGood;
        }
    }

    void Derivatives()
    {
        for (int f = 0; f < good_; ++f) {
            TriState& s = tris_[f];
            s.flags |= kTriGroupWithAny;
            const int c0 = corners_[f * 3], c1 = corners_[f * 3 + 1], c2 = corners_[f * 3 + 2];
            const Float3 d1 = P(c1) - P(c0), d2 = P(c2) - P(c0);
            const float t21x = T(c1).x - T(c0).x, t21y = T(c1).y - T(c0).y;
            const float t31x = T(c2).x - T(c0).x, t31y = T(c2).y - T(c0).y;
            const float area2 = t21x * t31y - t21y * t31x;
            const Float3 os = d1 * t31y - d2 * t21y;
            const Float3 ot = d1 * -t31x + d2 * t21x;
            if (area2 > 0) s.flags |= kTriOrientPreserving;
            if (!AboveMin(area2)) continue;
            const float absArea = std::fabs(area2);
            const float lenS = Len(os), lenT = Len(ot);
            const float sign = (s.flags & kTriOrientPreserving) ? 1.0f : -1.0f;
            if (AboveMin(lenS)) s.os = os * (sign / lenS);
            if (AboveMin(lenT)) s.ot = ot * (sign / lenT);
            s.magS = lenS / absArea;
            s.magT = lenT / absArea;
            if (AboveMin(s.magS) && AboveMin(s.magT)) s.flags &= ~kTriGroupWithAny;
        }
    }

    // edge number and (first, second) order of the edge {a, b} inside triangle t
    void EdgeOf(int t, int a, int b, int* first, int* second, int* edge) const
    {
        const int* c = &corners_[t * 3];
        if (c[0] == a || c[0] == b) {
            if (c[1] == a || c[1] == b) { *edge = 0; *first = c[0]; *second = c[1]; }
            else { *edge = 2; *first = c[2]; *second = c[0]; }
        } else {
            *edge = 1; *first = c[1]; *second = c[2];
        }
    }

    void Adjacency()
    {
        const int m = good_ * 3;
        std::vector<EdgeKey> e(m);
        for (int f = 0; f < good_; ++f)
            for (int i = 0; i < 3; ++i) {
                const int a = corners_[f * 3 + i], b = corners_[f * 3 + (i < 2 ? i + 1 : 0)];
                e[f * 3 + i] = { a < b ? a : b, !(a < b) ? a : b, f };
            }
        SortEdges(e, 0, m - 1, 0, kSortSeed);
        // sub-sorts of equal-key runs; a run is sorted when the next one starts, so the
        // last run of each pass stays in the order the previous pass left
        for (int pass = 1; pass <= 2; ++pass) {
            int runStart = 0;
            for (int i = 1; i < m; ++i) {
                const bool sameRun = pass == 1 ? e[runStart].lo == e[i].lo
                                               : (e[runStart].lo == e[i].lo && e[runStart].hi == e[i].hi);
                if (!sameRun) {
                    SortEdges(e, runStart, i - 1, pass, kSortSeed);
                    runStart = i;
                }
            }
        }
        for (int i = 0; i < m; ++i) {
            const int a = e[i].lo, b = e[i].hi, f = e[i].tri;
            int a0, a1, edgeA;
            EdgeOf(f, a, b, &a0, &a1, &edgeA);
            if (tris_[f].neighbor[edgeA] != -1) continue;
            for (int j = i + 1; j < m && e[j].lo == a && e[j].hi == b; ++j) {
                const int t = e[j].tri;
                int b0, b1, edgeB;
                EdgeOf(t, e[j].lo, e[j].hi, &b1, &b0, &edgeB);   // the neighbour runs the edge backwards
                if (a0 == b0 && a1 == b1 && tris_[t].neighbor[edgeB] == -1) {
                    tris_[f].neighbor[edgeA] = t;
                    tris_[t].neighbor[edgeB] = f;
                    break;
                }
            }
        }
    }

    int CornerOfRep(int t, int rep) const
    {
        const int* c = &corners_[t * 3];
        return c[0] == rep ? 0 : (c[1] == rep ? 1 : (c[2] == rep ? 2 : -1));
    }

    bool Grow(int t, int g)
    {
        VertexGroup& grp = groups_[g];
        TriState& s = tris_[t];
        const int i = CornerOfRep(t, grp.rep);
        if (s.group[i] == g) return true;
        if (s.group[i] != -1) return false;
        if ((s.flags & kTriGroupWithAny) && s.group[0] == -1 && s.group[1] == -1 && s.group[2] == -1) {
            // the first group to reach a group-with-anything triangle sets its orientation
            s.flags = (s.flags & ~kTriOrientPreserving) | (grp.orient ? kTriOrientPreserving : 0u);
        }
        if (((s.flags & kTriOrientPreserving) != 0) != grp.orient) return false;
        grp.tris.push_back(t);
        s.group[i] = g;
        const int left = s.neighbor[i], right = s.neighbor[i > 0 ? i - 1 : 2];
        if (left >= 0) Grow(left, g);
        if (right >= 0) Grow(right, g);
        return true;
    }

    void BuildGroups()
    {
        for (int f = 0; f < good_; ++f)
            for (int i = 0; i < 3; ++i) {
                TriState& s = tris_[f];
                if ((s.flags & kTriGroupWithAny) || s.group[i] != -1) continue;
                const int g = (int)groups_.size();
                groups_.push_back({ corners_[f * 3 + i], (s.flags & kTriOrientPreserving) != 0, {} });
                s.group[i] = g;
                groups_[g].tris.push_back(f);
                const int left = s.neighbor[i], right = s.neighbor[i > 0 ? i - 1 : 2];
                if (left >= 0) Grow(left, g);
                if (right >= 0) Grow(right, g);
            }
    }

    // os / ot of triangle t projected into the tangent plane of normal n
    void Projected(int t, const Float3& n, Float3* os, Float3* ot) const
    {
        *os = UnitIfNonZero(Tangential(tris_[t].os, n));
        *ot = UnitIfNonZero(Tangential(tris_[t].ot, n));
    }

    Frame AngleWeighted(const std::vector<int>& members, int rep) const
    {
        Frame r;
        r.os = Float3(0.0f, 0.0f, 0.0f);
        r.ot = Float3(0.0f, 0.0f, 0.0f);
        r.magS = 0.0f;
        r.magT = 0.0f;
        float angleSum = 0.0f;
        for (int f : members) {
            if (tris_[f].flags & kTriGroupWithAny) continue;
            const int i = CornerOfRep(f, rep);
            const int code = corners_[f * 3 + i];
            const Float3& n = N(code);
            Float3 os, ot;
            Projected(f, n, &os, &ot);
            const int prev = corners_[f * 3 + (i > 0 ? i - 1 : 2)], next = corners_[f * 3 + (i < 2 ? i + 1 : 0)];
            const Float3 e1 = UnitIfNonZero(Tangential(P(prev) - P(code), n));
            const Float3 e2 = UnitIfNonZero(Tangential(P(next) - P(code), n));
            float c = Dot(e1, e2);
            c = c > 1 ? 1 : (c < (-1) ? (-1) : c);
            const float angle = (float)std::acos((double)c);
            r.os = r.os + os * angle;
            r.ot = r.ot + ot * angle;
            r.magS += angle * tris_[f].magS;
            r.magT += angle * tris_[f].magT;
            angleSum += angle;
        }
        r.os = UnitIfNonZero(r.os);
        r.ot = UnitIfNonZero(r.ot);
        if (angleSum > 0) {
            r.magS /= angleSum;
            r.magT /= angleSum;
        }
        return r;
    }

    static Frame Average(const Frame& a, const Frame& b)
    {
        Frame r;
        if (a.magS == b.magS && a.magT == b.magT && Same(a.os, b.os) && Same(a.ot, b.ot)) {
            r.magS = a.magS; r.magT = a.magT; r.os = a.os; r.ot = a.ot;
        } else {
            r.magS = 0.5f * (a.magS + b.magS);
            r.magT = 0.5f * (a.magT + b.magT);
            r.os = UnitIfNonZero(a.os + b.os);
            r.ot = UnitIfNonZero(a.ot + b.ot);
        }
        return r;
    }

    void EvaluateGroups()
    {
        // the default 180 degree threshold: (float)cos(pi) as the reference computes it
        const float thresCos = (float)std::cos((double)((180.0f * (float)3.1415926535897932384626433832795) / 180.0f));
        std::vector<std::vector<int>> subsets;
        std::vector<Frame> subsetFrames;
        std::vector<int> members;
        for (int g = 0; g < (int)groups_.size(); ++g) {
            const VertexGroup& grp = groups_[g];
            subsets.clear();
            subsetFrames.clear();
            for (int f : grp.tris) {
                const TriState& s = tris_[f];
                const int index = s.group[0] == g ? 0 : (s.group[1] == g ? 1 : 2);
                const Float3& n = N(corners_[f * 3 + index]);
                Float3 os, ot;
                Projected(f, n, &os, &ot);
                members.clear();
                for (int t : grp.tris) {
                    Float3 os2, ot2;
                    Projected(t, n, &os2, &ot2);
                    const bool any = ((s.flags | tris_[t].flags) & kTriGroupWithAny) != 0;
                    const bool sameFace = s.srcTri == tris_[t].srcTri;
                    const float cosS = Dot(os, os2), cosT = Dot(ot, ot2);
                    if (any || sameFace || (cosS > thresCos && cosT > thresCos)) members.push_back(t);
                }
                std::sort(members.begin(), members.end());   // distinct triangle numbers
                size_t l = 0;
                while (l < subsets.size() && subsets[l] != members) ++l;
                if (l == subsets.size()) {
                    subsets.push_back(members);
                    subsetFrames.push_back(AngleWeighted(members, grp.rep));
                }
                Frame& out = frames_[(size_t)s.srcTri * 3 + index];
                if (out.uses == 1) { out = Average(out, subsetFrames[l]); out.uses = 2; }
                else { out = subsetFrames[l]; out.uses = 1; }
            }
        }
    }

    void PatchDegenerate()
    {
        for (int t = good_; t < n_; ++t)
            for (int i = 0; i < 3; ++i) {
                const int code = corners_[t * 3 + i];
                for (int j = 0; j < good_ * 3; ++j)
                    if (corners_[j] == code) {
                        frames_[(size_t)tris_[t].srcTri * 3 + i] = frames_[(size_t)tris_[j / 3].srcTri * 3 + j % 3];
                        break;
                    }
            }
    }

    const Float3 *pos_, *nrm_, *uvw_;
    int n_, good_ = 0;
    std::vector<int> corners_;
    std::vector<TriState> tris_;
    std::vector<VertexGroup> groups_;
    std::vector<Frame> frames_;
};

}  // namespace

bool GenerateMikkTangents(const std::vector<Float3>& positions, const std::vector<Float3>& normals,
                          const std::vector<Float3>& texcoords, std::vector<Float3>* out)
{
    const size_t corners = positions.size();
    if (corners % 3 != 0 || normals.size() != corners || texcoords.size() != corners || corners / 3 > (size_t)(INT_MAX >> 2))
        return false;
    MikkTangents m(positions.data(), normals.data(), texcoords.data(), (int)(corners / 3));
    return m.Run(out);
}

}  // namespace dcrt
